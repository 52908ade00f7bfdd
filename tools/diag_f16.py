"""Diagnostic: where do f16-mode hard-decision flips sit (|LLR_ref| bins), and BER vs truth."""
import numpy as np
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.helpers import make_case, run_engine, run_oracle, compare
from neural_rx_amd import synth

for name, kw in [("nrx_rt", dict(batch=8, users=2, prbs=4, snr_db=15)),
                 ("nrx_rt", dict(batch=8, users=2, prbs=4, snr_db=8)),
                 ("nrx_large_64qam", dict(batch=1, users=8, prbs=1, snr_db=25))]:
    case = make_case(name, **kw)
    ref = run_oracle(case)
    got = run_engine(case, "f16")
    r, g = ref["llr"][0], got["llr"][0]
    flip = np.sign(r) != np.sign(g)
    print(name, kw, compare(ref, got))
    for th in [0.1, 0.5, 1, 2, 4]:
        print(f"  flips with |ref|>{th}: {flip[np.abs(r)>th].mean():.2e}")
    print("  max |ref| among flips", np.abs(r[flip]).max() if flip.any() else 0)
    if case.slots is not None:
        nb = case.spec.bits[0]
        print("  BER oracle", [synth.uncoded_ber(r, case.slots, u, nb) for u in range(case.active.shape[1])],
              " f16", [synth.uncoded_ber(g, case.slots, u, nb) for u in range(case.active.shape[1])])
