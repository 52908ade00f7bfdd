"""Diagnostic (round 4): fused vs three-launch for U > 4, and the f32x path at cfg3 batch 2."""
import sys, os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.helpers import make_case, run_engine, run_oracle, compare
from tests.test_gpu_parity import engine_for


def run(case, fused, prec="f16"):
    eng = engine_for(case)
    eng.fused_config(enable=fused)
    try:
        return run_engine(case, prec, eng)
    finally:
        eng.fused_config(enable=True)


for cfgname, U, B, it in (("nrx_large_64qam", 8, 32, 1), ("nrx_large_64qam", 8, 32, None)):
    case = make_case(cfgname, batch=B, users=U, prbs=4, snr_db=20, seed=42)
    case.num_it = it
    a, b = run(case, False), run(case, True)
    d = np.abs(a["llr_raw"] - b["llr_raw"])
    print(cfgname, "U", U, "B", B, "num_it", it, "llr maxdiff", d.max(), "frac", (d > 0).mean(), flush=True)
case = make_case("nrx_large", batch=2, users=4, prbs=132, num_rx_ant=16, seeded_weights=True, random_inputs=True, seed=26)
ref = run_oracle(case)
for step in ("f32x first", "f16 three", "f32x after three", "f16 fused", "f32x after fused"):
    prec = "f32x" if step.startswith("f32x") else "f16"
    got = run(case, "fused" in step, prec)
    c = compare(ref, got)
    print("cfg3 B2", step, {k: round(v, 6) for k, v in c.items()}, flush=True)
    if step == "f16 three":
        three = got
    if step == "f16 fused":
        print("  fused vs three llr maxdiff", np.abs(three["llr_raw"] - got["llr_raw"]).max(), flush=True)
