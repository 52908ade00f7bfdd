"""The register-resident kernels (nrx_rr.inc, opt-in with NRX_RR) on the GPU.

They are a second schedule of the same math: every launch they replace must produce the
strip kernels' outputs bit for bit (same depthwise order, same f16 roundings, same HBM state
layout), and the whole forward stays within the oracle tolerances.  NRX_RR is read at every
forward, so one engine runs both paths.  Cases: the bench shape (aggregation-tail and readout
RR launches, StateInit RR), inactive users, U = 1, a partial last strip, 8 antennas
(StateInit A2P = 16) and the 64-QAM masking model (8 iterations, one 6-bit head)."""
import os

import numpy as np
import pytest

from tests.helpers import compare, make_case, run_engine, run_oracle
from tests.test_gpu_parity import F16_FLIP_TOL, F16_REL_TOL, F16_RMS_TOL, engine_for

pytestmark = pytest.mark.gpu

CASES = {
    "bench_b128_u2": dict(batch=128, users=2, prbs=4),
    "random_active_b128": dict(batch=128, users=2, prbs=4, active="random"),
    "u1_b512": dict(batch=512, users=1, prbs=4),
    "f60_partial_strip": dict(batch=128, users=2, prbs=5),
    "ant8_b128": dict(batch=128, users=2, prbs=4, num_rx_ant=8, seeded_weights=True, random_inputs=True),
    "masking_64qam_b128": dict(config="nrx_large_var_mcs_64qam_masking", batch=128, users=2, prbs=4, snr_db=22),
}


def _forward(eng, case, mask):
    import torch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()  # noqa: E731
    multi = case.spec.num_mcs > 1
    os.environ["NRX_RR"] = str(mask)
    try:
        llr, h = eng.forward(t(case.y), t(case.pe), t(case.h_hat), t(case.active),
                             t(case.mcs_mask) if multi else None, None, "f16")
        torch.cuda.synchronize()
    finally:
        os.environ.pop("NRX_RR", None)
    return llr.cpu().numpy(), h.cpu().numpy()


@pytest.mark.parametrize("name", list(CASES))
def test_rr_bit_identical_to_strip_kernels(name):
    kw = dict(CASES[name])
    if kw.get("active") == "random":
        rng = np.random.default_rng(7)
        kw["active"] = (rng.random((kw["batch"], kw["users"])) < 0.6).astype(np.float32)
    kw.setdefault("snr_db", 12)
    case = make_case(kw.pop("config", "nrx_rt"), seed=13, **kw)
    eng = engine_for(case)
    l0, h0 = _forward(eng, case, 0)
    l7, h7 = _forward(eng, case, 7)
    assert np.isfinite(l7).all()
    assert np.array_equal(l0, l7) and np.array_equal(h0, h7)


def test_rr_bench_shape_vs_oracle():
    case = make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=22)
    os.environ["NRX_RR"] = "7"
    try:
        got = run_engine(case, "f16", engine_for(case))
    finally:
        os.environ.pop("NRX_RR", None)
    c = compare(run_oracle(case), got)
    assert c["llr_rel"] <= F16_REL_TOL and c["llr_rms_rel"] <= F16_RMS_TOL and c["flip_rate"] <= F16_FLIP_TOL, c
