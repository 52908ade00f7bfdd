"""The one-launch forward (k_forward) against the three-launch forward (needs an MI355X).

k_forward runs the same per-item code as k_init / k_update, only scheduled through per-XCD
work queues with cross-workgroup dependency counters, so its outputs
must equal the three-launch path bit for bit (NRX_FUSED=0 selects that path at every
forward).  The oracle comparison of the same launch shape is tests/test_gpu_baseline_shapes.py
(cfg2, B = 128, which takes k_forward by default).  Covered here: the bench shape, inactive
users, U = 1, num_it = 1 (StateInit straight into the readout stage), repeated forwards (the
counters are reset by the last workgroup of each launch), a hipGraph replay, and the sticky
timeout word staying 0.
"""
import os

import numpy as np
import pytest

from tests.helpers import make_case, run_engine
from tests.test_gpu_parity import engine_for

pytestmark = pytest.mark.gpu


def _run(case, fused: bool):
    old = os.environ.get("NRX_FUSED")
    os.environ["NRX_FUSED"] = "1" if fused else "0"
    try:
        return run_engine(case, "f16", engine_for(case))
    finally:
        if old is None:
            del os.environ["NRX_FUSED"]
        else:
            os.environ["NRX_FUSED"] = old


def _took_fused(case) -> bool:
    """True when the profiler saw the one-launch kernel for this case."""
    eng = engine_for(case)
    eng.profile(True)
    _run(case, True)
    prof = eng.profile_read()
    eng.profile(False)
    return prof["forward"][0] == 1 and prof["state_update"][0] == 0


def _check_identical(case):
    assert _took_fused(case), "the case was expected to take k_forward"
    ref = _run(case, False)
    for rep in range(3):          # repeated launches: the counters reset themselves
        got = _run(case, True)
        assert np.array_equal(ref["llr_raw"], got["llr_raw"]), f"LLRs differ (repeat {rep})"
        assert np.array_equal(ref["h_hat"], got["h_hat"]), f"h_hat differs (repeat {rep})"
    assert engine_for(case).fused_status(reset=True) == 0


def test_fused_bench_shape_identical():
    _check_identical(make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=31))


def test_fused_random_activity_identical():
    rng = np.random.default_rng(32)
    active = (rng.random((128, 2)) < 0.6).astype(np.float32)
    _check_identical(make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=32, active=active))


def test_fused_one_user_identical():
    _check_identical(make_case("nrx_rt", batch=256, users=1, prbs=4, snr_db=12, seed=33))


def test_fused_num_it_1_identical():
    case = make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=34)
    case.num_it = 1
    _check_identical(case)


def test_fused_odd_batch_identical():
    # B not a multiple of the 8 queues: queues hold 17 or 16 slots
    _check_identical(make_case("nrx_rt", batch=131, users=2, prbs=4, snr_db=12, seed=35))


def test_fused_graph_replay():
    import torch
    case = make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=36)
    ref = _run(case, False)
    eng = engine_for(case)
    dev = "cuda:0"
    t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)  # noqa: E731
    args = (t(case.y), t(case.pe), t(case.h_hat), t(case.active), t(case.mcs_mask))
    os.environ["NRX_FUSED"] = "1"
    try:
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            eng.forward(*args, num_it=None, precision="f16")    # warm-up (workspace allocation)
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            llr, h = eng.forward(*args, num_it=None, precision="f16")
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
    finally:
        del os.environ["NRX_FUSED"]
    assert np.array_equal(ref["llr_raw"], llr.cpu().numpy())
    assert eng.fused_status(reset=True) == 0

