"""Slot chunks (nrx_api.cpp chunk_slots): an f16 forward whose workspace would reach the GZ
loader's 32-bit range (1 GB) runs as consecutive sub-forwards in one chunk-sized workspace.
Slots are independent (neural_rx.py:544-595 has no cross-slot term), so the chunked forward of
26 slots at 273 PRB (41 MB of workspace per slot: 1.07 GB unchunked) must equal, bit for bit,
two forwards of 13 slots each (535 MB, no chunking)."""
import numpy as np
import pytest

from tests.helpers import make_case, run_engine

pytestmark = pytest.mark.gpu


def _sub(case, lo, hi):
    import dataclasses
    c = dataclasses.replace(case, y=case.y[lo:hi], h_hat=case.h_hat[lo:hi], active=case.active[lo:hi],
                            mcs_mask=None if case.mcs_mask is None else case.mcs_mask[lo:hi])
    return c


def test_chunked_forward_equals_split_batches():
    from neural_rx_amd.receiver import CGNNEngine
    case = make_case("nrx_rt", batch=26, users=2, prbs=273, random_inputs=True, seed=61)
    eng = CGNNEngine(case.spec, case.weights)
    try:
        ws = eng.workspace_bytes(26, 2, 3276)
        assert ws < (1 << 30) and ws < 26 * 4 * 2 * 3276 * 14 * 56 * 2   # a chunk's workspace, not 26 slots'
        full = run_engine(case, "f16", eng)
        lo = run_engine(_sub(case, 0, 13), "f16", eng)
        hi = run_engine(_sub(case, 13, 26), "f16", eng)
    finally:
        eng.close()
    assert np.array_equal(full["llr_raw"], np.concatenate([lo["llr_raw"], hi["llr_raw"]], axis=1))
    assert np.array_equal(full["h_hat"], np.concatenate([lo["h_hat"], hi["h_hat"]], axis=0))


def test_chunked_forward_eight_users_combine_pass():
    # U = 8 (the combine pass between stages, RR aggregation updates): 8 slots at 273 PRB need
    # 1.3 GB unchunked and run as chunks; the result must equal forwards of 4 + 4 slots (random
    # activity, so the combine's 1/(n-1) differs per slot and chunk boundaries would show)
    from neural_rx_amd.receiver import CGNNEngine
    rng = np.random.default_rng(62)
    case = make_case("nrx_rt", batch=8, users=8, prbs=273, random_inputs=True, seed=62,
                     active=rng.integers(0, 2, size=(8, 8)).astype(np.float32))
    eng = CGNNEngine(case.spec, case.weights)
    try:
        assert eng.workspace_bytes(8, 8, 3276) < (1 << 30)
        full = run_engine(case, "f16", eng)
        lo = run_engine(_sub(case, 0, 4), "f16", eng)
        hi = run_engine(_sub(case, 4, 8), "f16", eng)
    finally:
        eng.close()
    assert np.array_equal(full["llr_raw"], np.concatenate([lo["llr_raw"], hi["llr_raw"]], axis=1))
    assert np.array_equal(full["h_hat"], np.concatenate([lo["h_hat"], hi["h_hat"]], axis=0))


def test_chunked_forward_multi_head():
    # Var-IO (two LLR heads: the LLR tensor keeps its head stride llr_B across chunks):
    # 26 slots at 273 PRB run as chunks and must equal forwards of 13 + 13 slots for every head
    from neural_rx_amd.receiver import CGNNEngine
    rng = np.random.default_rng(63)
    case = make_case("nrx_rt_var_mcs", batch=26, users=2, prbs=273, random_inputs=True, seed=63,
                     mcs_choice=rng.integers(0, 2, size=(26, 2)))
    eng = CGNNEngine(case.spec, case.weights)
    try:
        assert eng.workspace_bytes(26, 2, 3276) < (1 << 30)
        full = run_engine(case, "f16", eng)
        lo = run_engine(_sub(case, 0, 13), "f16", eng)
        hi = run_engine(_sub(case, 13, 26), "f16", eng)
    finally:
        eng.close()
    assert full["llr_raw"].shape[0] == 2
    assert np.array_equal(full["llr_raw"], np.concatenate([lo["llr_raw"], hi["llr_raw"]], axis=1))
    assert np.array_equal(full["h_hat"], np.concatenate([lo["h_hat"], hi["h_hat"]], axis=0))
