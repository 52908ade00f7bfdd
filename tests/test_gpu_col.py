"""Whole-column launches (k_init_col, k_update_col; nrx_col.inc).

Every MFMA of the column kernels sees the operands of the strip kernels' in the same order, so the
three-launch f16 forward must give the same LLRs and h_ref bit for bit whichever kernel runs a
stage: each case runs the forward with schedule mask 0 (strip k_init / k_update everywhere) and
with the column bits (16 StateInit, 4 aggregation updates, 8 readout update), checks from the
per-launch profile which kernel ran each stage, compares exactly, and the column result against
the fp64 oracle within the f16 gate of tests/test_gpu_parity.py."""
import numpy as np
import pytest

from tests.helpers import compare, make_case, run_engine, run_oracle

pytestmark = pytest.mark.gpu

COL = 4 | 8 | 16
WIDE = COL | 64      # column updates on grids wider than 48 subcarriers too (off by default)
_ENGINES = {}


def _engine(case):
    from neural_rx_amd.receiver import CGNNEngine
    key = (case.spec, case.weights[0].tobytes()[:64], len(case.weights))
    if key not in _ENGINES:
        _ENGINES.clear()
        _ENGINES[key] = CGNNEngine(case.spec, case.weights)
    return _ENGINES[key]


def _run(case, mask):
    eng = _engine(case)
    eng.fused_config(enable=False)      # the three-launch forward (whose stages these are)
    eng.update_schedule(mask)
    try:
        eng.profile(True)
        out = run_engine(case, "f16", eng)
        prof = eng.profile_read()
        eng.profile(False)
    finally:
        eng.fused_config(enable=True)
    return out, prof


def _check(case, oracle=True, init_col=True, mask=COL):
    n_it = case.num_it or case.spec.num_it
    ref, pr = _run(case, 0)
    got, pg = _run(case, mask)
    assert pr["state_update_col"][0] == 0 and pr["state_init_col"][0] == 0 and pr["state_update"][0] == n_it
    n_col = (n_it - 1 if mask & 4 else 0) + (1 if mask & 8 else 0)
    assert pg["state_update_col"][0] == n_col, pg
    assert pg["state_init_col"][0] == (1 if init_col and mask & 16 else 0), pg
    assert np.array_equal(ref["llr_raw"], got["llr_raw"]), np.abs(ref["llr_raw"] - got["llr_raw"]).max()
    assert np.array_equal(ref["h_hat"], got["h_hat"])
    if oracle:
        c = compare(run_oracle(case), got)
        assert c["llr_rel"] < 0.10 and c["llr_rms_rel"] < 0.02 and c["flip_rate_confident"] <= 1e-3, c


def test_col_bench_shape():
    # BASELINE configs[1]: nrx_rt, 2 UE, 4 PRB (F = 48: one item per (slot, user), no halo), B = 128
    _check(make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=71))


@pytest.mark.parametrize("mask", [16, 4, 8])
def test_col_stage_masks(mask):
    # each column stage alone beside the strip kernels of the others
    _check(make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=72), oracle=False, mask=mask)


def test_col_u1_two_strips_random_activity():
    # U = 1 (no other user), F = 60 > 48: two strips of 44 outputs with a 2-row halo, the second
    # strip's rows 16..47 past the grid; inactive slots
    case = make_case("nrx_rt", batch=96, users=1, prbs=5, snr_db=10, seed=73,
                     active=np.random.default_rng(73).integers(0, 2, size=(96, 1)).astype(np.float32))
    _check(case, mask=WIDE)


def test_col_u2_inactive_user():
    case = make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=14, seed=74,
                     active=np.random.default_rng(74).integers(0, 2, size=(128, 2)).astype(np.float32))
    _check(case)


def test_col_one_prb_rows_past_the_grid():
    # F = 12 < 48: one item per (slot, user) whose positions 12..47 lie past the grid (zero rows)
    _check(make_case("nrx_rt", batch=640, users=1, prbs=1, snr_db=12, seed=75))


def test_col_several_items_per_workgroup():
    # F = 96: three strips, 768 items on 256 CUs -- the readout launch restages its conv1 / conv2
    # images after every item (the heads sit over them), the StateInit / aggregation launches loop
    case = make_case("nrx_rt", batch=128, users=2, prbs=8, snr_db=12, seed=76)
    _check(case, mask=WIDE)


def test_col_large_grid_norm_pass():
    # 273 PRB (F = 3276 > kNormFusedMaxQ float4s per slot): the slot norm comes from the k_norm
    # pass; 75 strips, more items than CUs
    case = make_case("nrx_rt", batch=2, users=2, prbs=273, snr_db=12, seed=77)
    _check(case, oracle=False, mask=WIDE)


def test_col_16_antennas_8_iterations():
    # 2A = 32 (ChEst head CHP = 32): StateInit stays on the strip kernel (A2P = 32), every update
    # stage runs the column launch; nrx_large topology (8 iterations), seeded weights, 132 PRB
    case = make_case("nrx_large", batch=4, users=2, prbs=132, num_rx_ant=16, seeded_weights=True,
                     random_inputs=True, seed=78)
    _check(case, oracle=False, init_col=False, mask=WIDE)


def test_col_wide_grid_default_keeps_rr():
    # by default a grid wider than one column runs the column StateInit and the RR aggregation /
    # strip readout updates (measured faster there: DESIGN.md section 5)
    case = make_case("nrx_rt", batch=64, users=2, prbs=8, snr_db=12, seed=70)
    ref, _ = _run(case, 0)
    got, pg = _run(case, 29)
    assert pg["state_update_col"][0] == 0 and pg["state_update_rr"][0] == 1 and pg["state_init_col"][0] == 1, pg
    assert np.array_equal(ref["llr_raw"], got["llr_raw"])


def test_col_var_io():
    # Var-IO (two StateInits: two column StateInit launches, the second accumulating; the profiler
    # times the stage as one event pair), one-hot MCS mask; the aggregation update runs the column
    # launch, the readout (two LLR heads) the strip kernel
    rng = np.random.default_rng(79)
    case = make_case("nrx_rt_var_mcs", batch=128, users=2, prbs=4, snr_db=14, seed=79,
                     mcs_choice=rng.integers(0, 2, size=(128, 2)))
    n_it = case.spec.num_it
    ref, _ = _run(case, 0)
    got, pg = _run(case, COL)
    assert pg["state_init_col"][0] == 1 and pg["state_init"][0] == 0, pg
    assert pg["state_update_col"][0] == n_it - 1, pg
    assert np.array_equal(ref["llr_raw"], got["llr_raw"])
    assert np.array_equal(ref["h_hat"], got["h_hat"])
    c = compare(run_oracle(case), got)
    assert c["llr_rel"] < 0.10 and c["llr_rms_rel"] < 0.02 and c["flip_rate_confident"] <= 1e-3, c


def test_col_var_io_one_mcs_everywhere():
    # every (slot, user) on MCS 1: StateInit 0's launch has weight 0 everywhere (its items' output
    # enters as 0 * finite), StateInit 1's launch adds the whole state
    # (B = 128, 4 PRB: more items than the small-strip latency tiers take)
    case = make_case("nrx_rt_var_mcs", batch=128, users=2, prbs=4, snr_db=14, seed=81,
                     mcs_choice=np.ones((128, 2), np.int64))
    ref, _ = _run(case, 0)
    got, pg = _run(case, COL)
    assert pg["state_init_col"][0] == 1, pg
    assert np.array_equal(ref["llr_raw"], got["llr_raw"])
    assert np.array_equal(ref["h_hat"], got["h_hat"])


@pytest.mark.parametrize("users", [3, 8])
def test_col_users_combine_pass(users):
    # U = 3 / 8: conv1 of every column update item reads the a_u planes k_combine wrote (GZ)
    case = make_case("nrx_rt", batch=64, users=users, prbs=4, snr_db=12, seed=80 + users,
                     active=np.random.default_rng(80 + users).integers(0, 2, size=(64, users)).astype(np.float32))
    _check(case, oracle=users == 3)


# ---------------------------------------------------------------- one-launch column forward
FWD = COL | 32


def _run_fwd(case, mask=FWD):
    eng = _engine(case)
    eng.fused_config(enable=True)
    eng.update_schedule(mask)
    eng.profile(True)
    out = run_engine(case, "f16", eng)
    prof = eng.profile_read()
    eng.profile(False)
    eng.check()          # no dependency-wait timeout, every counter complete
    return out, prof


def _check_fwd(case, oracle=True):
    ref, _ = _run(case, 0)
    got, pg = _run_fwd(case)
    assert pg["forward_col"][0] == 1 and pg["state_update"][0] == 0 and pg["forward"][0] == 0, pg
    assert np.array_equal(ref["llr_raw"], got["llr_raw"]), np.abs(ref["llr_raw"] - got["llr_raw"]).max()
    assert np.array_equal(ref["h_hat"], got["h_hat"])
    if oracle:
        c = compare(run_oracle(case), got)
        assert c["llr_rel"] < 0.10 and c["llr_rms_rel"] < 0.02 and c["flip_rate_confident"] <= 1e-3, c


def test_fwd_col_bench_shape():
    # BASELINE configs[1] as ONE launch (k_fwd_col): StateInit, aggregation and readout items behind
    # per-slot counters, bit-identical to the three strip launches
    _check_fwd(make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=91))


def test_fwd_col_repeated_and_inactive_users():
    # the counters are reset by the last workgroup: consecutive forwards on one handle agree; random
    # activity, fewer items than CUs
    case = make_case("nrx_rt", batch=96, users=2, prbs=4, snr_db=12, seed=92,
                     active=np.random.default_rng(92).integers(0, 2, size=(96, 2)).astype(np.float32))
    ref, _ = _run(case, 0)
    for _ in range(3):
        got, pg = _run_fwd(case)
        assert pg["forward_col"][0] == 1
        assert np.array_equal(ref["llr_raw"], got["llr_raw"])


def test_fwd_col_u1_two_prb():
    # U = 1 (ips = 1), F = 24 (positions 24..47 past the grid); 200 slots <= 256 CUs (and too many
    # items for the small-strip latency tiers, which take precedence)
    _check_fwd(make_case("nrx_rt", batch=200, users=1, prbs=2, snr_db=12, seed=93))


def test_fwd_col_masking_8_iterations():
    # nrx_large_var_mcs_64qam_masking (BASELINE cfg4'): one StateInit, 8 iterations (9 stages), one
    # 6-bit head; 128 slots x 2 users = 256 items per stage
    case = make_case("nrx_large_var_mcs_64qam_masking", batch=128, users=2, prbs=4, snr_db=14, seed=94)
    ref, _ = _run(case, 0)
    got, pg = _run_fwd(case)
    assert pg["forward_col"][0] == 1, pg
    assert np.array_equal(ref["llr_raw"], got["llr_raw"])
    assert np.array_equal(ref["h_hat"], got["h_hat"])


def test_fwd_col_not_taken_beyond_one_item_per_cu():
    # 256 slots x 2 users > CUs: the three column launches run instead
    case = make_case("nrx_rt", batch=256, users=2, prbs=4, snr_db=12, seed=95)
    _, pg = _run_fwd(case)
    assert pg["forward_col"][0] == 0 and pg["state_update_col"][0] == 2, pg
