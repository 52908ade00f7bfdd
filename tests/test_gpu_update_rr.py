"""Register-resident update launch (k_update_rr, nrx_rr.inc; DESIGN.md sections A.13-A.14).

Every MFMA of k_update_rr sees the operands of the strip kernel's GZ items in the same order, so
its outputs must equal the strip update kernels' bit for bit: each case runs the three-launch
f16 forward twice on one engine, update_schedule(0) (strip k_update) and a stage mask (default 3:
k_update_rr for every update stage), checks from the per-launch profile that the intended kernel ran, compares LLRs and
h_ref exactly, and the RR result against the fp64 oracle within the f16 gate of
tests/test_gpu_parity.py."""
import numpy as np
import pytest

from tests.helpers import compare, make_case, run_engine, run_oracle

pytestmark = pytest.mark.gpu

_ENGINES = {}


def _engine(case):
    from neural_rx_amd.receiver import CGNNEngine
    key = (case.spec, case.weights[0].tobytes()[:64], len(case.weights))
    if key not in _ENGINES:
        _ENGINES.clear()
        _ENGINES[key] = CGNNEngine(case.spec, case.weights)
    return _ENGINES[key]


def _run(case, rr):
    eng = _engine(case)
    eng.fused_config(enable=False)      # the three-launch forward (whose update stage this is)
    eng.update_schedule(rr)
    try:
        eng.profile(True)
        out = run_engine(case, "f16", eng)
        prof = eng.profile_read()
        eng.profile(False)
    finally:
        eng.update_schedule(1)          # the library default: register-resident aggregation updates
        eng.fused_config(enable=True)
    return out, prof


def _check(case, oracle=True, rr_launches=None, mask=3):
    n_it = case.num_it or case.spec.num_it
    rr_launches = n_it if rr_launches is None else rr_launches
    ref, pr = _run(case, 0)
    got, pg = _run(case, mask)
    assert pr["state_update_rr"][0] == 0 and pr["state_update"][0] == n_it
    assert pg["state_update_rr"][0] == rr_launches and pg["state_update"][0] == n_it - rr_launches, pg
    assert np.array_equal(ref["llr_raw"], got["llr_raw"]), np.abs(ref["llr_raw"] - got["llr_raw"]).max()
    assert np.array_equal(ref["h_hat"], got["h_hat"])
    if oracle:
        c = compare(run_oracle(case), got)
        assert c["llr_rel"] < 0.10 and c["llr_rms_rel"] < 0.02 and c["flip_rate_confident"] <= 1e-3, c


def test_rr_bench_shape():
    # BASELINE configs[1]: nrx_rt, 2 UE, 4 PRB (F = 48: three 16-row strips), B = 128
    _check(make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=51))


def test_rr_random_activity_u1_f_not_multiple_of_16():
    # U = 1 (no other user: a chunks out of range), F = 60 (5 PRB: the last strip has 12 rows
    # in the grid), inactive slots
    case = make_case("nrx_rt", batch=96, users=1, prbs=5, snr_db=10, seed=52,
                     active=np.random.default_rng(52).integers(0, 2, size=(96, 1)).astype(np.float32))
    _check(case)


def test_rr_u2_inactive_user():
    case = make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=14, seed=53,
                     active=np.random.default_rng(53).integers(0, 2, size=(128, 2)).astype(np.float32))
    _check(case)


def test_rr_16_antennas_8_iterations():
    # 2A = 32 (ChEst head CHP = 32), nrx_large topology (8 iterations), seeded weights, 132 PRB
    case = make_case("nrx_large", batch=4, users=2, prbs=132, num_rx_ant=16, seeded_weights=True,
                     random_inputs=True, seed=54)
    _check(case, oracle=False)


def test_rr_var_io_three_launch():
    # Var-IO (two StateInits), one-hot MCS mask: the aggregation update runs register-resident,
    # the readout (two LLR heads) the strip kernel
    rng = np.random.default_rng(55)
    case = make_case("nrx_rt_var_mcs", batch=128, users=2, prbs=4, snr_db=14, seed=55,
                     mcs_choice=rng.integers(0, 2, size=(128, 2)))
    _check(case, oracle=False, rr_launches=case.spec.num_it - 1)


@pytest.mark.parametrize("mask", [1, 2])
def test_rr_stage_masks(mask):
    # nrx_update_schedule is a stage mask: 1 (the default) the aggregation updates only, 2 the
    # readout update only; the other stages run the strip kernel, outputs unchanged
    # (nrx_large topology: 8 iterations, so 7 aggregation updates and one readout update; B = 128
    # so that the grid takes the 24-row strip tier, the one with the RR launch)
    case = make_case("nrx_large", batch=128, users=2, prbs=4, seeded_weights=True, random_inputs=True, seed=56)
    n_it = case.num_it or case.spec.num_it
    _check(case, oracle=False, rr_launches=n_it - 1 if mask == 1 else 1, mask=mask)


def test_rr_one_prb_strip_past_the_grid():
    # F = 12 < 16: the only strip's rows 12..18 lie past the grid (zeroed behind the uniform
    # branch of rr_to_own); U = 1, B = 640 so that the 24-row tier (and the RR launch) is taken
    case = make_case("nrx_rt", batch=640, users=1, prbs=1, snr_db=12, seed=57)
    _check(case)


def test_rr_three_users_combine_pass():
    # U = 3: conv1 reads the a_u planes k_combine wrote (GZ), both update stages register-resident
    case = make_case("nrx_rt", batch=128, users=3, prbs=4, snr_db=12, seed=58,
                     active=np.random.default_rng(58).integers(0, 2, size=(128, 3)).astype(np.float32))
    _check(case)


@pytest.mark.parametrize("users", [4, 8])
def test_rr_users_4_8_combine_pass(users):
    # U = 4 / 8: conv1 of every RR item reads the a_u planes k_combine wrote (GZ); outputs must
    # equal the strip kernels' bit for bit, with random activity (p = 1/(n-1) varies per slot)
    case = make_case("nrx_rt", batch=64, users=users, prbs=4, snr_db=12, seed=59 + users,
                     active=np.random.default_rng(59 + users).integers(0, 2, size=(64, users)).astype(np.float32))
    _check(case, oracle=users == 4)


def test_update_schedule_mask_validation(monkeypatch):
    # nrx_update_schedule takes a stage mask 0..127 (< 0: unchanged); NRX_UPDATE_RR must be a
    # decimal 0..127 or nrx_create fails (no silent fallback to a schedule the caller did not ask for)
    from neural_rx_amd import _lib
    from neural_rx_amd.receiver import CGNNEngine
    case = make_case("nrx_rt", batch=2, users=2, prbs=4, seed=63)
    eng = CGNNEngine(case.spec, case.weights)
    try:
        for m in (0, 1, 2, 3, 4, 16, 29, 31, 61, 63, 64, 127, -1, True, False, None):
            eng.update_schedule(m)
        with pytest.raises(_lib.NRXError):
            eng.update_schedule(128)
        # nrx_fused_config: enable 0 / 1 / 2 (< 0 unchanged); 3 is an error, not "force" 
        assert eng._lib.nrx_fused_config(eng._h, 3, -1, -1) == _lib.NRX_ERR_INVALID_ARG
        assert eng._lib.nrx_fused_config(eng._h, 2, -1, -1) == 0
        assert eng._lib.nrx_fused_config(eng._h, 1, -1, -1) == 0
    finally:
        eng.close()
    for bad in ("128", "on", "1x", "-1"):
        monkeypatch.setenv("NRX_UPDATE_RR", bad)
        with pytest.raises(_lib.NRXError):
            CGNNEngine(case.spec, case.weights)
