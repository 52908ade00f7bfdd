"""Every BASELINE.json per-GPU shape takes the schedule DESIGN.md section 5 documents as its
default: the per-launch profile of one default forward names the kernels that
ran each stage.  Random inputs (the schedule depends on shapes only); seeded weights where no
trained model of that topology exists."""
import numpy as np
import pytest

from tests.helpers import make_case, run_engine

pytestmark = pytest.mark.gpu


def _profile(case):
    from neural_rx_amd.receiver import CGNNEngine
    eng = CGNNEngine(case.spec, case.weights)
    try:
        run_engine(case, "f16", eng)          # warm (workspace, code objects)
        eng.profile(True)
        run_engine(case, "f16", eng)
        prof = {k: v[0] for k, v in eng.profile_read().items() if v[0]}
        eng.profile(False)
        eng.check()
    finally:
        eng.close()
    return prof


def test_cfg1_latency_tier():
    # 1 UE, 4 PRB, B = 1: the small-strip latency tier (strip kernels, three launches)
    prof = _profile(make_case("nrx_rt", batch=1, users=1, prbs=4, random_inputs=True, seed=1))
    assert prof == {"state_init": 1, "state_update": 2}, prof


def test_cfg2_column_launches():
    # the bench shape: column StateInit, aggregation and readout launches
    prof = _profile(make_case("nrx_rt", batch=128, users=2, prbs=4, random_inputs=True, seed=2))
    assert prof == {"state_init_col": 1, "state_update_col": 2}, prof


def test_cfg3_rr_updates_on_a_wide_grid():
    # 4 UE, 132 PRB, 16 rx antennas, B = 64 (3 slot chunks): strip StateInit (2A = 32), the RR
    # aggregation updates, the strip readout, a combine pass after StateInit and every aggregation
    case = make_case("nrx_large", batch=64, users=4, prbs=132, num_rx_ant=16, seeded_weights=True,
                     random_inputs=True, seed=3)
    prof = _profile(case)
    ch = 3
    assert prof == {"norm": ch, "state_init": ch, "state_update_rr": 7 * ch, "state_update": ch, "combine": 8 * ch}, prof


def test_cfg4_var_io():
    # Var-IO (two StateInits), 2 UE, 4 PRB, 128 slots: two column StateInit launches, the column
    # aggregation update, the strip readout (two LLR heads)
    rng = np.random.default_rng(4)
    case = make_case("nrx_rt_var_mcs", batch=128, users=2, prbs=4, random_inputs=True, seed=4,
                     mcs_choice=rng.integers(0, 2, size=(128, 2)))
    prof = _profile(case)
    # (the profiler times the StateInit stage's two launches as one event pair)
    assert prof == {"state_init_col": 1, "state_update_col": 1, "state_update": 1}, prof


def test_cfg4p_masking_8_iterations():
    case = make_case("nrx_large_var_mcs_64qam_masking", batch=128, users=2, prbs=4, random_inputs=True, seed=5)
    prof = _profile(case)
    assert prof == {"state_init_col": 1, "state_update_col": 8}, prof


def test_cfg5_wide_grid_8_users():
    # 8 UE, 273 PRB, 32 slots (6 slot chunks): k_norm, column StateInit, RR aggregation updates,
    # strip readout, combine passes
    case = make_case("nrx_large_64qam", batch=32, users=8, prbs=273, random_inputs=True, seed=6)
    prof = _profile(case)
    ch = 6
    assert prof == {"norm": ch, "state_init_col": ch, "state_update_rr": 7 * ch, "state_update": ch,
                    "combine": 8 * ch}, prof
