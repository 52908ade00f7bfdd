"""CPU tests of the oracle: pinned to the reference's golden vectors, param counts and
known PE values, plus invariances of the full CGNN restatement."""
import os

import numpy as np
import pytest

from neural_rx_amd import synth
from neural_rx_amd import weights as W
from neural_rx_amd.config import BUILTIN, dmrs_symbols, get_config, spec_from_config, user_cdm_groups
from oracle import cgnn_ref, pe_ref
from tests.helpers import make_case, run_oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "ref_modules_nrx_rt.npz")


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN)


@pytest.fixture(scope="module")
def rt():
    cfg = get_config("nrx_rt")
    spec = spec_from_config(cfg)
    return cfg, spec, cgnn_ref.split_keras_weights(W.load("nrx_rt"), spec)


def test_param_counts_match_reference_notebook():
    # nrx_architecture.ipynb:257 / 295-308 (nrx_rt) and :382 (nrx_large)
    c = cgnn_ref.count_params(spec_from_config(get_config("nrx_rt")))
    assert (c["state_init"], c["cgnn_it"], c["readout_llrs"][0], c["readout_chest"], c["total"]) == \
        (28634, 49074, 7812, 8328, 142922)
    assert cgnn_ref.count_params(spec_from_config(get_config("nrx_large")))["total"] == 437366


@pytest.mark.parametrize("name", sorted(BUILTIN))
def test_weight_files_match_topology(name):
    spec = spec_from_config(get_config(name))
    arrays = W.load(name)
    cgnn_ref.split_keras_weights(arrays, spec)       # asserts every shape
    assert sum(a.size for a in arrays) == cgnn_ref.count_params(spec)["total"]


def test_golden_aggregate_user_states(golden, rt):
    _, _, w = rt
    for pre in ("agg", "agg4"):
        s = golden[f"{pre}_s"].astype(np.float64)[:, :, None, None, :]
        act = golden[f"{pre}_active"].astype(np.float64)
        a = cgnn_ref.aggregate(s, act, w.agg[0])[:, :, 0, 0, :]
        np.testing.assert_allclose(a, golden[f"{pre}_a"], rtol=1e-5, atol=2e-4)


def test_golden_readouts(golden, rt):
    _, _, w = rt
    s = golden["ro_s"].astype(np.float64)
    llr = cgnn_ref.dense(cgnn_ref.dense(s, w.llr[0][0], True), w.llr[0][1], False)
    h = cgnn_ref.dense(cgnn_ref.dense(s, w.chest[0], True), w.chest[1], False)
    np.testing.assert_allclose(llr, golden["ro_llr"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(h, golden["ro_h"], rtol=1e-5, atol=1e-5)


def test_golden_focc_removal(golden):
    np.testing.assert_allclose(pe_ref.focc_removal(golden["focc_in"]), golden["focc_out"], atol=1e-6)


def test_pe_known_values():
    # nrx_rt, DMRS on symbols 2/11, user 0 on even / user 1 on odd
    cfg = get_config("nrx_rt")
    assert dmrs_symbols(cfg) == (2, 11)
    assert user_cdm_groups(cfg, 2) == (0, 1)
    pe = pe_ref.pe_for_groups(48, 14, (2, 11), (0, 1))
    want_t = [0.115, -0.688, -1.491, -0.688, 0.115, 0.918, 1.721, 1.721, 0.918, 0.115,
              -0.688, -1.491, -0.688, 0.115]
    np.testing.assert_allclose(pe[0, 0, :, 0], want_t, atol=1e-3)
    np.testing.assert_allclose(pe[:, 5, 3, 0], pe[:, 30, 3, 0])           # time comp independent of f
    np.testing.assert_array_equal(pe[0, :4, 0, 1], [-1, 1, -1, 1])
    np.testing.assert_array_equal(pe[1, :4, 0, 1], [1, -1, 1, -1])


def test_aerial_pe_equals_sionna_pe_for_type1():
    # the per-PRB Aerial variant with TF meshgrid order and population std reproduces a1
    ofdm = np.array([[2, 11], [2, 11]])
    sc = np.array([[0, 2, 4, 6, 8, 10], [1, 3, 5, 7, 9, 11]])
    _, pe_a = pe_ref.aerial_nn_indices(ofdm, sc, 14, 4)
    np.testing.assert_allclose(pe_a, pe_ref.pe_for_groups(48, 14, (2, 11), (0, 1)), atol=1e-6)


def test_ber_sanity_real_weights():
    # the oracle with the trained weights decodes synthetic slots (SURVEY.md 8c probe)
    case = make_case("nrx_rt", batch=4, users=2, prbs=4, snr_db=30, seed=5)
    r = run_oracle(case)
    bers = [synth.uncoded_ber(r["llr"][0], case.slots, u, 4) for u in range(2)]
    assert max(bers) < 5e-3, bers
    case.num_it = 1
    r1 = run_oracle(case)
    assert synth.uncoded_ber(r1["llr"][0], case.slots, 0, 4) > max(bers)


def test_user_permutation_equivariance(rt):
    cfg, spec, w = rt
    case = make_case("nrx_rt", batch=2, users=2, prbs=2, random_inputs=True, seed=11)
    r = run_oracle(case)
    perm = [1, 0]
    case.pe, case.h_hat, case.active, case.mcs_mask = (case.pe[perm], case.h_hat[:, perm],
                                                       case.active[:, perm], case.mcs_mask[:, perm])
    rp = run_oracle(case)
    np.testing.assert_allclose(rp["llr"][0], r["llr"][0][:, perm], atol=1e-9)


def test_inactive_user_does_not_influence_active_users():
    case = make_case("nrx_rt", batch=1, users=2, prbs=2, random_inputs=True, seed=12,
                     active=[[1, 0]])
    r = run_oracle(case)
    case.h_hat = case.h_hat.copy()
    case.h_hat[:, 1] *= -3.0
    r2 = run_oracle(case)
    np.testing.assert_allclose(r2["llr"][0][:, 0], r["llr"][0][:, 0], atol=1e-9)


def test_joint_scaling_invariance_and_batch_independence():
    case = make_case("nrx_rt", batch=3, users=2, prbs=2, random_inputs=True, seed=13)
    r = run_oracle(case)
    case.y = case.y * 8.0              # power of two: exact in f32, so exact invariance
    case.h_hat = case.h_hat * 8.0
    r2 = run_oracle(case)
    np.testing.assert_allclose(r2["llr"][0], r["llr"][0], atol=1e-9)
    one = make_case("nrx_rt", batch=3, users=2, prbs=2, random_inputs=True, seed=13)
    one.y, one.h_hat, one.active, one.mcs_mask = one.y[1:2], one.h_hat[1:2], one.active[1:2], one.mcs_mask[1:2]
    r1 = run_oracle(one)
    np.testing.assert_allclose(r1["llr"][0][0], r["llr"][0][1], atol=1e-9)


def test_single_user_aggregation_is_zero(rt):
    _, _, w = rt
    s = np.random.default_rng(0).standard_normal((2, 1, 3, 14, 56))
    a = cgnn_ref.aggregate(s, np.ones((2, 1)), w.agg[0])
    assert np.abs(a).max() == 0.0


def test_all_zero_slot_is_finite():
    case = make_case("nrx_rt", batch=2, users=2, prbs=1, random_inputs=True, seed=14)
    case.y[0] = 0
    case.h_hat[0] = 0
    r = run_oracle(case)
    assert np.isfinite(r["llr"][0]).all()
    assert r["norm_scale"][0] == 0.0


def test_fp32_oracle_close_to_fp64():
    # documents the fp32 rounding noise of the reference arithmetic (DESIGN.md "Parity")
    case = make_case("nrx_rt", batch=2, users=2, prbs=4, snr_db=15, seed=2)
    r64 = run_oracle(case)
    r32 = run_oracle(case, dtype=np.float32)
    d = np.abs(r64["llr"][0] - r32["llr"][0]).max()
    assert d < 1e-2


@pytest.mark.parametrize("config,users,kw", [
    ("nrx_rt", 2, {}),
    ("nrx_rt_var_mcs", 2, {"mcs_choice": [[0, 1], [1, 0]]}),
    ("nrx_large_var_mcs_64qam_masking", 2, {"mcs_choice": [[2, 0], [1, 2]], "snr_db": 22}),
])
def test_torch_cpu_restatement_matches_numpy_oracle(config, users, kw):
    # oracle/cgnn_torch.py (conv2d(groups=C) + 1x1 conv, the CPU baseline) vs the numpy
    # oracle: two independent restatements of the same TF model agree to fp32 rounding
    from oracle import cgnn_ref
    from oracle.cgnn_torch import TorchCGNN
    case = make_case(config, batch=2, users=users, prbs=2, **kw)
    w = cgnn_ref.split_keras_weights(case.weights, case.spec)
    ref = run_oracle(case)
    got = TorchCGNN(w, case.spec).forward(case.y, case.pe, case.h_hat, case.active, case.mcs_mask)
    for r, g in zip(ref["llr"], got["llr"]):
        assert r.shape == g.shape
        assert np.abs(r - g).max() < 2e-3
    assert np.abs(ref["h_hat"] - got["h_hat"]).max() < 1e-4
