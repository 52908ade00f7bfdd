"""Parity of the HIP engine against the oracle (needs an MI355X).

Tolerances (stated per precision, DESIGN.md "Parity"):
* NRX_PREC_F32X (f32 activations, f64 arithmetic): LLR max-abs < 1e-3 against the
  fp64 oracle -- the north-star bound -- and h_hat max-abs < 1e-4.
* NRX_PREC_F16 (perf mode, like the reference's own ``trtexec --fp16`` export):
  hard decisions agree on >= 99.9 % of the bits whose reference |LLR| > 0.5 and on
  >= 99.5 % of all bits; RMS LLR error <= 2 % of the RMS LLR; max-abs LLR error
  <= 10 % of max|LLR|.  The max-abs bound is looser than SURVEY.md 8(d)'s suggested
  3 % because rounding the *trained weights* to f16 alone moves the fp64 oracle's
  LLRs by up to 8.6 % of max|LLR| (tools/fp16_sensitivity.py); the deviation sits on
  large, confident LLRs and leaves decisions and BER unchanged.  SURVEY.md 8(d)'s third
  criterion backs the bound: tests/test_gpu_ber_equivalence.py holds the f16 engine's
  uncoded BER on generated slots within 3 sigma of the fp64 oracle's (nrx_rt and the 64-QAM
  masking model, two Eb/N0 points each).
"""
import numpy as np
import pytest

from tests.helpers import compare, make_case, run_engine, run_oracle

pytestmark = pytest.mark.gpu

F32X_LLR_TOL = 1e-3
F32X_H_TOL = 1e-4
F16_REL_TOL = 0.10
F16_RMS_TOL = 0.02
F16_FLIP_TOL = 5e-3
F16_FLIP_CONF_TOL = 1e-3

_engines = {}


def _weights_key(ws):
    # content fingerprint: two seeded weight sets of one spec must not share an engine
    return tuple((np.shape(w), float(np.asarray(w, np.float64).ravel()[:16].sum())) for w in ws)


def engine_for(case):
    """One engine per (model, spec, weight set)."""
    from neural_rx_amd.receiver import CGNNEngine
    key = (case.name, case.spec, _weights_key(case.weights))
    if key not in _engines:
        _engines[key] = CGNNEngine(case.spec, case.weights)
    return _engines[key]


def check_both(case, f16=True):
    ref = run_oracle(case)
    got = run_engine(case, "f32x", engine_for(case))
    c = compare(ref, got)
    assert np.isfinite(got["llr_raw"]).all()
    assert c["llr_maxabs"] < F32X_LLR_TOL, c
    assert c["h_maxabs"] < F32X_H_TOL, c
    if f16:
        got16 = run_engine(case, "f16", engine_for(case))
        c16 = compare(ref, got16)
        assert np.isfinite(got16["llr_raw"]).all()
        assert c16["llr_rel"] <= F16_REL_TOL, c16
        assert c16["llr_rms_rel"] <= F16_RMS_TOL, c16
        assert c16["flip_rate"] <= F16_FLIP_TOL, c16
        assert c16["flip_rate_confident"] <= F16_FLIP_CONF_TOL, c16
    return c


def test_nrx_rt_two_users():
    check_both(make_case("nrx_rt", batch=3, users=2, prbs=4, snr_db=15))


def test_nrx_rt_single_user_batch1():
    # BASELINE config 1 shape: 1 UE, 4 PRB, B = 1
    check_both(make_case("nrx_rt", batch=1, users=1, prbs=4, snr_db=20))


def test_inactive_user():
    check_both(make_case("nrx_rt", batch=2, users=2, prbs=4, active=[[1, 0], [1, 1]]))


def test_num_it_1():
    check_both(make_case("nrx_rt", batch=2, users=2, prbs=4, num_it=1))


def test_odd_grid_width_random_inputs():
    # F = 50 is not a multiple of the strip width: partial last strip
    case = make_case("nrx_rt", batch=2, users=2, prbs=4, random_inputs=True)
    from oracle import pe_ref
    rng = np.random.default_rng(7)
    case.y = rng.standard_normal((2, 50, 14, 8)).astype(np.float32)
    case.h_hat = rng.standard_normal((2, 2, 50, 14, 8)).astype(np.float32)
    case.pe = pe_ref.pe_for_groups(50, 14, (2, 11), (0, 1))
    check_both(case)


def test_all_zero_slot():
    case = make_case("nrx_rt", batch=2, users=2, prbs=2)
    case.y[1] = 0
    case.h_hat[1] = 0
    check_both(case)


def test_large_grid_separate_norm_pass():
    # 25 PRB x 4 antennas: the slot grid exceeds the fused-normalisation limit, so the
    # per-slot k_norm pass runs before StateInit (one slot all-zero: divide-no-nan)
    case = make_case("nrx_rt", batch=2, users=1, prbs=25, snr_db=12)
    case.y[0] = 0
    case.h_hat[0] = 0
    check_both(case)


def test_var_io_mixed_mcs():
    check_both(make_case("nrx_rt_var_mcs", batch=4, users=2, prbs=4,
                         mcs_choice=[[0, 1], [1, 0], [1, 1], [0, 0]]))


def test_masking_64qam_8_iterations():
    check_both(make_case("nrx_large_var_mcs_64qam_masking", batch=2, users=2, prbs=2,
                         mcs_choice=[[2, 1], [0, 2]], snr_db=22))


def test_nrx_large_four_users():
    check_both(make_case("nrx_large", batch=2, users=4, prbs=2, snr_db=15))


def test_sixteen_antennas_seeded_weights():
    # BASELINE config 3 topology: no trained 16-antenna weights exist
    case = make_case("nrx_large", batch=1, users=4, prbs=1, num_rx_ant=16, seeded_weights=True,
                     random_inputs=True)
    check_both(case)


def test_eight_users_64qam():
    check_both(make_case("nrx_large_64qam", batch=1, users=8, prbs=1, snr_db=25))


def test_receiver_layouts_consistent():
    import torch
    from neural_rx_amd.receiver import NeuralReceiver
    case = make_case("nrx_rt", batch=2, users=2, prbs=4)
    nrx = NeuralReceiver("nrx_rt", precision="f32x")
    yc = torch.from_numpy(case.slots.y_complex).cuda()
    h = torch.from_numpy(case.h_hat).cuda()
    act = torch.from_numpy(case.active).cuda()
    llr_s = nrx(yc, active_dmrs=act, h_hat=h, layout="sionna")
    y = torch.from_numpy(case.y).cuda()
    llr_a = nrx((y[..., :4].contiguous(), y[..., 4:].contiguous()), active_dmrs=act, h_hat=h,
                layout="aerial")
    torch.cuda.synchronize()
    assert tuple(llr_a.shape) == (2, 4, 2, 48, 14)
    np.testing.assert_allclose(llr_a.cpu().numpy(), -llr_s.permute(0, 4, 1, 2, 3).cpu().numpy(),
                               atol=1e-5)
    ref = run_oracle(case)
    assert np.abs(llr_s.cpu().numpy() - ref["llr"][0]).max() < F32X_LLR_TOL


# Paired update path (two aggregation-tail items per workgroup, the second item's z image
# DMA'd during the first one's epilogue; taken when items % 16 == 0 and items >= 2 x CUs).
# Each case is compared bit for bit with a run of only 4 of its slots: a slot's outputs must
# not depend on the batch it runs in or on which workgroup ran it.  The 4-slot run has no
# more items than CUs, so it takes the small-strip tier (8-row strips, P16S, unpaired): the
# check covers pairing AND strip-width invariance together (a failure does not say which;
# tests/test_gpu_baseline_shapes.py compares the paired bench path with the oracle directly).  Cases: the bench shape; U = 1 (no other user: zero aggregate chunks);
# a random active mask (act = 0 users, p = 1 / (#active - 1)); B = 136 (not a multiple of 8:
# work_item's plain-order tail); F = 60 (a partial last strip, 3 strips).  The last update
# pairs too when its heads fit beside the strip image (TAIL_READOUT_WB: one LLR head, W2
# rows truncated to the real bits / ChEst outputs): the 64-QAM masking model (6 bits, 8
# iterations) covers a second truncation; Var-IO (two heads) keeps the unpaired readout.
PAIRED_CASES = {
    "bench_b128_u2": dict(batch=128, users=2, prbs=4),
    "u1_b512": dict(batch=512, users=1, prbs=4),
    "random_active_b128": dict(batch=128, users=2, prbs=4, active="random"),
    "b136_tail": dict(batch=136, users=2, prbs=4),
    "f60_partial_strip": dict(batch=128, users=2, prbs=5),
    "masking_64qam_b128": dict(config="nrx_large_var_mcs_64qam_masking", batch=128, users=2, prbs=4, snr_db=22),
    "var_io_b128": dict(config="nrx_rt_var_mcs", batch=128, users=2, prbs=4),
    # U = 8 > kInlineUsers: k_combine forms a_u in place (register z-load, unpaired)
    "u8_combined_b16": dict(config="nrx_large_64qam", batch=16, users=8, prbs=8, snr_db=25),
}


@pytest.mark.parametrize("name", list(PAIRED_CASES))
def test_batch_composition_invariance_paired_items(name):
    import torch
    kw = dict(PAIRED_CASES[name])
    rng = np.random.default_rng(5)
    if kw.get("active") == "random":
        kw["active"] = (rng.random((kw["batch"], kw["users"])) < 0.6).astype(np.float32)
    kw.setdefault("snr_db", 12)
    case = make_case(kw.pop("config", "nrx_rt"), seed=11, **kw)
    eng = engine_for(case)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()
    multi = case.spec.num_mcs > 1
    llr, h = eng.forward(t(case.y), t(case.pe), t(case.h_hat), t(case.active),
                         t(case.mcs_mask) if multi else None, None, "f16")
    B = kw["batch"]
    llr_np, h_np = llr.cpu().numpy(), h.cpu().numpy()
    assert np.isfinite(llr_np).all()
    bad = []
    # every slot, 4 at a time (each 4-slot run stays in the small-strip tier)
    for s0 in range(0, B, 4):
        sel = list(range(s0, min(s0 + 4, B)))
        llr4, h4 = eng.forward(t(case.y[sel]), t(case.pe), t(case.h_hat[sel]), t(case.active[sel]),
                               t(case.mcs_mask[sel]) if multi else None, None, "f16")
        l4, hh4 = llr4.cpu().numpy(), h4.cpu().numpy()
        for i, b in enumerate(sel):
            if not (np.array_equal(llr_np[:, b], l4[:, i]) and np.array_equal(h_np[b], hh4[i])):
                bad.append(b)
    assert not bad, f"slots whose outputs depend on the batch: {bad}"
