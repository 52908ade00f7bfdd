"""Aerial (NeuralReceiverONNX / TensorRT) contract: FOCC removal, per-PRB nearest-pilot
interpolation and positional encoding on the GPU, LLRs in the Aerial
layout and sign (8(a) a14).

CPU tests pin the oracle's restatement (oracle/pe_ref.aerial_preprocess, TF semantics of
NRPreprocessing, neural_rx.py:1614-1711) against an element-wise restatement and the
reference's golden FOCC vector; GPU tests compare nrx_forward_aerial with it:
* preprocessing is a gather + pair average: checked bit-exactly through the engine's own
  CGNN (Aerial forward == plain forward on the oracle-preprocessed tensors, f32x, LLR
  agreement < 1e-5 -- the only inexact step is the PE's mean/std, computed in f64 on both);
* end to end against the fp64 oracle: f32x LLR max-abs < 1e-3, h_hat < 1e-4; f16 within the
  gates of tests/test_gpu_parity.py;
* shapes of the reference's TRT engine at 132 PRB (real_time_nrx.ipynb:776-777).
"""
import numpy as np
import pytest

from oracle import pe_ref
from tests.helpers import compare, make_aerial_case, run_engine, run_engine_aerial, run_oracle

F32X_LLR_TOL = 1e-3
F32X_H_TOL = 1e-4


def _oracle_gather_direct(hr, hi, nn, B, U, F, T, A, nsym, npil):
    nprb = F // 12
    out = np.zeros((B, U, F, T, 2 * A), np.float32)
    for b in range(B):
        for u in range(U):
            for f in range(F):
                for t in range(T):
                    i = nn[u, 0, t, f % 12]
                    k, j = divmod(i, npil)
                    p = (k * nprb + f // 12) * npil + j
                    q = p ^ 1
                    out[b, u, f, t, :A] = (hr[b, p, u] + hr[b, q, u]) / np.float32(2)
                    out[b, u, f, t, A:] = (hi[b, p, u] + hi[b, q, u]) / np.float32(2)
    return out


@pytest.mark.parametrize("groups", [(0, 1), (1, 0), (0, 0)])
def test_oracle_preprocess_matches_elementwise_restatement(groups):
    rng = np.random.default_rng(3)
    B, F, T, A, U = 2, 24, 14, 4, len(groups)
    yr, yi = rng.standard_normal((2, B, F, T, A)).astype(np.float32)
    hr, hi = rng.standard_normal((2, B, 2 * (F // 12) * 6, U, A)).astype(np.float32)
    ofdm = np.array([[2, 11]] * U, np.int32)
    scp = np.array([[g + 2 * j for j in range(6)] for g in groups], np.int32)
    y, h, pe = pe_ref.aerial_preprocess(yr, yi, hr, hi, ofdm, scp, U)
    np.testing.assert_array_equal(y, np.concatenate([yr, yi], -1))
    nn, _ = pe_ref.aerial_nn_indices(ofdm, scp, T, F // 12)
    np.testing.assert_array_equal(h, _oracle_gather_direct(hr, hi, nn, B, U, F, T, A, 2, 6))
    assert pe.shape == (U, F, T, 2)


def test_nn_index_is_first_minimum_in_symbol_major_order():
    # RE (t=0, sc=1) of a group-0 user: pilots (k=0: sym 2) at sc 0 and 2 are both at
    # Manhattan distance 3; the first in the (k, j) list order (sc 0, j = 0) wins.
    nn, _ = pe_ref.aerial_nn_indices(np.array([[2, 11]], np.int32),
                                     np.array([[0, 2, 4, 6, 8, 10]], np.int32), 14, 1)
    assert nn[0, 0, 0, 1] == 0
    assert nn[0, 0, 13, 1] == 6          # nearer to the symbol-11 pilots (k = 1)


def test_aerial_case_ber_is_sane():
    # the trained nrx_rt weights decode the Aerial-preprocessed synthetic slots (15 dB)
    from neural_rx_amd import synth
    ac = make_aerial_case(batch=2, users=2, prbs=4, snr_db=15.0, seed=5)
    ref = run_oracle(ac.case)
    for u in range(2):
        assert synth.uncoded_ber(ref["llr"][0], ac.case.slots, u, 4) < 0.02


# ------------------------------------------------------------------------------ GPU
_engines = {}


def _engine(case):
    from neural_rx_amd.receiver import CGNNEngine
    key = case.name
    if key not in _engines:
        _engines[key] = CGNNEngine(case.spec, case.weights)
    return _engines[key]


@pytest.mark.gpu
@pytest.mark.parametrize("prbs,users", [(4, 2), (3, 1)])
def test_aerial_forward_matches_plain_forward_on_preprocessed_inputs(prbs, users):
    ac = make_aerial_case(batch=2, users=users, prbs=prbs, seed=11)
    eng = _engine(ac.case)
    llr_a, h_a = run_engine_aerial(ac, "f32x", eng)
    plain = run_engine(ac.case, "f32x", eng)
    bits = ac.case.spec.bits[0]
    ref_layout = -np.transpose(plain["llr_raw"][0][..., :bits], (0, 4, 1, 2, 3))
    assert llr_a.shape == ref_layout.shape
    assert np.abs(llr_a - ref_layout).max() < 1e-5 * max(1.0, np.abs(ref_layout).max())
    assert np.abs(h_a - plain["h_hat"]).max() < 1e-6


@pytest.mark.gpu
def test_aerial_forward_matches_oracle():
    ac = make_aerial_case(batch=3, users=2, prbs=4, seed=12, active=[[1, 1], [1, 0], [1, 1]])
    eng = _engine(ac.case)
    ref = run_oracle(ac.case)
    bits = ac.case.spec.bits[0]
    for prec in ("f32x", "f16"):
        llr_a, h_a = run_engine_aerial(ac, prec, eng)
        got = {"llr": [-np.transpose(llr_a, (0, 2, 3, 4, 1))], "h_hat": h_a}
        c = compare({"llr": [ref["llr"][0][..., :bits]], "h_hat": ref["h_hat"]}, got)
        if prec == "f32x":
            assert c["llr_maxabs"] < F32X_LLR_TOL, c
            assert c["h_maxabs"] < F32X_H_TOL, c
        else:
            assert c["llr_rel"] <= 0.10 and c["llr_rms_rel"] <= 0.02, c
            assert c["flip_rate_confident"] <= 1e-3, c


@pytest.mark.gpu
def test_aerial_receiver_trt_shapes():
    # the reference TRT engine's I/O at 132 PRB: llr (1, 4, 2, 1584, 14), h_hat
    # (1, 2, 1584, 14, 8) (real_time_nrx.ipynb:776-777)
    import torch
    from neural_rx_amd.receiver import AerialReceiver
    ac = make_aerial_case(batch=1, users=2, prbs=132, seed=13)
    nrx = AerialReceiver("nrx_rt", precision="f16")
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in ac.inputs.items()}
    llr, h = nrx((t["y_real"], t["y_imag"], t["h_ls_real"], t["h_ls_imag"], t["dmrs_port_mask"],
                  t["dmrs_ofdm_pos"], t["dmrs_subcarrier_pos"]))
    torch.cuda.synchronize()
    assert tuple(llr.shape) == (1, 4, 2, 1584, 14)
    assert tuple(h.shape) == (1, 2, 1584, 14, 8)
    assert torch.isfinite(llr).all() and torch.isfinite(h).all()


# ------------------------------------------------------------------ coded-bit layout (f2)
def test_data_re_count_matches_reference_kat():
    # 4 PRB, 16-QAM, DMRS on 2 symbols without data: 2304 coded bits per user
    # (jumpstart_tutorial.ipynb:312)
    from neural_rx_amd.config import data_re_indices, get_config
    re = data_re_indices(get_config("nrx_rt"), 48)
    assert re.size * 4 == 2304
    # grid order = argsort of the RG type grid (data = 0 first, stable, symbol-major)
    typ = np.ones((14, 48), np.int32)
    typ[[t for t in range(14) if t not in (2, 11)]] = 0
    np.testing.assert_array_equal(np.argsort(typ.ravel(), kind="stable")[:re.size], re)


@pytest.mark.gpu
def test_llr_demap_matches_numpy_gather():
    import torch
    from neural_rx_amd.config import data_re_indices, get_config
    from neural_rx_amd.receiver import NeuralReceiver
    case_rng = np.random.default_rng(5)
    B, U, F, T, S = 3, 2, 48, 14, 6
    llr = case_rng.standard_normal((B, U, F, T, S)).astype(np.float32)
    re = data_re_indices(get_config("nrx_rt"), F)
    nrx = NeuralReceiver("nrx_rt")
    out = nrx.cgnn.engine.llr_demap(torch.from_numpy(llr).cuda(), 4, torch.from_numpy(re).cuda())
    torch.cuda.synchronize()
    t, f = re // F, re % F
    ref = llr[:, :, f, t, :4].reshape(B, U, -1)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.gpu
def test_receiver_demap_output_is_coded_bits():
    import torch
    from neural_rx_amd import synth
    from neural_rx_amd.receiver import NeuralReceiver
    from tests.helpers import make_case
    case = make_case("nrx_rt", batch=2, users=2, prbs=4, snr_db=20.0, seed=8)
    nrx = NeuralReceiver("nrx_rt", precision="f32x")
    yc = torch.from_numpy(case.slots.y_complex).cuda()
    llr = nrx(yc, active_dmrs=torch.from_numpy(case.active).cuda(),
              h_hat=torch.from_numpy(case.h_hat).cuda(), demap=True)
    torch.cuda.synchronize()
    assert tuple(llr.shape) == (2, 2, 2304)
    # coded bits in grid order: the transmitted bits of the data REs, symbol-major
    dm = case.slots.data_mask
    bits = case.slots.bits[:, :, :, dm, :4].transpose(0, 1, 3, 2, 4).reshape(2, 2, -1)
    ber = float(((llr.cpu().numpy() > 0).astype(np.uint8) != bits).mean())
    assert ber < 0.01
