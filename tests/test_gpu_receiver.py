"""NeuralReceiver wrapper semantics against CGNNOFDM.forward (neural_rx.py:813-881), on the GPU.

* layout="sionna": the complex resource grid ``[B,1,A,14,F]`` goes to libnrx as is
  (``nrx_forward_ex``, NRX_Y_SIONNA_RG); the result is bit-identical to feeding the
  CGNN-layout ``y`` (the layout change is an exact copy) and within the f32x bound of the
  oracle.
* layout="aerial": (rx_slot_real, rx_slot_imag) through NRX_Y_SPLIT, bit-identical too.
* ``mcs_arr_eval``: the state-init mask defaults to one_hot(mcs_arr_eval[0]) and the
  demapped output is head mcs_arr_eval[0] (the reference returns ``llrs[-1][0]``);
  ``all_mcs`` demaps every listed MCS with its own head and bit count.
"""
import numpy as np
import pytest

from tests.helpers import make_case, run_oracle

pytestmark = pytest.mark.gpu


def _t(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_sionna_grid_layout_in_libnrx():
    import torch
    from neural_rx_amd.receiver import NeuralReceiver
    case = make_case("nrx_rt", batch=3, users=2, prbs=4, snr_db=12, seed=31)
    nrx = NeuralReceiver("nrx_rt", precision="f32x")
    yc = _t(case.slots.y_complex)                      # [B, 1, A, 14, F] complex64
    assert yc.dtype == torch.complex64 and yc.dim() == 5
    h, act = _t(case.h_hat), _t(case.active)
    llr_rg, h_rg = nrx(yc, active_dmrs=act, h_hat=h, layout="sionna", return_h_hat=True)
    llr_cg, h_cg = nrx(_t(case.y), active_dmrs=act, h_hat=h, layout="cgnn", return_h_hat=True)
    torch.cuda.synchronize()
    assert torch.equal(llr_rg, llr_cg) and torch.equal(h_rg, h_cg)
    ref = run_oracle(case)
    assert np.abs(llr_rg.cpu().numpy() - ref["llr"][0]).max() < 1e-3


def test_split_layout_in_libnrx():
    import torch
    from neural_rx_amd.receiver import NeuralReceiver
    case = make_case("nrx_rt", batch=2, users=2, prbs=4, snr_db=12, seed=32)
    nrx = NeuralReceiver("nrx_rt", precision="f16")
    y = _t(case.y)
    h, act = _t(case.h_hat), _t(case.active)
    llr_a = nrx((y[..., :4].contiguous(), y[..., 4:].contiguous()), active_dmrs=act, h_hat=h, layout="aerial")
    llr_c = nrx(y, active_dmrs=act, h_hat=h, layout="cgnn")
    torch.cuda.synchronize()
    assert torch.equal(llr_a, -llr_c.permute(0, 4, 1, 2, 3))


def test_mcs_arr_eval_var_io():
    import torch
    from neural_rx_amd.receiver import NeuralReceiver
    case = make_case("nrx_rt_var_mcs", batch=2, users=2, prbs=4, snr_db=12, seed=33, mcs_choice=[[1, 1], [1, 1]])
    nrx = NeuralReceiver("nrx_rt_var_mcs", precision="f32x")
    yc, h, act = _t(case.slots.y_complex), _t(case.h_hat), _t(case.active)
    # mcs_arr_eval = [1]: mask one_hot(1) (== case.mcs_mask), output = head 1 (16-QAM)
    got = nrx(yc, active_dmrs=act, h_hat=h, mcs_arr_eval=[1], demap=True)
    ref = run_oracle(case)["llr"][1]                                 # [B, U, F, T, 4]
    from neural_rx_amd.config import data_re_indices, get_config
    dre = data_re_indices(get_config("nrx_rt_var_mcs"), 48)
    t_idx, f_idx = dre // 48, dre % 48
    ref_cb = ref[:, :, f_idx, t_idx, :].reshape(2, 2, -1)
    torch.cuda.synchronize()
    assert got.shape == (2, 2, ref_cb.shape[-1])
    assert np.abs(got.cpu().numpy() - ref_cb).max() < 1e-3
    # every listed MCS demapped with its own head; same state (mask from mcs_arr_eval[0])
    both = nrx(yc, active_dmrs=act, h_hat=h, mcs_arr_eval=[1, 0], demap=True, all_mcs=True)
    torch.cuda.synchronize()
    assert len(both) == 2 and torch.equal(both[0], got)
    assert both[1].shape == (2, 2, ref_cb.shape[-1] // 2)            # QPSK: 2 bits per RE
    ref0 = run_oracle(case)["llr"][0][:, :, f_idx, t_idx, :].reshape(2, 2, -1)
    assert np.abs(both[1].cpu().numpy() - ref0).max() < 1e-3
