"""Python face of the engine, mirroring the reference's receiver interfaces.

* ``CGNNEngine`` -- one ``libnrx.so`` handle; ``forward(y, pe, h_hat, active, mcs_mask)``
  on device-resident torch tensors.
* ``CGNN`` -- the reference's core layer call, ``CGNN.forward([y, pe, h_hat, active_tx,
  mcs_ue_mask]) -> (llrs, h_hats)`` (neural_rx.py:544-595) with the ``num_it`` property
  and its assertion (neural_rx.py:532-542).
* ``NeuralReceiver`` -- the drop-in named by the north star:
  ``NeuralReceiver.__call__(rx_grid, pe=None, active_dmrs=None, h_hat=None,
  mcs_ue_mask=None, num_it=None, layout="sionna") -> llr`` reproducing both wrapper
  layouts: Sionna/``CGNNOFDM.forward`` (neural_rx.py:813-881: ``y[:,0]``
  permuted to ``[B,F,T,A]`` and split into real/imag channels) and Aerial/
  ``NeuralReceiverONNX.forward`` (neural_rx.py:1773-1812: real/imag inputs, LLRs
  permuted to ``[B,bits,U,F,T]`` and negated).

PyTorch tensors are used only as device containers; all arithmetic of the forward pass
runs in the HIP kernels of ``libnrx.so``.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .config import (ModelSpec, NRXConfig, data_re_indices, dmrs_symbols, get_config, spec_from_config,
                     user_cdm_groups)
from . import weights as _weights

NUM_SYMBOLS = 14


def _torch():
    import torch
    return torch


def compute_pe(num_tx: int, num_subcarriers: int, dmrs_syms: Sequence[int],
               cdm_groups: Sequence[int], num_symbols: int = NUM_SYMBOLS) -> np.ndarray:
    """Nearest-pilot positional encoding ``[U, F, T, 2]`` via the C ABI
    (``nrx_compute_pe``; reference formula onnx_utils.py:206-260)."""
    lib = _lib.load()
    pe = np.zeros((num_tx, num_subcarriers, num_symbols, 2), np.float32)
    syms = (ctypes.c_int32 * len(dmrs_syms))(*dmrs_syms)
    grp = (ctypes.c_int32 * num_tx)(*cdm_groups[:num_tx])
    _lib.check(lib.nrx_compute_pe(num_tx, num_subcarriers, num_symbols, syms, len(dmrs_syms), grp,
                                  pe.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
    return pe


class CGNNEngine:
    """Owns one engine handle (packed fp16 + fp64 weights on the device)."""

    def __init__(self, spec: ModelSpec, weight_list: Sequence[np.ndarray], device: int = 0):
        self.spec = spec
        self.device = device
        lib = _lib.load()
        self._lib = lib
        self._desc = _lib.make_desc(spec)
        n = ctypes.c_int32()
        _lib.check(lib.nrx_weight_layout(ctypes.byref(self._desc), ctypes.byref(n), None, 0))
        sizes = (ctypes.c_int64 * n.value)()
        _lib.check(lib.nrx_weight_layout(ctypes.byref(self._desc), ctypes.byref(n), sizes, n.value))
        if len(weight_list) != n.value:
            raise ValueError(f"expected {n.value} weight arrays, got {len(weight_list)}")
        arrs = [np.ascontiguousarray(w, dtype=np.float32) for w in weight_list]
        for i, (a, s) in enumerate(zip(arrs, sizes)):
            if a.size != s:
                raise ValueError(f"weight {i}: {a.shape} has {a.size} elements, expected {s}")
        ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
        self._keep = arrs
        h = ctypes.c_void_p()
        _lib.check(lib.nrx_create(ctypes.byref(self._desc), ptrs, sizes, n.value, device,
                                  ctypes.byref(h)))
        self._h = h
        self._ws = {}

    def close(self):
        if getattr(self, "_h", None):
            self._lib.nrx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -------------------------------------------------------------- profiling
    def profile(self, enable: bool = True):
        _lib.check(self._lib.nrx_profile_enable(self._h, int(enable)))

    def fused_status(self, reset: bool = False, full: bool = False):
        """One-launch forward counters since the last reset: the sticky error bits (1: a
        dependency wait timed out, 2: items left undone), or with ``full`` the dict
        {error, waited, polls} (update items that could not be prefetched, and their polls).
        Reads, never raises on the error bits (``check`` does)."""
        st = (ctypes.c_int32 * 3)()
        rc = self._lib.nrx_fused_status(self._h, st, int(reset))
        if rc != _lib.NRX_ERR_FUSED:
            _lib.check(rc)
        if full:
            return {"error": st[0], "waited": st[1], "polls": st[2]}
        return st[0]

    def check(self):
        """Raise ``NRXError`` (code NRX_ERR_FUSED) if a one-launch forward since the last check
        reported an error -- its LLRs are invalid (include/nrx.h nrx_fused_status).  Blocking
        (synchronises the stream of the last forward); clears the counters."""
        st = (ctypes.c_int32 * 3)()
        _lib.check(self._lib.nrx_fused_status(self._h, st, 1))

    def fused_config(self, enable=None, spin_limit: Optional[int] = None, inject_err: Optional[int] = None):
        """One-launch forward control (include/nrx.h nrx_fused_config): ``enable`` False / 0,
        True / 1 (where it is the faster schedule), "force" / 2 (every shape it applies to), None:
        unchanged; the dependency-wait bound (0: default) and error bits to inject (test hook),
        None: unchanged."""
        if enable is None:
            en = -1
        elif enable == "force" or (isinstance(enable, int) and not isinstance(enable, bool) and enable == 2):
            en = 2
        elif isinstance(enable, (bool, int)) and int(enable) in (0, 1):
            en = int(enable)
        else:
            raise ValueError(f"enable must be False/0, True/1, 'force'/2 or None, got {enable!r}")
        sl = -1 if spin_limit is None else max(int(spin_limit), 0)
        ie = -1 if inject_err is None else int(inject_err)
        _lib.check(self._lib.nrx_fused_config(self._h, en, sl, ie))

    def update_schedule(self, rr=None):
        """Stage schedule of the three-launch f16 forward (include/nrx.h nrx_update_schedule): a
        mask -- bits 0 / 1 run the aggregation / readout update stages as the register-resident
        16-row launch (k_update_rr), bits 2 / 3 as the whole-column launch (k_update_col, taken
        over the RR bit), bit 4 runs StateInit as k_init_col, bit 5 the whole forward as the
        one-launch column forward k_fwd_col -- each where it applies (the strip kernels elsewhere;
        outputs are bit-identical either way); True = 3, False = 0 (strip kernels everywhere),
        None = unchanged."""
        m = -1 if rr is None else 3 if rr is True else 0 if rr is False else int(rr)
        _lib.check(self._lib.nrx_update_schedule(self._h, m))

    def profile_read(self):
        """{kernel: (launches, total_ms)} since the last profile(True)."""
        out = {}
        for k, name in enumerate(_lib.KERNELS):
            n, ms = ctypes.c_int64(), ctypes.c_double()
            _lib.check(self._lib.nrx_profile_read(self._h, k, ctypes.byref(n), ctypes.byref(ms)))
            out[name] = (n.value, ms.value)
        return out

    # -------------------------------------------------------------- helpers
    def flops_per_re_user(self, num_it: Optional[int] = None) -> float:
        return float(self._lib.nrx_flops_per_re_user(ctypes.byref(self._desc),
                                                     num_it or self.spec.num_it))

    def workspace_bytes(self, batch, num_tx, num_subcarriers, precision="f16", y_layout="cgnn") -> int:
        shape = _lib.nrx_shape(batch, num_tx, num_subcarriers, NUM_SYMBOLS)
        out = ctypes.c_size_t()
        _lib.check(self._lib.nrx_workspace_size_ex(self._h, ctypes.byref(shape), _lib.PRECISIONS[precision],
                                                   _lib.Y_LAYOUTS[y_layout], ctypes.byref(out)))
        return out.value

    def _workspace(self, nbytes: int):
        torch = _torch()
        ws = self._ws.get("buf")
        if ws is None or ws.numel() < nbytes:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{self.device}")
            self._ws["buf"] = ws
        return ws

    def alloc_outputs(self, batch, num_tx, num_subcarriers, want_h=True):
        torch = _torch()
        sp = self.spec
        dev = f"cuda:{self.device}"
        llr = torch.empty((sp.num_llr_heads, batch, num_tx, num_subcarriers, NUM_SYMBOLS, sp.bits_max),
                          dtype=torch.float32, device=dev)
        h = (torch.empty((batch, num_tx, num_subcarriers, NUM_SYMBOLS, 2 * sp.num_rx_ant),
                         dtype=torch.float32, device=dev) if want_h else None)
        return llr, h

    # -------------------------------------------------------------- forward
    def forward(self, y, pe, h_hat, active, mcs_mask=None, num_it=None, precision="f16",
                out=None, want_h=True, stream=None, y_layout="cgnn", y_imag=None):
        """All inputs are float32 CUDA tensors in the CGNN layout (see include/nrx.h), except
        ``y`` with ``y_layout``: "sionna" = the complex64 resource grid ``[B,1,A,14,F]``
        CGNNOFDM.forward receives, "split" = ``y`` / ``y_imag`` = rx_slot_real / imag
        ``[B,F,14,A]`` (NeuralReceiverONNX); the layout change runs in libnrx
        (``nrx_forward_ex``).  Returns ``(llr [H,B,U,F,T,bits_max], h_ref [B,U,F,T,2A] or
        None)``."""
        torch = _torch()
        sp = self.spec
        A = sp.num_rx_ant
        if y_layout == "cgnn":
            if y.dim() != 4 or y.shape[2] != NUM_SYMBOLS or y.shape[3] != 2 * A:
                raise ValueError(f"y must be [B,F,14,{2 * A}], got {tuple(y.shape)}")
            B, F = y.shape[0], y.shape[1]
        elif y_layout == "sionna":
            if y.is_complex():
                if y.dtype != torch.complex64:
                    raise ValueError("the resource grid must be complex64")
                y = torch.view_as_real(y.contiguous())
            if y.dim() != 6 or y.shape[1] != 1 or y.shape[2] != A or y.shape[3] != NUM_SYMBOLS or y.shape[5] != 2:
                raise ValueError(f"resource grid must be [B,1,{A},14,F] complex, got {tuple(y.shape)}")
            B, F = y.shape[0], y.shape[4]
        elif y_layout == "split":
            if y.dim() != 4 or y.shape[2] != NUM_SYMBOLS or y.shape[3] != A or y_imag is None or \
                    tuple(y_imag.shape) != tuple(y.shape):
                raise ValueError(f"rx_slot_real / rx_slot_imag must be [B,F,14,{A}]")
            B, F = y.shape[0], y.shape[1]
        else:
            raise ValueError(f"unknown y layout {y_layout}")
        U = active.shape[1]
        if tuple(pe.shape) != (U, F, NUM_SYMBOLS, 2):
            if pe.shape[0] >= U and tuple(pe.shape[1:]) == (F, NUM_SYMBOLS, 2):
                pe = pe[:U]          # pe[:num_tx] (neural_rx.py:817)
            else:
                raise ValueError(f"pe must be [U,F,14,2], got {tuple(pe.shape)}")
        if h_hat is not None and tuple(h_hat.shape) != (B, U, F, NUM_SYMBOLS, 2 * A):
            raise ValueError(f"h_hat has shape {tuple(h_hat.shape)}")
        if mcs_mask is not None and tuple(mcs_mask.shape) != (B, U, sp.num_mcs):
            mcs_mask = mcs_mask.expand(B, U, sp.num_mcs)
        tensors = [y, pe, h_hat, active, mcs_mask, y_imag if y_layout == "split" else None]
        for t in tensors:
            if t is not None and (not t.is_cuda or t.dtype != torch.float32):
                raise ValueError("inputs must be float32 CUDA tensors")
        y, pe, h_hat, active, mcs_mask, y_im = [None if t is None else t.contiguous() for t in tensors]
        if out is None:
            out = self.alloc_outputs(B, U, F, want_h)
        llr, h_ref = out
        prec = _lib.PRECISIONS[precision]
        nbytes = self.workspace_bytes(B, U, F, precision, y_layout)
        ws = self._workspace(nbytes)
        io = _lib.nrx_io()
        io.shape = _lib.nrx_shape(B, U, F, NUM_SYMBOLS)
        io.num_it = sp.num_it if num_it is None else num_it
        io.precision = prec
        io.y, io.pe, io.active, io.llr = y.data_ptr(), pe.data_ptr(), active.data_ptr(), llr.data_ptr()
        io.h_hat = h_hat.data_ptr() if h_hat is not None else None
        io.mcs_mask = mcs_mask.data_ptr() if mcs_mask is not None else None
        io.h_ref = h_ref.data_ptr() if h_ref is not None else None
        if stream is None:
            stream = torch.cuda.current_stream(y.device).cuda_stream
        _lib.check(self._lib.nrx_forward_ex(self._h, ctypes.byref(io), _lib.Y_LAYOUTS[y_layout],
                                            y_im.data_ptr() if y_im is not None else None, ws.data_ptr(),
                                            ws.numel(), stream))
        # keep inputs alive until the stream consumed them
        self._last_inputs = tensors
        return llr, h_ref

    # -------------------------------------------------------------- coded-bit layout
    def llr_demap(self, llr_head, bits, data_re, stream=None):
        """``llr_head [B,U,F,T,bits_stride]`` (one head of ``forward``'s output, Sionna sign)
        -> ``[B,U,n_data*bits]``: the data REs in resource-grid order (include/nrx.h
        nrx_llr_demap; ResourceGridDemapper + flatten of CGNNOFDM.forward, neural_rx.py:843-852)."""
        torch = _torch()
        if not llr_head.is_contiguous():
            raise ValueError("llr_head must be contiguous (a head slice of the forward output)")
        B, U, F, T, stride = llr_head.shape
        out = torch.empty((B, U, data_re.numel() * bits), dtype=torch.float32, device=llr_head.device)
        if stream is None:
            stream = torch.cuda.current_stream(llr_head.device).cuda_stream
        _lib.check(self._lib.nrx_llr_demap(llr_head.data_ptr(), B, U, F, T, stride, bits, data_re.data_ptr(),
                                           data_re.numel(), out.data_ptr(), stream))
        return out

    # -------------------------------------------------------------- Aerial contract
    def forward_aerial(self, y_real, y_imag, h_ls_real, h_ls_imag, dmrs_port_mask, dmrs_ofdm_pos,
                       dmrs_subcarrier_pos, num_it=None, precision="f16", want_h=True, stream=None):
        """NeuralReceiverONNX I/O on the GPU (include/nrx.h, nrx_forward_aerial).

        ``y_real/imag [B,F,T,A]``, ``h_ls_real/imag [B,Npil,U,A]`` (LS at the DMRS pilots,
        pilot p = (k * F/12 + prb) * npil + j), ``dmrs_port_mask [B,U]`` float,
        ``dmrs_ofdm_pos [U,nsym]`` / ``dmrs_subcarrier_pos [U,npil]`` int32 CUDA tensors.
        Returns ``(llr [B,bits,U,F,T], h_hat [B,U,F,T,2A] or None)`` with the Aerial sign."""
        torch = _torch()
        sp = self.spec
        B, F, T, A = y_real.shape
        U = dmrs_port_mask.shape[1]
        if T != NUM_SYMBOLS or A != sp.num_rx_ant:
            raise ValueError(f"y must be [B,F,14,{sp.num_rx_ant}], got {tuple(y_real.shape)}")
        nsym, npil = dmrs_ofdm_pos.shape[1], dmrs_subcarrier_pos.shape[1]
        if h_ls_real.shape[1] != nsym * (F // 12) * npil or h_ls_real.shape[3] != A:
            raise ValueError(f"h_ls must be [B,{nsym * (F // 12) * npil},U,{A}], got {tuple(h_ls_real.shape)}")
        if h_ls_real.shape[2] != U:        # h_hat[:, 0, :, :num_tx] (neural_rx.py:1709)
            h_ls_real, h_ls_imag = h_ls_real[:, :, :U], h_ls_imag[:, :, :U]
        f32 = [y_real, y_imag, h_ls_real, h_ls_imag, dmrs_port_mask]
        for t in f32:
            if not t.is_cuda or t.dtype != torch.float32:
                raise ValueError("y / h_ls / dmrs_port_mask must be float32 CUDA tensors")
        pos = [dmrs_ofdm_pos[:U], dmrs_subcarrier_pos[:U]]
        for t in pos:
            if not t.is_cuda or t.dtype != torch.int32:
                raise ValueError("dmrs positions must be int32 CUDA tensors")
        y_real, y_imag, h_ls_real, h_ls_imag, mask = [t.contiguous() for t in f32]
        ofdm, scp = [t.contiguous() for t in pos]
        bits = sp.bits_max if sp.masking else sp.bits[0]
        llr = torch.empty((B, bits, U, F, NUM_SYMBOLS), dtype=torch.float32, device=y_real.device)
        h = (torch.empty((B, U, F, NUM_SYMBOLS, 2 * A), dtype=torch.float32, device=y_real.device)
             if want_h else None)
        io = _lib.nrx_aerial_io()
        io.shape = _lib.nrx_shape(B, U, F, NUM_SYMBOLS)
        io.num_it = sp.num_it if num_it is None else num_it
        io.precision = _lib.PRECISIONS[precision]
        io.num_dmrs_symbols, io.num_dmrs_subcarriers = nsym, npil
        io.y_real, io.y_imag = y_real.data_ptr(), y_imag.data_ptr()
        io.h_ls_real, io.h_ls_imag = h_ls_real.data_ptr(), h_ls_imag.data_ptr()
        io.dmrs_port_mask = mask.data_ptr()
        io.dmrs_ofdm_pos, io.dmrs_subcarrier_pos = ofdm.data_ptr(), scp.data_ptr()
        io.llr = llr.data_ptr()
        io.h_hat = h.data_ptr() if h is not None else None
        nbytes = ctypes.c_size_t()
        _lib.check(self._lib.nrx_aerial_workspace_size(self._h, ctypes.byref(io), ctypes.byref(nbytes)))
        ws = self._workspace(nbytes.value)
        if stream is None:
            stream = torch.cuda.current_stream(y_real.device).cuda_stream
        _lib.check(self._lib.nrx_forward_aerial(self._h, ctypes.byref(io), ws.data_ptr(), ws.numel(), stream))
        self._last_inputs = [y_real, y_imag, h_ls_real, h_ls_imag, mask, ofdm, scp]
        return llr, h


class AerialReceiver:
    """Mirror of NeuralReceiverONNX (neural_rx.py:1717-1812): the TensorRT engine's feed
    dict (real_time_nrx.ipynb:792-844) in, ``(llr [B,bits,U,F,T], h_hat [B,U,F,T,2A])`` out,
    LLR = log p(b=0)/p(b=1).  Single MCS, as the ONNX export."""

    def __init__(self, config: str | NRXConfig = "nrx_rt", weight_list=None, device: int = 0,
                 precision: str = "f16", num_tx: Optional[int] = None, num_rx_ant: Optional[int] = None):
        self.cfg = get_config(config) if isinstance(config, str) else config
        self.spec = spec_from_config(self.cfg, num_rx_ant)
        if weight_list is None:
            weight_list = _weights.load(self.cfg.label)
        self.engine = CGNNEngine(self.spec, weight_list, device)
        self.precision = precision
        self._num_tx = num_tx or self.cfg.max_num_tx
        self._num_it = self.cfg.num_nrx_iter_eval

    @property
    def num_it(self):
        return self._num_it

    @num_it.setter
    def num_it(self, val):
        assert (val >= 1) and (val <= self.spec.num_it), "Invalid number of iterations"
        self._num_it = val

    def forward(self, inputs):
        (y_real, y_imag, h_hat_real, h_hat_imag, dmrs_port_mask, dmrs_ofdm_pos,
         dmrs_subcarrier_pos) = inputs
        U = self._num_tx
        return self.engine.forward_aerial(y_real, y_imag, h_hat_real, h_hat_imag, dmrs_port_mask[:, :U],
                                          dmrs_ofdm_pos, dmrs_subcarrier_pos, self._num_it, self.precision)

    __call__ = forward


def spec_for(config: str | NRXConfig, num_rx_ant: Optional[int] = None) -> ModelSpec:
    cfg = get_config(config) if isinstance(config, str) else config
    return spec_from_config(cfg, num_rx_ant)


class CGNN:
    """Reference-shaped core layer (neural_rx.py:407-595) backed by the engine."""

    def __init__(self, config: str | NRXConfig = "nrx_rt", weight_list=None, device: int = 0,
                 precision: str = "f16", num_rx_ant: Optional[int] = None):
        self.cfg = get_config(config) if isinstance(config, str) else config
        self.spec = spec_from_config(self.cfg, num_rx_ant)
        if weight_list is None:
            weight_list = _weights.load(self.cfg.label)
        self.engine = CGNNEngine(self.spec, weight_list, device)
        self.precision = precision
        self._num_it = self.cfg.num_nrx_iter_eval

    @property
    def num_it(self):
        return self._num_it

    @num_it.setter
    def num_it(self, val):
        assert (val >= 1) and (val <= self.spec.num_it), "Invalid number of iterations"
        self._num_it = val

    def forward(self, inputs, y_layout="cgnn", y_imag=None):
        """``inputs = [y, pe, h_hat, active_tx, mcs_ue_mask]`` -> ``(llrs, h_hats)`` with
        ``llrs[-1][m]`` = LLRs of MCS m ``[B,U,F,T,bits_m]`` and ``h_hats[-1]``."""
        y, pe, h_hat, active_tx, mcs_ue_mask = inputs
        llr, h = self.engine.forward(y, pe, h_hat, active_tx, mcs_ue_mask, self._num_it,
                                     self.precision, y_layout=y_layout, y_imag=y_imag)
        self.last_raw_llr = llr          # [H, B, U, F, T, bits_max] (for coded-bit demapping)
        sp = self.spec
        per_mcs = []
        for m, nb in enumerate(sp.bits):
            head = 0 if sp.masking else m
            per_mcs.append(llr[head, ..., :nb])
        return [per_mcs], [h]

    __call__ = forward

    def check(self):
        """Raise if a one-launch forward since the last check reported an error."""
        self.engine.check()


class NeuralReceiver:
    """Drop-in receiver: rx grid + PE + active DMRS ports (+ h_hat) -> LLRs."""

    def __init__(self, config: str | NRXConfig = "nrx_rt", weight_list=None, device: int = 0,
                 precision: str = "f16", num_rx_ant: Optional[int] = None,
                 cdm_groups: Optional[Sequence[int]] = None):
        cfg = get_config(config) if isinstance(config, str) else config
        if cfg.mask_pilots:
            # CGNNOFDM.forward zeroes y on the pilot REs of the resource-grid type grid when
            # mask_pilots is set (neural_rx.py:828-830).  Only the e2e configs set it, and
            # their models (learned constellation, no h_hat, d_s = 64) are out of scope.
            raise NotImplementedError("mask_pilots = True (e2e configs) is not supported by this engine")
        self.cgnn = CGNN(cfg, weight_list, device, precision, num_rx_ant)
        self.cfg = self.cgnn.cfg
        self.spec = self.cgnn.spec
        self.device = device
        self._cdm_groups = cdm_groups
        self._pe_cache = {}

    @property
    def num_it(self):
        return self.cgnn.num_it

    @num_it.setter
    def num_it(self, val):
        self.cgnn.num_it = val

    def check(self):
        """Raise ``NRXError`` if a one-launch forward since the last check reported an error
        (its outputs are invalid); blocking."""
        self.cgnn.check()

    def positional_encoding(self, num_tx: int, num_subcarriers: int):
        torch = _torch()
        key = (num_tx, num_subcarriers)
        if key not in self._pe_cache:
            groups = self._cdm_groups or user_cdm_groups(self.cfg, num_tx)
            pe = compute_pe(num_tx, num_subcarriers, dmrs_symbols(self.cfg), groups)
            self._pe_cache[key] = torch.from_numpy(pe).to(f"cuda:{self.device}")
        return self._pe_cache[key]

    def data_re(self, num_subcarriers: int):
        """Device int32 table of the data REs (t * F + f, resource-grid order)."""
        torch = _torch()
        key = ("re", num_subcarriers)
        if key not in self._pe_cache:
            self._pe_cache[key] = torch.from_numpy(data_re_indices(self.cfg, num_subcarriers)).to(
                f"cuda:{self.device}")
        return self._pe_cache[key]

    def _mcs_mask(self, mcs_arr_eval, B, U, device):
        """CGNNOFDM.forward's default mask: one_hot(mcs_arr_eval[0]) (neural_rx.py:817-820)."""
        torch = _torch()
        m = torch.zeros((B, U, self.spec.num_mcs), dtype=torch.float32, device=device)
        m[..., int(mcs_arr_eval[0])] = 1.0
        return m

    def __call__(self, rx_grid, pe=None, active_dmrs=None, h_hat=None, mcs_ue_mask=None,
                 num_it=None, layout: str = "sionna", return_h_hat: bool = False, demap: bool = False,
                 mcs_arr_eval: Optional[Sequence[int]] = None, all_mcs: bool = False):
        """``layout`` "sionna": rx_grid = y ``[B,1,A,14,F]`` complex (CGNNOFDM.forward);
        "aerial": rx_grid = (rx_slot_real, rx_slot_imag) ``[B,F,14,A]`` and LLRs returned as
        ``[B,bits,U,F,T]`` with the Aerial sign (NeuralReceiverONNX.forward); "cgnn": rx_grid
        is already ``[B,F,14,2A]``.

        ``mcs_arr_eval`` (CGNNOFDM.forward(inputs, mcs_arr_eval, mcs_ue_mask_eval)): the MCS
        indices to read out; without ``mcs_ue_mask`` the state-init mask is
        one_hot(mcs_arr_eval[0]).  With ``demap`` the output is the coded bits of the data
        REs ``[B,U,num_coded_bits]`` of head mcs_arr_eval[0] (the reference returns
        ``llrs[-1][0]``, neural_rx.py:881); ``all_mcs`` returns the list for every listed
        MCS, each demapped with its own head and bit count (neural_rx.py:843-852)."""
        torch = _torch()
        if num_it is not None:
            self.num_it = num_it
        y_imag = None
        if layout == "sionna":
            # CGNNOFDM.forward: y [B,1,A,T,F] complex -> [B,F,T,2A] (neural_rx.py:831-833),
            # done by libnrx (nrx_forward_ex, NRX_Y_SIONNA_RG)
            y, y_layout = rx_grid, "sionna"
            if y.dtype != torch.complex64:   # real or complex128 grids
                y = y.to(torch.complex64)
            B, F = y.shape[0], y.shape[4]
        elif layout == "aerial":
            # NeuralReceiverONNX.forward: (rx_slot_real, rx_slot_imag) [B,F,T,A]
            y, y_imag = rx_grid
            y, y_imag, y_layout = y.to(torch.float32), y_imag.to(torch.float32), "split"
            B, F = y.shape[0], y.shape[1]
        elif layout == "cgnn":
            y, y_layout = rx_grid, "cgnn"
            B, F = y.shape[0], y.shape[1]
        else:
            raise ValueError(f"unknown layout {layout}")
        dev = y.device
        if active_dmrs is None:
            active_dmrs = torch.ones((B, self.cfg.max_num_tx), dtype=torch.float32, device=dev)
        active = active_dmrs.to(torch.float32).contiguous()
        U = active.shape[1]
        if pe is None:
            pe = self.positional_encoding(U, F)
        if mcs_arr_eval is None:
            mcs_arr_eval = [0]
        for m in mcs_arr_eval:
            if not 0 <= int(m) < self.spec.num_mcs:
                raise ValueError(f"mcs index {m} outside 0..{self.spec.num_mcs - 1}")
        if mcs_ue_mask is None and self.spec.num_mcs > 1:
            mcs_ue_mask = self._mcs_mask(mcs_arr_eval, B, U, dev)
        llrs, h_hats = self.cgnn([y, pe, h_hat, active, mcs_ue_mask], y_layout=y_layout, y_imag=y_imag)
        h_ref = h_hats[-1]
        if demap:
            # CGNNOFDM.forward's output (neural_rx.py:843-858): per-user coded bits of the
            # data REs, [B, U, num_coded_bits], one entry per listed MCS with its own head
            raw = self.cgnn.last_raw_llr
            sp = self.spec
            outs = []
            for m in (mcs_arr_eval if all_mcs else mcs_arr_eval[:1]):
                head = 0 if sp.masking else int(m)
                outs.append(self.cgnn.engine.llr_demap(raw[head], sp.bits[int(m)], self.data_re(F)))
            llr = outs if all_mcs else outs[0]
            return (llr, h_ref) if return_h_hat else llr
        if all_mcs:
            llr = [llrs[-1][int(m)] for m in mcs_arr_eval]
        else:
            llr = llrs[-1][int(mcs_arr_eval[0])] if self.spec.num_mcs > 1 else llrs[-1][0]
        if layout == "aerial":
            neg = lambda t: -t.permute(0, 4, 1, 2, 3)   # [B,bits,U,F,T], LLR = log p0/p1
            llr = [neg(t) for t in llr] if all_mcs else neg(llr)
        return (llr, h_ref) if return_h_hat else llr
