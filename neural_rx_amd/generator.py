"""Seeded PUSCH slot generator and uncoded error counters on the GPU.

Mirrors the data side of the reference's ``E2E_Model.forward``
(utils/e2e_model.py:219-344): random active DMRS ports (``_active_dmrs_mask``, 187-193),
bits -> Gray QAM on a DMRS type-1 resource grid, channel + AWGN at an Eb/N0-derived noise
variance (323-332), LS channel estimate -> the CGNN's inputs; and the counting side of
``sim_ber`` with ``_mask_active_dmrs`` (195-209).  Sionna's UMi channel and LDPC chain
are not available here; the generator's channel is the seeded tapped-delay line stated in
``oracle/synth_ref.py`` and the counters are uncoded (hard decisions on the LLRs).

Everything runs through ``libnrx.so`` (``nrx_generate_slots`` / ``nrx_count_errors``,
include/nrx.h); torch tensors are only device containers.
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Optional, Sequence

import numpy as np

from . import _lib
from .config import NRXConfig, dmrs_symbols, get_config, user_cdm_groups

NUM_SYMBOLS = 14


def _torch():
    import torch
    return torch


def ebno_to_no(ebno_db: float, num_dmrs_symbols: int = 2, num_symbols: int = NUM_SYMBOLS) -> float:
    """Rate-adjusted SNR of the torch E2E model (e2e_model.py:323-332, ``ebno = True`` in
    nrx_rt.cfg:13): ``ebno_db -= 10 log10(1 - pilots / REs)``; ``no = 10^(-ebno_db / 10)``.
    With two CDM groups without data every RE of a DMRS symbol is a pilot RE."""
    ebno_db = ebno_db - 10.0 * np.log10(1.0 - num_dmrs_symbols / num_symbols)
    return float(10.0 ** (-ebno_db / 10.0))


@dataclasses.dataclass
class GenParams:
    """Everything that defines a batch of generated slots (besides ``no``/offset)."""
    num_tx: int
    num_subcarriers: int
    num_rx_ant: int
    dmrs_symbols: Sequence[int] = (2, 11)
    cdm_group: Sequence[int] = (0, 1)
    mcs_bits: Sequence[int] = (4,)
    mcs_of_user: Optional[Sequence[int]] = None    # per port; -1 = drawn per slot
    num_active: Optional[int] = None               # None = all ports active
    num_taps: int = 6
    num_sinusoids: int = 4
    max_delay_s: float = 300e-9
    max_doppler_hz: float = 400.0
    subcarrier_spacing: float = 30e3
    seed: int = 1234

    @classmethod
    def from_config(cls, cfg: NRXConfig | str, num_tx: Optional[int] = None, num_prbs: Optional[int] = None,
                    num_rx_ant: Optional[int] = None, var_mcs: bool = False, **kw) -> "GenParams":
        """Generator parameters for a reference config: its DMRS symbols and ports
        (config.dmrs_symbols / user_cdm_groups), its MCS list (``mcs_index``; with
        ``var_mcs`` the MCS of each (slot, user) is drawn, as the var-MCS evaluation's
        random ``mcs_ue_mask``), its PRBs and antennas."""
        if isinstance(cfg, str):
            cfg = get_config(cfg)
        u = num_tx or cfg.max_num_tx
        return cls(num_tx=u, num_subcarriers=12 * (num_prbs or cfg.n_size_bwp),
                   num_rx_ant=num_rx_ant or cfg.num_rx_antennas, dmrs_symbols=dmrs_symbols(cfg),
                   cdm_group=user_cdm_groups(cfg, u), mcs_bits=cfg.bits_per_head,
                   mcs_of_user=[-1] * u if var_mcs else [0] * u, **kw)

    @property
    def bits_max(self) -> int:
        return max(self.mcs_bits)

    def desc(self, batch: int, no: float, slot_offset: int = 0) -> _lib.nrx_gen_desc:
        d = _lib.nrx_gen_desc()
        d.batch, d.num_tx, d.num_subcarriers, d.num_symbols = batch, self.num_tx, self.num_subcarriers, NUM_SYMBOLS
        d.num_rx_ant = self.num_rx_ant
        d.num_dmrs_symbols = len(self.dmrs_symbols)
        mask = 0
        for k, t in enumerate(self.dmrs_symbols):
            d.dmrs_symbols[k] = t
            mask |= 1 << t
        d.dmrs_symbol_mask = mask
        for u in range(self.num_tx):
            d.cdm_group[u] = self.cdm_group[u]
            d.mcs_of_user[u] = self.mcs_of_user[u] if self.mcs_of_user is not None else 0
        d.num_mcs = len(self.mcs_bits)
        for m, b in enumerate(self.mcs_bits):
            d.mcs_bits[m] = b
        d.num_active = self.num_tx if self.num_active is None else self.num_active
        d.num_taps, d.num_sinusoids = self.num_taps, self.num_sinusoids
        d.max_delay_s, d.max_doppler_hz = self.max_delay_s, self.max_doppler_hz
        d.subcarrier_spacing, d.no = self.subcarrier_spacing, no
        d.seed, d.slot_offset = self.seed, slot_offset
        return d


@dataclasses.dataclass
class SlotBatch:
    """Device tensors of one generated batch (CGNN layout, include/nrx.h)."""
    y: "object"            # [B, F, T, 2A] f32
    h_hat: "object"        # [B, U, F, T, 2A] f32
    active: "object"       # [B, U] f32
    mcs_mask: "object"     # [B, U, M] f32
    mcs: "object"          # [B, U] u8
    bits: "object"         # [B, U, F, T, bits_max] u8
    h: "object" = None     # [B, U, F, T, 2A] f32 (true channel) or None
    y_real: "object" = None
    y_imag: "object" = None
    h_ls_real: "object" = None
    h_ls_imag: "object" = None


class SlotGenerator:
    """``gen(batch, no, slot_offset) -> SlotBatch`` on one GPU.  Slot ``slot_offset + b``
    is the same slot whichever call, rank or batch split generates it."""

    def __init__(self, params: GenParams, device: int = 0, want_h: bool = False, aerial: bool = False):
        self.p = params
        self.device = device
        self.want_h = want_h
        self.aerial = aerial
        self._lib = _lib.load()
        self._ws = None
        self._bufs = {}

    def workspace_bytes(self, batch: int) -> int:
        n = ctypes.c_size_t()
        d = self.p.desc(batch, 0.0)
        _lib.check(self._lib.nrx_gen_workspace_size(ctypes.byref(d), ctypes.byref(n)))
        return n.value

    def _alloc(self, batch: int) -> SlotBatch:
        torch = _torch()
        key = batch
        if key in self._bufs:
            return self._bufs[key]
        p, dev = self.p, f"cuda:{self.device}"
        U, F, A, M = p.num_tx, p.num_subcarriers, p.num_rx_ant, len(p.mcs_bits)
        f32 = dict(dtype=torch.float32, device=dev)
        sb = SlotBatch(
            y=torch.empty((batch, F, NUM_SYMBOLS, 2 * A), **f32),
            h_hat=torch.empty((batch, U, F, NUM_SYMBOLS, 2 * A), **f32),
            active=torch.empty((batch, U), **f32),
            mcs_mask=torch.empty((batch, U, M), **f32),
            mcs=torch.empty((batch, U), dtype=torch.uint8, device=dev),
            bits=torch.empty((batch, U, F, NUM_SYMBOLS, p.bits_max), dtype=torch.uint8, device=dev),
            h=torch.empty((batch, U, F, NUM_SYMBOLS, 2 * A), **f32) if self.want_h else None)
        if self.aerial:
            npil = len(p.dmrs_symbols) * (F // 12) * 6
            sb.y_real = torch.empty((batch, F, NUM_SYMBOLS, A), **f32)
            sb.y_imag = torch.empty_like(sb.y_real)
            sb.h_ls_real = torch.empty((batch, npil, U, A), **f32)
            sb.h_ls_imag = torch.empty_like(sb.h_ls_real)
        self._bufs = {key: sb}
        return sb

    def __call__(self, batch: int, no: float, slot_offset: int = 0, stream=None, out: Optional[SlotBatch] = None
                 ) -> SlotBatch:
        torch = _torch()
        sb = out if out is not None else self._alloc(batch)
        nbytes = self.workspace_bytes(batch)
        if self._ws is None or self._ws.numel() < nbytes:
            self._ws = torch.empty(nbytes, dtype=torch.uint8, device=f"cuda:{self.device}")
        d = self.p.desc(batch, no, slot_offset)
        o = _lib.nrx_gen_out()
        ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
        o.y, o.h_hat, o.h, o.active = ptr(sb.y), ptr(sb.h_hat), ptr(sb.h), ptr(sb.active)
        o.mcs_mask, o.mcs, o.bits, o.bits_stride = ptr(sb.mcs_mask), ptr(sb.mcs), ptr(sb.bits), self.p.bits_max
        o.y_real, o.y_imag = ptr(sb.y_real), ptr(sb.y_imag)
        o.h_ls_real, o.h_ls_imag = ptr(sb.h_ls_real), ptr(sb.h_ls_imag)
        if stream is None:
            stream = torch.cuda.current_stream(sb.y.device).cuda_stream
        _lib.check(self._lib.nrx_generate_slots(ctypes.byref(d), ctypes.byref(o), self._ws.data_ptr(),
                                                self._ws.numel(), stream))
        return sb


def count_errors(llr, bits, active, mcs, mcs_bits: Sequence[int], dmrs_syms: Sequence[int], counts=None,
                 stream=None):
    """Accumulate per-user uncoded counters ``counts [U, 4]`` int64 (bit errors, bits,
    block errors, blocks) on the device (include/nrx.h nrx_count_errors).  ``llr`` is the
    engine output ``[H, B, U, F, T, bits_stride]``; head = MCS index if H > 1."""
    torch = _torch()
    lib = _lib.load()
    H, B, U, F, T, bs = llr.shape
    if counts is None:
        counts = torch.zeros((U, 4), dtype=torch.int64, device=llr.device)
    if tuple(bits.shape) != (B, U, F, T, bs):
        raise ValueError(f"bits must be {(B, U, F, T, bs)}, got {tuple(bits.shape)}")
    c = _lib.nrx_count_io()
    c.batch, c.num_tx, c.num_subcarriers, c.num_symbols = B, U, F, T
    c.num_heads, c.bits_stride, c.num_mcs = H, bs, len(mcs_bits)
    for m, b in enumerate(mcs_bits):
        c.mcs_bits[m] = b
    c.dmrs_symbol_mask = sum(1 << t for t in dmrs_syms)
    c.llr, c.bits, c.active, c.counts = llr.data_ptr(), bits.data_ptr(), active.data_ptr(), counts.data_ptr()
    c.mcs = mcs.data_ptr() if mcs is not None else None
    if stream is None:
        stream = torch.cuda.current_stream(llr.device).cuda_stream
    _lib.check(lib.nrx_count_errors(ctypes.byref(c), stream))
    return counts
