"""Slot-generator restatement (oracle; TEST INFRASTRUCTURE ONLY).

CPU statement of the algorithm the GPU slot generator (``nrx_generate_slots``,
``neural_rx_amd/csrc/nrx_synth.hip``) implements -- SURVEY.md 8(f) f3, the stand-in for
the reference's transmitter + channel + LS chain ``E2E_Model.forward``
(utils/e2e_model.py:219-344) whose Sionna blocks cannot run here.  It follows the
reference where the reference is explicit:

* active DMRS ports: ``num_active`` ones among ``U`` ports, randomly permuted per slot
  (``E2E_Model._active_dmrs_mask``, e2e_model.py:187-193); inactive ports transmit
  zeros (``x = x * a_tx``, e2e_model.py:311-313);
* noise variance from Eb/N0 with the pilot-overhead correction of the torch port
  (e2e_model.py:323-332): ``ebno_db -= 10 log10(1 - pilots / REs)``, ``no = 10^(-ebno_db/10)``;
* Gray QAM (TS 38.211 5.1, Sionna's labelling) on data REs; DMRS type 1 QPSK x sqrt(2)
  on the user's CDM group (jumpstart_tutorial.ipynb:331-339), zeros on the other group;
* LS at the user's own pilots + Manhattan nearest-neighbour interpolation
  (NearestNeighborInterpolator, neural_rx.py:973-992; first minimum in the
  pilot order (subcarrier-major, then DMRS symbol), as ``argmin`` picks it).

and defines its own seeded pieces where Sionna's are unavailable: a counter-based
Philox4x32-10 RNG (Salmon et al., SC'11; pinned by the Random123 known-answer vectors in
tests/test_synth.py) so that every random draw is a pure function of (seed, global slot
index, stream, element) -- identical on CPU and GPU and independent of how slots are split
over launches or ranks -- and a tapped-delay-line channel (L taps, exponential power
delay profile, sum-of-sinusoids Doppler per tap) standing in for Sionna's UMi.

All arithmetic is float64; the float32 outputs are rounded once at the end (the GPU does
the same in f64, so outputs agree to an f32 ulp).  LS divides the float32 received
grid (what a receiver sees) by the f64 pilot symbol.
"""
from __future__ import annotations

import dataclasses
from typing import Optional, Sequence

import numpy as np

# Philox4x32-10 constants (Random123 philox.h)
_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = 0x9E3779B9
_W1 = 0xBB67AE85
_MASK = np.uint64(0xFFFFFFFF)

# Stream ids of the counter word c3 (shared with nrx_synth.hip)
STREAM_RE, STREAM_ACTIVE, STREAM_MCS, STREAM_DELAY, STREAM_TAP, STREAM_NOISE = range(6)

CP_FACTOR = 1.07      # OFDM symbol duration incl. normal cyclic prefix = 1.07 / scs
PDP_DECAY = 3.0       # exponential PDP time constant = max_delay / 3


def philox4x32(c0, c1, c2, c3, k0, k1, rounds: int = 10):
    """Vectorised Philox4x32-R; arguments are broadcastable uint32-valued arrays/ints.
    Returns four uint64 arrays holding 32-bit words."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & _MASK for c in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = int(k0) & 0xFFFFFFFF
    k1 = int(k1) & 0xFFFFFFFF
    for r in range(rounds):
        if r:
            k0 = (k0 + _W0) & 0xFFFFFFFF
            k1 = (k1 + _W1) & 0xFFFFFFFF
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
    return c0, c1, c2, c3


def draw(seed: int, slot, stream: int, idx):
    """The four words for (seed, global slot index, stream, element idx)."""
    slot = np.asarray(slot, dtype=np.int64).astype(np.uint64)
    return philox4x32(idx, slot & _MASK, slot >> np.uint64(32), stream,
                      seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)


def uniform(w):
    """(w + 0.5) * 2^-32 in (0, 1), float64."""
    return (w.astype(np.float64) + 0.5) * 2.0 ** -32


def box_muller(w0, w1):
    r = np.sqrt(-2.0 * np.log(uniform(w0)))
    th = 2.0 * np.pi * uniform(w1)
    return r * np.cos(th), r * np.sin(th)


def qam(bits: np.ndarray, m: int) -> np.ndarray:
    """Gray QAM of TS 38.211 5.1.3-5.1.5 (unit energy); bits [..., >= m]."""
    b = 1.0 - 2.0 * bits[..., :m].astype(np.float64)
    if m == 2:
        return (b[..., 0] + 1j * b[..., 1]) / np.sqrt(2.0)
    if m == 4:
        return (b[..., 0] * (2.0 - b[..., 2]) + 1j * b[..., 1] * (2.0 - b[..., 3])) / np.sqrt(10.0)
    if m == 6:
        return (b[..., 0] * (4.0 - b[..., 2] * (2.0 - b[..., 4]))
                + 1j * b[..., 1] * (4.0 - b[..., 3] * (2.0 - b[..., 5]))) / np.sqrt(42.0)
    raise ValueError(m)


def ebno_to_no(ebno_db: float, num_dmrs_symbols: int = 2, num_symbols: int = 14) -> float:
    """e2e_model.py:323-332 (rate-adjusted SNR, ``ebno = True`` in nrx_rt.cfg:13): all REs
    of the DMRS symbols are pilot REs (2 CDM groups without data)."""
    ebno_db = ebno_db - 10.0 * np.log10(1.0 - num_dmrs_symbols / num_symbols)
    return float(10.0 ** (-ebno_db / 10.0))


@dataclasses.dataclass
class GenSpec:
    batch: int
    num_tx: int
    num_subcarriers: int
    num_rx_ant: int
    dmrs_symbols: Sequence[int] = (2, 11)
    cdm_group: Sequence[int] = (0, 1)
    mcs_bits: Sequence[int] = (4,)
    mcs_of_user: Optional[Sequence[int]] = None     # per user, -1 = drawn per slot
    num_active: Optional[int] = None                # None = all ports
    num_taps: int = 6
    num_sinusoids: int = 4
    max_delay_s: float = 300e-9
    max_doppler_hz: float = 400.0
    subcarrier_spacing: float = 30e3
    no: float = 0.01
    seed: int = 1234
    slot_offset: int = 0
    num_symbols: int = 14

    @property
    def bits_max(self) -> int:
        return max(self.mcs_bits)


@dataclasses.dataclass
class GenOut:
    y: np.ndarray           # [B, F, T, 2A] f32
    h_hat: np.ndarray       # [B, U, F, T, 2A] f32
    h: np.ndarray           # [B, U, F, T, 2A] f32 (true channel)
    active: np.ndarray      # [B, U] f32
    mcs: np.ndarray         # [B, U] u8
    bits: np.ndarray        # [B, U, F, T, bits_max] u8
    x: np.ndarray           # [B, U, F, T] c128 transmitted grid (after the active mask)
    y_c: np.ndarray         # [B, A, F, T] c128, unrounded


def nearest_pilot(num_subcarriers: int, dmrs_symbols: Sequence[int], cdm_group: int,
                  num_symbols: int = 14):
    """(fp[F,T], tp[F,T]): the first nearest own pilot of every RE, found by the general
    argmin over the pilot list (subcarrier-major, symbol-minor) -- NearestNeighborInterpolator
    semantics; the GPU uses a closed form for the same answer."""
    F, T = num_subcarriers, num_symbols
    pf = np.array([f for f in range(F) if f % 2 == cdm_group])
    pt = np.array(list(dmrs_symbols))
    pil_f, pil_t = np.meshgrid(pf, pt, indexing="ij")
    pil_f, pil_t = pil_f.ravel(), pil_t.ravel()
    ff, tt = np.meshgrid(np.arange(F), np.arange(T), indexing="ij")
    d = np.abs(ff[..., None] - pil_f) + np.abs(tt[..., None] - pil_t)
    nn = d.argmin(-1)
    return pil_f[nn], pil_t[nn]


def generate(s: GenSpec) -> GenOut:
    B, U, F, A, T = s.batch, s.num_tx, s.num_subcarriers, s.num_rx_ant, s.num_symbols
    L, NS, M = s.num_taps, s.num_sinusoids, len(s.mcs_bits)
    slots = s.slot_offset + np.arange(B, dtype=np.int64)
    dm = np.zeros(T, bool)
    dm[list(s.dmrs_symbols)] = True

    # active ports (e2e_model.py:187-193): Fisher-Yates over [1]*num_active + [0]*rest
    na = U if s.num_active is None else s.num_active
    w = np.stack(draw(s.seed, slots[:, None], STREAM_ACTIVE, np.arange(4)[None, :]), -1).reshape(B, 16)
    active = np.zeros((B, U), np.float32)
    for b in range(B):
        arr = [1 if i < na else 0 for i in range(U)]
        for i in range(U - 1, 0, -1):
            j = int(w[b, i] % np.uint64(i + 1))
            arr[i], arr[j] = arr[j], arr[i]
        active[b] = arr

    # MCS per (slot, user): fixed per user, or drawn (-1)
    mou = np.array(list(s.mcs_of_user) if s.mcs_of_user is not None else [0] * U)
    wm = draw(s.seed, slots[:, None], STREAM_MCS, np.arange(U)[None, :])[0]
    mcs = np.where(mou[None, :] >= 0, mou[None, :], (wm % np.uint64(M)).astype(np.int64)).astype(np.uint8)
    nbits = np.array(s.mcs_bits)[mcs]                                   # [B,U]

    # transmitted grid: one draw per (u, f, t); word 0 = data bits, word 1 = pilot bits
    idx = (np.arange(U)[:, None, None] * F + np.arange(F)[None, :, None]) * T + np.arange(T)[None, None, :]
    w0, w1, _, _ = draw(s.seed, slots[:, None, None, None], STREAM_RE, idx[None])   # [B,U,F,T]
    kk = np.arange(s.bits_max, dtype=np.uint64)
    bits = ((w0[..., None] >> kk) & np.uint64(1)).astype(np.uint8)      # [B,U,F,T,bmax]
    keep = (np.arange(s.bits_max)[None, None, None, None, :] < nbits[:, :, None, None, None])
    keep = keep & ~dm[None, None, None, :, None]
    bits = (bits * keep).astype(np.uint8)
    x = np.zeros((B, U, F, T), np.complex128)
    for m_i, m in enumerate(s.mcs_bits):
        x = np.where((mcs == m_i)[:, :, None, None], qam(bits, m), x)
    x[:, :, :, dm] = 0
    pb = np.stack([w1 & np.uint64(1), (w1 >> np.uint64(1)) & np.uint64(1)], -1)
    pil = qam(pb.astype(np.uint8), 2) * np.sqrt(2.0)
    own = (np.arange(F)[None, :] % 2) == np.array(s.cdm_group)[:U, None]      # [U,F]
    pmask = own[None, :, :, None] & dm[None, None, None, :]
    x = np.where(pmask, pil, x)
    x = x * active[:, :, None, None]

    # channel: delays / PDP per (slot, user)
    didx = np.arange(U)[:, None] * L + np.arange(L)[None, :]
    dw = draw(s.seed, slots[:, None, None], STREAM_DELAY, didx[None])[0]
    tau = np.sort(uniform(dw) * s.max_delay_s, axis=-1)                 # [B,U,L]
    tau[..., 0] = 0.0
    pdp = np.exp(-tau / (s.max_delay_s / PDP_DECAY + 1e-12))
    pdp = pdp / pdp.sum(-1, keepdims=True)
    tidx = (((np.arange(U)[:, None, None, None] * A + np.arange(A)[None, :, None, None]) * L
             + np.arange(L)[None, None, :, None]) * NS + np.arange(NS)[None, None, None, :])
    t0, t1, t2, _ = draw(s.seed, slots[:, None, None, None, None], STREAM_TAP, tidx[None])  # [B,U,A,L,NS]
    nre, nim = box_muller(t0, t1)
    g0 = (nre + 1j * nim) / np.sqrt(2.0 * NS)
    fd = s.max_doppler_hz * np.cos(2.0 * np.pi * uniform(t2))
    tsym = CP_FACTOR / s.subcarrier_spacing
    tt = np.arange(T) * tsym
    ph = 2.0 * np.pi * (fd[..., None] * tt)                            # [B,U,A,L,NS,T]
    gt = (g0[..., None] * (np.cos(ph) + 1j * np.sin(ph))).sum(-2)       # [B,U,A,L,T]
    gt = gt * np.sqrt(pdp)[:, :, None, :, None]
    fa = 2.0 * np.pi * ((np.arange(F)[None, None, None, :] * s.subcarrier_spacing) * tau[..., None])  # [B,U,L,F]
    e = np.cos(fa) - 1j * np.sin(fa)
    h = np.einsum("bualt,bulf->buaft", gt, e)                           # [B,U,A,F,T]

    nidx = (np.arange(A)[:, None, None] * F + np.arange(F)[None, :, None]) * T + np.arange(T)[None, None, :]
    n0, n1, _, _ = draw(s.seed, slots[:, None, None, None], STREAM_NOISE, nidx[None])      # [B,A,F,T]
    zr, zi = box_muller(n0, n1)
    sd = np.sqrt(s.no / 2.0)
    y_c = np.einsum("buaft,buft->baft", h, x) + sd * (zr + 1j * zi)

    def to_ch(z):   # [..., A, F, T] -> [..., F, T, 2A] f32
        z = np.moveaxis(z, -3, -1)
        return np.concatenate([z.real, z.imag], axis=-1).astype(np.float32)

    y = to_ch(y_c)
    yr = y[..., :A].astype(np.float64) + 1j * y[..., A:].astype(np.float64)    # [B,F,T,A] as received
    h_hat = np.zeros((B, U, F, T, A), np.complex128)
    for u in range(U):
        fp, tp = nearest_pilot(F, s.dmrs_symbols, s.cdm_group[u], T)
        xp = x[:, u, fp, tp]                                            # [B,F,T]
        yp = yr[:, fp, tp, :]                                           # [B,F,T,A]
        safe = np.where(xp != 0, xp, 1.0)
        h_hat[:, u] = np.where((xp != 0)[..., None], yp / safe[..., None], 0)
    h_hat_ch = np.concatenate([h_hat.real, h_hat.imag], axis=-1).astype(np.float32)
    return GenOut(y=y, h_hat=h_hat_ch, h=to_ch(h), active=active, mcs=mcs, bits=bits, x=x, y_c=y_c)


def count_errors(llr: np.ndarray, bits: np.ndarray, mcs: np.ndarray, mcs_bits: Sequence[int],
                 active: np.ndarray, dmrs_symbols: Sequence[int]) -> np.ndarray:
    """Per-user uncoded counters [U, 4] = (bit errors, bits, block errors, blocks) over
    active (slot, user) pairs and data REs; LLR > 0 decides 1 (Sionna sign); a block is
    one (slot, user) grid.  ``llr`` [H, B, U, F, T, bs]: head = mcs if H > 1 else 0."""
    H, B, U, F, T, _ = llr.shape
    dm = np.ones(T, bool)
    dm[list(dmrs_symbols)] = False
    out = np.zeros((U, 4), np.int64)
    for b in range(B):
        for u in range(U):
            if active[b, u] <= 0:
                continue
            m = int(mcs[b, u])
            nb = mcs_bits[m]
            hd = llr[m if H > 1 else 0, b, u][:, dm, :nb] > 0
            ref = bits[b, u][:, dm, :nb].astype(bool)
            e = int((hd != ref).sum())
            out[u] += (e, hd.size, int(e > 0), 1)
    return out
