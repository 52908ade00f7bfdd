"""Seeded synthetic PUSCH slot generator (host, numpy).

Stands in for the reference's Sionna transmitter + channel + LS estimator chain
(``E2E_Model.forward`` e2e_model.py:272-344; ``DataGeneratorAerial.call``
onnx_utils.py:289-410), which cannot run here (Sionna/TF are not installed).  It
produces inputs with the statistics the trained CGNN expects, as described in
SURVEY.md section 8(d):

* Gray QAM (TS 38.211 section 5.1, Sionna's labelling) on data REs;
* DMRS type 1 on symbols 2/11: QPSK x sqrt(2) on the user's CDM-group subcarriers,
  zeros on the other group (2 CDM groups without data, so DMRS symbols carry no
  data; jumpstart_tutorial.ipynb:331-339);
* a tapped-delay-line "UMi proxy" channel (<= 300 ns, exponential PDP, Doppler up
  to ``max_doppler_hz``), i.i.d. over rx antennas; codebook precoding
  ``w = [1, 1]/sqrt(2)`` folds into an effective per-user channel;
* AWGN at a per-RE SNR; ``h_hat`` = LS at the user's own pilots + Manhattan
  nearest-neighbour interpolation (NearestNeighborInterpolator semantics,
  neural_rx.py:973-992).

All arrays use the CGNN layout: ``y [B,F,T,2A]`` with channels
``[Re a0..a(A-1), Im a0..a(A-1)]`` (neural_rx copy_pytorch.py:733-735).
"""
from __future__ import annotations

import dataclasses
from typing import Optional, Sequence

import numpy as np

SUBCARRIER_SPACING = 30e3
SYMBOL_TIME = (1.0 / SUBCARRIER_SPACING) * (1 + 0.07)  # incl. normal CP


def qam_map(bits: np.ndarray) -> np.ndarray:
    """Map bits [..., m] to unit-energy Gray QAM (TS 38.211 5.1.3-5.1.5)."""
    m = bits.shape[-1]
    b = 1 - 2 * bits.astype(np.float64)
    if m == 2:
        return (b[..., 0] + 1j * b[..., 1]) / np.sqrt(2)
    if m == 4:
        re = b[..., 0] * (2 - b[..., 2])
        im = b[..., 1] * (2 - b[..., 3])
        return (re + 1j * im) / np.sqrt(10)
    if m == 6:
        re = b[..., 0] * (4 - b[..., 2] * (2 - b[..., 4]))
        im = b[..., 1] * (4 - b[..., 3] * (2 - b[..., 5]))
        return (re + 1j * im) / np.sqrt(42)
    raise ValueError(f"unsupported modulation order {m}")


@dataclasses.dataclass
class Slots:
    y: np.ndarray          # [B, F, T, 2A] float32
    h_hat: np.ndarray      # [B, U, F, T, 2A] float32 (LS + NN interpolation)
    h: np.ndarray          # [B, U, F, T, 2A] float32 (true effective channel)
    bits: np.ndarray       # [B, U, F, T, bits] uint8 (zeros on DMRS symbols)
    data_mask: np.ndarray  # [T] bool, data-carrying symbols
    active: np.ndarray     # [B, U] float32
    y_complex: np.ndarray  # [B, 1, A, T, F] complex64 (Sionna layout)
    x: Optional[np.ndarray] = None   # [B, U, F, T] complex64 transmitted grid (data + DMRS)


def _tdl(rng, batch, users, ants, f, t, max_delay_s, max_doppler_hz, taps=6):
    delays = np.sort(rng.uniform(0, max_delay_s, size=(batch, users, 1, taps)), axis=-1)
    delays[..., 0] = 0.0
    pdp = np.exp(-delays / (max_delay_s / 3 + 1e-12))
    pdp /= pdp.sum(-1, keepdims=True)
    # per-tap time evolution: sum of 4 sinusoids (Jakes-like)
    nsin = 4
    g0 = (rng.standard_normal((batch, users, ants, taps, nsin))
          + 1j * rng.standard_normal((batch, users, ants, taps, nsin))) / np.sqrt(2 * nsin)
    fd = max_doppler_hz * np.cos(rng.uniform(0, 2 * np.pi, size=(batch, users, ants, taps, nsin)))
    tt = np.arange(t) * SYMBOL_TIME
    g = (g0[..., None] * np.exp(2j * np.pi * fd[..., None] * tt)).sum(-2)   # [B,U,A,L,T]
    g = g * np.sqrt(pdp)[:, :, :, :, None]
    ff = np.arange(f) * SUBCARRIER_SPACING
    ph = np.exp(-2j * np.pi * ff[None, None, None, None, :] * delays[..., None])  # [B,U,1,L,F]
    h = np.einsum("bualt,bualf->buaft", g, np.broadcast_to(ph, (batch, users, ants, taps, f)))
    return h  # [B, U, A, F, T]


def generate(batch: int, num_users: int, num_prbs: int, num_rx_ant: int,
             bits_per_user: Sequence[int], cdm_groups: Sequence[int],
             dmrs_symbols: Sequence[int] = (2, 11), snr_db: float = 20.0,
             seed: int = 1234, active: Optional[np.ndarray] = None,
             max_delay_s: float = 300e-9, max_doppler_hz: float = 400.0) -> Slots:
    rng = np.random.default_rng(seed)
    f = 12 * num_prbs
    t = 14
    a = num_rx_ant
    data_mask = np.ones(t, bool)
    data_mask[list(dmrs_symbols)] = False
    bmax = max(bits_per_user)
    bits = np.zeros((batch, num_users, f, t, bmax), np.uint8)
    x = np.zeros((batch, num_users, f, t), np.complex128)
    for u in range(num_users):
        m = bits_per_user[u]
        bu = rng.integers(0, 2, size=(batch, f, t, m), dtype=np.uint8)
        bu[:, :, ~data_mask] = 0
        bits[:, u, :, :, :m] = bu
        x[:, u] = np.where(data_mask[None, None, :], qam_map(bu), 0)
        pil = qam_map(rng.integers(0, 2, size=(batch, f, len(dmrs_symbols), 2))) * np.sqrt(2)
        gmask = (np.arange(f) % 2 == cdm_groups[u])
        for k, ts in enumerate(dmrs_symbols):
            x[:, u, :, ts] = np.where(gmask[None, :], pil[:, :, k], 0)
    if active is None:
        active = np.ones((batch, num_users), np.float32)
    x = x * active[:, :, None, None]
    h = _tdl(rng, batch, num_users, a, f, t, max_delay_s, max_doppler_hz)  # [B,U,A,F,T]
    no = 10 ** (-snr_db / 10)
    noise = (rng.standard_normal((batch, a, f, t)) + 1j * rng.standard_normal((batch, a, f, t))) * np.sqrt(no / 2)
    yc = np.einsum("buaft,buft->baft", h, x) + noise                      # [B,A,F,T]
    # LS at own pilots + Manhattan-NN interpolation
    h_hat = np.zeros((batch, num_users, a, f, t), np.complex128)
    ff, tt = np.meshgrid(np.arange(f), np.arange(t), indexing="ij")
    for u in range(num_users):
        pf = np.array([p for p in range(f) if p % 2 == cdm_groups[u]])
        pts = np.array(list(dmrs_symbols))
        pil_f, pil_t = np.meshgrid(pf, pts, indexing="ij")
        pil_f, pil_t = pil_f.ravel(), pil_t.ravel()
        xp = x[:, u][:, pil_f, pil_t]                                       # [B,P]
        safe = np.where(np.abs(xp) > 0, xp, 1.0)
        ls = np.where(np.abs(xp)[:, None, :] > 0, yc[:, :, pil_f, pil_t] / safe[:, None, :], 0)  # [B,A,P]
        d = np.abs(ff[..., None] - pil_f) + np.abs(tt[..., None] - pil_t)        # [F,T,P]
        nn = d.argmin(-1)
        h_hat[:, u] = ls[:, :, nn]
    def to_ch(z):  # [..., A, F, T] complex -> [..., F, T, 2A] float32
        z = np.moveaxis(z, -3, -1)
        return np.concatenate([z.real, z.imag], axis=-1).astype(np.float32)
    y = to_ch(yc)
    return Slots(y=y, h_hat=to_ch(h_hat), h=to_ch(h), bits=bits, data_mask=data_mask,
                 active=active.astype(np.float32),
                 y_complex=np.transpose(yc, (0, 1, 3, 2))[:, None].astype(np.complex64),
                 x=x.astype(np.complex64))


def aerial_ls_pilots(y_complex_bfta, x_pilot_bupf, cdm_groups, dmrs_symbols, num_prbs):
    """LS estimates at each user's DMRS REs in the Aerial pilot order
    ``[B, Npil, U, A]`` (real, imag), Npil = nsym * nprb * 6.  ``y_complex_bfta``
    [B, F, T, A], ``x_pilot_bupf`` [B, U, F, T] transmitted symbols."""
    B, F, T, A = y_complex_bfta.shape
    U = len(cdm_groups)
    nsym = len(dmrs_symbols)
    out = np.zeros((B, nsym * num_prbs * 6, U, A), np.complex128)
    for u, g in enumerate(cdm_groups):
        for k, ts in enumerate(dmrs_symbols):
            for prb in range(num_prbs):
                for j in range(6):
                    f = prb * 12 + g + 2 * j
                    x = x_pilot_bupf[:, u, f, ts]
                    safe = np.where(np.abs(x) > 0, x, 1.0)
                    ls = np.where(np.abs(x)[:, None] > 0, y_complex_bfta[:, f, ts, :] / safe[:, None], 0)
                    out[:, (k * num_prbs + prb) * 6 + j, u, :] = ls
    return out.real.astype(np.float32), out.imag.astype(np.float32)


def hard_bits(llr: np.ndarray) -> np.ndarray:
    """Sionna convention: LLR = log(p1/p0), so LLR > 0 decides bit 1."""
    return (llr > 0).astype(np.uint8)


def uncoded_ber(llr: np.ndarray, slots: Slots, user: int, bits: int) -> float:
    dm = slots.data_mask
    est = hard_bits(llr[:, user][:, :, dm, :bits])
    ref = slots.bits[:, user][:, :, dm, :bits]
    act = slots.active[:, user] > 0
    if not act.any():
        return float("nan")
    return float((est[act] != ref[act]).mean())
