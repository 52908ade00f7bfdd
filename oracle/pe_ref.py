"""Positional encoding restatement (oracle; test infrastructure only).

Follows ``utils/onnx_utils.py:172-260`` (``DataGeneratorAerial.__init__``), which is
identical to ``precalculate_nnrx_indices`` (onnx_utils.py:580-667) and to the
commented torch copy (``neural_rx copy_pytorch.py:612-701``):

* per user, per RE: distance to the nearest of the user's non-zero pilots in time
  ``min_i |t_i - t|`` and, independently, in frequency ``min_i |f_i - f|``;
* time component normalised over the symbol axis (axis 1 of [tx, t, f]), frequency
  component over the subcarrier axis (axis 2), population ``np.std`` with
  ``where(std > 0)``;
* stacked [time, freq] and transposed to ``[num_tx, F, T, 2]``.

Pilot REs come from the DMRS description (type 1, single symbol): CDM group lambda
occupies subcarriers ``k = 4n + 2k' + lambda`` on the DMRS symbols.  Also restated:
the Aerial per-PRB variant ``NRPreprocessing._calculate_nn_indices``
(neural_rx.py:1631-1665, faithful copy 981-1035) with the TF ``meshgrid`` 'xy'
ordering and population std (SURVEY.md section 0 lists the live port's bugs).
"""
from __future__ import annotations

from typing import Sequence, Tuple

import numpy as np


def pilot_positions(num_subcarriers: int, dmrs_symbols: Sequence[int], cdm_group: int):
    """Non-zero pilot REs of one user: list of (t, f)."""
    fs = [f for f in range(num_subcarriers) if f % 2 == cdm_group]
    return [(t, f) for t in dmrs_symbols for f in fs]


def nearest_pilot_pe(num_subcarriers: int, num_symbols: int,
                     pilots_per_user: Sequence[Sequence[Tuple[int, int]]]) -> np.ndarray:
    """onnx_utils.py:206-260 restated; returns pe [num_tx, F, T, 2] float32."""
    num_tx = len(pilots_per_user)
    t_ind = np.arange(num_symbols)
    f_ind = np.arange(num_subcarriers)
    dist_t = np.zeros([num_tx, num_symbols, num_subcarriers])
    dist_f = np.zeros([num_tx, num_symbols, num_subcarriers])
    for tx, pil in enumerate(pilots_per_user):
        pt = np.array([p[0] for p in pil])
        pf = np.array([p[1] for p in pil])
        # min over pilots of |p_t - t| (broadcast over f) and |p_f - f| (over t)
        dist_t[tx] = np.min(np.abs(pt[:, None] - t_ind[None, :]), axis=0)[:, None]
        dist_f[tx] = np.min(np.abs(pf[:, None] - f_ind[None, :]), axis=0)[None, :]
    dist_t -= np.mean(dist_t, axis=1, keepdims=True)
    std_ = np.std(dist_t, axis=1, keepdims=True)
    dist_t = np.where(std_ > 0.0, dist_t / np.where(std_ > 0, std_, 1.0), dist_t)
    dist_f -= np.mean(dist_f, axis=2, keepdims=True)
    std_ = np.std(dist_f, axis=2, keepdims=True)
    dist_f = np.where(std_ > 0.0, dist_f / np.where(std_ > 0, std_, 1.0), dist_f)
    pe = np.stack([dist_t, dist_f], axis=-1)          # [tx, t, f, 2]
    return np.transpose(pe, (0, 2, 1, 3)).astype(np.float32)


def pe_for_groups(num_subcarriers: int, num_symbols: int, dmrs_symbols: Sequence[int],
                  cdm_groups: Sequence[int]) -> np.ndarray:
    pil = [pilot_positions(num_subcarriers, dmrs_symbols, g) for g in cdm_groups]
    return nearest_pilot_pe(num_subcarriers, num_symbols, pil)


def aerial_nn_indices(dmrs_ofdm_pos: np.ndarray, dmrs_subcarrier_pos: np.ndarray,
                      num_symbols: int, num_prbs: int):
    """NRPreprocessing._calculate_nn_indices with TF semantics.

    Returns ``nn_idx [U, 1, T, 12]`` (index into the per-PRB pilot list ordered
    symbol-major: ``i = i_sym * n_sc + i_sc``, the flattening of TF's default 'xy'
    ``meshgrid(dmrs_subcarrier_pos, dmrs_ofdm_pos)`` of shape [n_sym, n_sc]) and
    ``pe [U, F, T, 2]``.  Ties in the Manhattan distance go to the first pilot in that
    order (argmin); the PE normalisation uses the population std (tf.math.reduce_std).
    """
    num_tx = dmrs_ofdm_pos.shape[0]
    # RE list in symbol-major order: TF meshgrid default 'xy' -> shape [T, 12]
    sc, sym = np.meshgrid(np.arange(12), np.arange(num_symbols))   # 'xy'
    re_pos = np.stack([sc, sym], axis=-1).reshape(-1, 1, 2)         # [(T*12), 1, 2]
    pes, idxs = [], []
    for tx in range(num_tx):
        psc, psym = np.meshgrid(dmrs_subcarrier_pos[tx], dmrs_ofdm_pos[tx], indexing="xy")
        pilot_pos = np.stack([psc, psym], axis=-1).reshape(1, -1, 2)
        diff = np.abs(re_pos - pilot_pos)
        dist = diff.sum(-1)
        nn = dist.argmin(axis=1).reshape(1, 1, num_symbols, 12)
        pe = diff.min(axis=1).reshape(1, num_symbols, 12, 2).transpose(0, 2, 1, 3).astype(np.float64)
        comps = []
        for c in (1, 0):                  # [time, freq]
            v = pe[..., c:c + 1] - pe[..., c:c + 1].mean()
            sd = v.std()
            comps.append(v / sd if sd > 0 else v)
        pes.append(np.concatenate(comps, axis=-1))
        idxs.append(nn)
    pe = np.tile(np.concatenate(pes, axis=0), (1, num_prbs, 1, 1)).astype(np.float32)
    return np.concatenate(idxs, axis=0), pe


def focc_removal(h_hat: np.ndarray) -> np.ndarray:
    """NRPreprocessing._focc_removal (neural_rx.py:1620-1629): average adjacent pilot
    pairs along the last axis and repeat."""
    s = h_hat.shape
    h = h_hat.reshape(s[:-1] + (-1, 2))
    h = h.sum(-1, keepdims=True) / 2.0
    h = np.repeat(h, 2, axis=-1)
    return h.reshape(s)


def aerial_preprocess(y_real, y_imag, h_ls_real, h_ls_imag, dmrs_ofdm_pos, dmrs_subcarrier_pos,
                      num_tx: int):
    """NeuralReceiverONNX input stage with TF semantics (neural_rx.py:1773-1797 +
    NRPreprocessing.forward 1698-1711; TF structure in "neural_rx copy_pytorch.py"
    959-1092).

    y_real/imag [B, F, T, A]; h_ls_real/imag [B, Npil, U, A] with the pilot axis ordered
    (DMRS symbol k, PRB, pilot j): ``p = (k * nprb + prb) * n_sc + j`` (the two
    ``split_dim`` calls of ``_nn_interpolation``).  Returns ``y [B, F, T, 2A]``,
    ``h_hat [B, U, F, T, 2A]`` (FOCC pair average, then per-PRB nearest-pilot gather)
    and ``pe [U, F, T, 2]``.
    """
    y = np.concatenate([y_real, y_imag], axis=-1)
    h = np.concatenate([h_ls_real, h_ls_imag], axis=-1)           # [B, Npil, U, 2A]
    h = np.transpose(h, (0, 3, 2, 1))                              # [B, 2A, U, Npil]
    h = focc_removal(h)
    B, F, T = y.shape[0], y.shape[1], y.shape[2]
    nsym = dmrs_ofdm_pos.shape[-1]
    nsc = dmrs_subcarrier_pos.shape[-1]
    nprb = h.shape[-1] // (nsc * nsym)
    assert nprb * 12 == F
    # [B, 2A, U, nsym, nprb, nsc] -> [B, 2A, U, nprb, nsym * nsc]
    hp = h.reshape(B, h.shape[1], h.shape[2], nsym, nprb, nsc).transpose(0, 1, 2, 4, 3, 5)
    hp = hp.reshape(B, h.shape[1], h.shape[2], nprb, nsym * nsc)
    nn, pe = aerial_nn_indices(dmrs_ofdm_pos, dmrs_subcarrier_pos, T, nprb)
    out = np.zeros((B, num_tx, F, T, h.shape[1]), h.dtype)
    for u in range(num_tx):
        idx = nn[u, 0]                                             # [T, 12]
        g = hp[:, :, u][:, :, :, idx]                              # [B, 2A, nprb, T, 12]
        g = g.transpose(0, 2, 4, 3, 1).reshape(B, F, T, h.shape[1])
        out[:, u] = g
    return y, out, pe[:num_tx]

