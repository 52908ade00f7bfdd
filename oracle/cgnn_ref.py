"""numpy restatement of the trained CGNN forward pass (oracle; test infrastructure only).

Structure follows the faithful (commented) torch translation of the TF model,
``utils/neural_rx copy_pytorch.py``:

* ``SeparableConv2d``            copy_pytorch.py:34-51  (Keras SeparableConv2D, SAME)
* ``StateInit``                  copy_pytorch.py:82-188 (concat [y, pe, h_hat], :168-175)
* ``AggregateUserStates``        copy_pytorch.py:191-231 (== live neural_rx.py:135-207)
* ``UpdateState``                copy_pytorch.py:234-287 (concat [a, s, pe], :276; skip :283)
* ``CGNNIt``                     copy_pytorch.py:290-321
* ``ReadoutLLRs``/``ReadoutChEst`` copy_pytorch.py:324-362 (== neural_rx.py:309-404)
* ``CGNN.forward``               copy_pytorch.py:474-514 (normalisation :478-484,
  Var-IO mix :487-494, iterations + readouts :497-514; live port neural_rx.py:544-595)

Keras semantics restated here (TF 2.15 is not in the repository):
depthwise kernel ``[3,3,Cin,1]`` is a cross-correlation over (F, T) with SAME zero
padding, followed by the pointwise kernel ``[1,1,Cin,Cout]`` plus bias; Dense kernel
``[in, out]`` plus bias.  Normalisation uses divide-no-nan semantics (an all-zero
slot gets scale 0 instead of the live port's ``rsqrt`` -> inf -> NaN).

The weight list is the Keras ``get_weights()`` order.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Sequence

import numpy as np


@dataclasses.dataclass
class SepConvW:
    dw: np.ndarray   # [3, 3, Cin, 1]
    pw: np.ndarray   # [1, 1, Cin, Cout]
    b: np.ndarray    # [Cout]


@dataclasses.dataclass
class DenseW:
    w: np.ndarray    # [in, out]
    b: np.ndarray    # [out]


@dataclasses.dataclass
class CGNNWeights:
    init: List[List[SepConvW]]          # num_init x 3
    agg: List[List[DenseW]]             # num_it x 2
    update: List[List[SepConvW]]        # num_it x 3
    llr: List[List[DenseW]]             # num_llr_heads x 2
    chest: List[DenseW]                 # 2


def split_keras_weights(arrays: Sequence[np.ndarray], spec) -> CGNNWeights:
    """Split a Keras ``get_weights()`` list (SURVEY.md a15 ordering rule)."""
    it = iter(arrays)

    def sep(cin, cout):
        dw, pw, b = next(it), next(it), next(it)
        assert dw.shape == (3, 3, cin, 1), dw.shape
        assert pw.shape == (1, 1, cin, cout), pw.shape
        assert b.shape == (cout,), b.shape
        return SepConvW(dw, pw, b)

    def dense(cin, cout):
        w, b = next(it), next(it)
        assert w.shape == (cin, cout), (w.shape, cin, cout)
        assert b.shape == (cout,)
        return DenseW(w, b)

    u1, u2 = spec.init_units
    init = [[sep(spec.init_in_ch, u1), sep(u1, u2), sep(u2, spec.d_s)]
            for _ in range(spec.num_init)]
    agg, upd = [], []
    v1, v2 = spec.state_units
    for _ in range(spec.num_it):
        agg.append([dense(spec.d_s, spec.agg_units), dense(spec.agg_units, spec.d_s)])
        upd.append([sep(spec.update_in_ch, v1), sep(v1, v2), sep(v2, spec.d_s)])
    llr = [[dense(spec.d_s, spec.readout_units), dense(spec.readout_units, nb)]
           for nb in spec.head_bits]
    chest = [dense(spec.d_s, spec.readout_units),
             dense(spec.readout_units, 2 * spec.num_rx_ant)]
    rest = list(it)
    if rest:
        raise ValueError(f"{len(rest)} unused weight arrays")
    return CGNNWeights(init, agg, upd, llr, chest)


def sepconv(x: np.ndarray, w: SepConvW, relu: bool) -> np.ndarray:
    """Keras SeparableConv2D(3x3, padding='same') on NHWC ``x`` = [N, F, T, C]."""
    n, f, t, c = x.shape
    dt = x.dtype
    xp = np.zeros((n, f + 2, t + 2, c), dtype=dt)
    xp[:, 1:-1, 1:-1] = x
    dw = w.dw[..., 0].astype(dt)
    d = np.zeros_like(x)
    for i in range(3):
        for j in range(3):
            d += dw[i, j] * xp[:, i:i + f, j:j + t, :]
    out = d @ w.pw[0, 0].astype(dt) + w.b.astype(dt)
    return np.maximum(out, 0) if relu else out


def dense(x: np.ndarray, w: DenseW, relu: bool) -> np.ndarray:
    out = x @ w.w.astype(x.dtype) + w.b.astype(x.dtype)
    return np.maximum(out, 0) if relu else out


def sep_stack(z: np.ndarray, layers: List[SepConvW]) -> np.ndarray:
    for k, w in enumerate(layers):
        z = sepconv(z, w, relu=k < len(layers) - 1)
    return z


def normalise(y: np.ndarray, h_hat: Optional[np.ndarray]):
    """Per-slot unit-power scaling (neural_rx.py:551-557; copy_pytorch.py:478-484)."""
    ms = np.mean(y * y, axis=(1, 2, 3), keepdims=True)
    with np.errstate(divide="ignore"):
        ns = np.where(ms > 0, 1.0 / np.sqrt(np.where(ms > 0, ms, 1.0)), 0.0).astype(y.dtype)
    y = y * ns
    if h_hat is not None:
        h_hat = h_hat * ns[:, None]
    return y, h_hat, ns.reshape(-1)


def state_init(y, pe, h_hat, layers):
    """StateInit (copy_pytorch.py:160-188): tile y over users, tile pe over batch,
    concat [y, pe, h_hat], 3 separable convs."""
    b, f, t, _ = y.shape
    u = pe.shape[0]
    yt = np.repeat(y[:, None], u, axis=1).reshape(b * u, f, t, -1)
    pt = np.broadcast_to(pe[None], (b,) + pe.shape).reshape(b * u, f, t, -1)
    parts = [yt, pt]
    if h_hat is not None:
        parts.append(h_hat.reshape(b * u, f, t, -1))
    z = np.concatenate(parts, axis=-1)
    return sep_stack(z, layers).reshape(b, u, f, t, -1)


def aggregate(s, active, layers: List[DenseW]):
    """AggregateUserStates (neural_rx.py:135-207; copy_pytorch.py:207-231)."""
    sp = dense(dense(s, layers[0], True), layers[1], False)
    act = active.astype(s.dtype)[:, :, None, None, None]
    sp = sp * act
    a = sp.sum(axis=1, keepdims=True) - sp
    p = np.maximum(act.sum(axis=1, keepdims=True) - 1.0, 0.0)
    p = np.where(p == 0.0, 1.0, 1.0 / np.where(p == 0.0, 1.0, p)).astype(s.dtype)
    return a * p


def update(s, a, pe, layers):
    """UpdateState (copy_pytorch.py:267-287): concat [a, s, pe], 3 sep convs, skip."""
    b, u, f, t, ds = s.shape
    pt = np.broadcast_to(pe[None], (b,) + pe.shape)
    z = np.concatenate([a, s, pt], axis=-1).reshape(b * u, f, t, -1)
    z = sep_stack(z, layers).reshape(b, u, f, t, ds)
    return z + s


def cgnn_forward(y, pe, h_hat, active, mcs_ue_mask, weights: CGNNWeights, spec,
                 num_it: Optional[int] = None, dtype=np.float64,
                 return_state: bool = False) -> Dict:
    """CGNN.forward (copy_pytorch.py:474-514) at inference (readouts after the last
    iteration only).  Returns ``{"llr": [per-MCS arrays [B,U,F,T,bits_m]],
    "h_hat": [B,U,F,T,2A]}``."""
    num_it = spec.num_it if num_it is None else num_it
    if not 1 <= num_it <= spec.num_it:
        raise ValueError("Invalid number of iterations")
    y = np.asarray(y, dtype=dtype)
    pe = np.asarray(pe, dtype=dtype)
    h_hat = None if h_hat is None else np.asarray(h_hat, dtype=dtype)
    active = np.asarray(active, dtype=dtype)
    y, h_hat, ns = normalise(y, h_hat)
    if spec.masking:
        s = state_init(y, pe, h_hat, weights.init[0])
    else:
        mask = np.asarray(mcs_ue_mask, dtype=dtype)
        s = None
        for m in range(spec.num_init):
            sm = state_init(y, pe, h_hat, weights.init[m]) * mask[:, :, m, None, None, None]
            s = sm if s is None else s + sm
    states = [s]
    for i in range(num_it):
        a = aggregate(s, active, weights.agg[i])
        s = update(s, a, pe, weights.update[i])
        states.append(s)
    llrs = []
    for m in range(spec.num_mcs):
        if spec.masking:
            head = weights.llr[0]
            out = dense(dense(s, head[0], True), head[1], False)[..., :spec.bits[m]]
        else:
            head = weights.llr[m]
            out = dense(dense(s, head[0], True), head[1], False)
        llrs.append(out)
    h_ref = dense(dense(s, weights.chest[0], True), weights.chest[1], False)
    res = {"llr": llrs, "h_hat": h_ref, "norm_scale": ns}
    if return_state:
        res["states"] = states
    return res


def load_npz_weights(path: str) -> List[np.ndarray]:
    d = np.load(path)
    return [d[f"w{i:03d}"] for i in range(int(d["count"]))]


def count_params(spec) -> Dict[str, int]:
    """Per-block parameter counts (cf. nrx_architecture.ipynb:295-308)."""
    def sep(ci, co):
        return 9 * ci + ci * co + co

    def den(ci, co):
        return ci * co + co
    u1, u2 = spec.init_units
    v1, v2 = spec.state_units
    init = sep(spec.init_in_ch, u1) + sep(u1, u2) + sep(u2, spec.d_s)
    it = (den(spec.d_s, spec.agg_units) + den(spec.agg_units, spec.d_s)
          + sep(spec.update_in_ch, v1) + sep(v1, v2) + sep(v2, spec.d_s))
    llr = [den(spec.d_s, spec.readout_units) + den(spec.readout_units, nb)
           for nb in spec.head_bits]
    ch = den(spec.d_s, spec.readout_units) + den(spec.readout_units, 2 * spec.num_rx_ant)
    total = init * spec.num_init + it * spec.num_it + sum(llr) + ch
    return {"state_init": init, "cgnn_it": it, "readout_llrs": llr,
            "readout_chest": ch, "total": total}
