"""Algorithmic work per kernel.

FLOPs count 2 per multiply-accumulate of the reference network, per resource element
(RE = one subcarrier x one OFDM symbol, T = 14, no padding) and per user; padding
work (T 14 -> 16, channels 56 -> 64 / 114 -> 128 / bits -> 16) is real work the
kernels do but is NOT counted, so it shows up as lost roofline fraction.
``sep(ci, co) = 9 ci + ci co`` (depthwise 3x3 + pointwise).
"""
from __future__ import annotations

from .config import ModelSpec


def sep(ci: int, co: int) -> int:
    return 9 * ci + ci * co


def kernel_flops_per_re_user(spec: ModelSpec) -> dict:
    u1, u2 = spec.init_units
    v1, v2 = spec.state_units
    init = 2 * spec.num_init * (sep(spec.init_in_ch, u1) + sep(u1, u2) + sep(u2, spec.d_s))
    agg = 2 * (spec.d_s * spec.agg_units + spec.agg_units * spec.d_s)
    upd = 2 * (sep(spec.update_in_ch, v1) + sep(v1, v2) + sep(v2, spec.d_s))
    ro = 2 * (sum(spec.d_s * spec.readout_units + spec.readout_units * b for b in spec.head_bits)
              + spec.d_s * spec.readout_units + spec.readout_units * 2 * spec.num_rx_ant)
    return {"norm": 0, "state_init": init, "aggregate": agg, "state_update": upd, "readout": ro}


def launch_flops_per_re_user(spec: ModelSpec, num_it: int) -> dict:
    """Algorithmic FLOPs per RE-user of each *launch* of the engine's kernels, as fused:
    k_init = StateInit(s) + aggregation MLP of iteration 0 (tail); k_update (average
    over its num_it launches) = state update + the next aggregation MLP, or the readouts
    after the last iteration."""
    k = kernel_flops_per_re_user(spec)
    out = {"norm": 0,
           "state_init": k["state_init"] + k["aggregate"],
           "state_update": k["state_update"] + ((num_it - 1) * k["aggregate"] + k["readout"]) / num_it,
           "forward": forward_flops_per_re_user(spec, num_it)}
    out["state_update_rr"] = out["state_update"]   # the register-resident update launch: same work
    out["state_update_col"] = out["state_update"]  # the whole-column update launch: same work
    out["state_init_col"] = out["state_init"]
    out["forward_col"] = out["forward"]            # the one-launch column forward
    out["combine"] = 0   # U > 2: the leave-one-out mean pass (k_combine), byte work
    return out


def update_launch_bytes_per_re_user(spec: ModelSpec, num_it: int, elem: int = 2) -> float:
    """Algorithmic HBM bytes per RE-user of one k_update launch (average over num_it):
    non-last launches read s, a and write s', act*sp; the last reads s, a and writes the
    f32 LLRs of every head and the f32 ChEst (pe is shared over slots and not counted)."""
    st = spec.d_s * elem
    mid = 4 * st
    last = 2 * st + 4 * (spec.bits_max * spec.num_llr_heads + 2 * spec.num_rx_ant)
    return ((num_it - 1) * mid + last) / num_it


def init_launch_bytes_per_re_user(spec: ModelSpec, num_users: int, elem: int = 2) -> float:
    """Algorithmic HBM bytes per RE-user of the StateInit launch: y (f32, shared by the
    slot's users) and h_hat (f32) in, s and act*sp out in storage precision."""
    a2 = 2 * spec.num_rx_ant
    return a2 * 4 / num_users + (a2 * 4 if spec.use_h_hat else 0) + 2 * spec.d_s * elem


def forward_bytes_per_re_user(spec: ModelSpec, num_it: int, num_users: int, elem: int = 2) -> float:
    """Algorithmic HBM bytes per RE-user of the one-launch forward (k_forward): the same
    hand-offs as the three-launch schedule -- StateInit's, then every update's."""
    return init_launch_bytes_per_re_user(spec, num_users, elem) + num_it * update_launch_bytes_per_re_user(
        spec, num_it, elem)


def forward_split_per_re_user(spec: ModelSpec, num_it: int) -> dict:
    """The whole forward's algorithmic FLOPs split by pipe (depthwise taps on the VALU)."""
    u1, u2 = spec.init_units
    v1, v2 = spec.state_units
    dw = 2 * 9 * (spec.num_init * (spec.init_in_ch + u1 + u2) + num_it * (spec.update_in_ch + v1 + v2))
    total = forward_flops_per_re_user(spec, num_it)
    return {"depthwise_valu": dw, "dense_mfma": total - dw, "total": total}


def forward_mixed_bound_tflops(spec: ModelSpec, num_it: int, mfma_tflops: float = 2500.0,
                               valu_tflops: float = 157.3) -> float:
    """mixed_bound_tflops for the whole forward (the one-launch kernel)."""
    s = forward_split_per_re_user(spec, num_it)
    return s["total"] / (s["dense_mfma"] / mfma_tflops + s["depthwise_valu"] / valu_tflops)


def forward_flops_per_re_user(spec: ModelSpec, num_it: int) -> int:
    k = kernel_flops_per_re_user(spec)
    return k["state_init"] + num_it * (k["aggregate"] + k["state_update"]) + k["readout"]


def io_bytes_per_slot(spec: ModelSpec, num_tx: int, num_subcarriers: int, elem: int = 4,
                      with_h: bool = True) -> dict:
    """Compulsory HBM bytes of one slot: inputs y, h_hat, pe and outputs llr (+ h_ref)."""
    re = num_subcarriers * 14
    a2 = 2 * spec.num_rx_ant
    inp = re * a2 * elem + num_tx * re * a2 * elem + num_tx * re * 2 * elem
    out = num_tx * re * spec.bits_max * 4 * spec.num_llr_heads + (num_tx * re * a2 * 4 if with_h else 0)
    return {"in": inp, "out": out}


def compulsory_bytes_per_forward(spec: ModelSpec, batch: int, num_tx: int, num_subcarriers: int,
                                 with_h: bool = True) -> int:
    """SURVEY.md 8(d) compulsory HBM bytes of one forward over ``batch`` slots, as the C ABI
    takes and returns them (f32): y ``[B,F,14,2A]`` and h_hat ``[B,U,F,14,2A]`` in, the f32
    LLRs of every head and (with_h) h_ref ``[B,U,F,14,2A]`` out, pe ``[U,F,14,2]`` once (shared
    by the slots).  cfg2 (B 128, 2 UE, 4 PRB): 16.5 MB."""
    re = num_subcarriers * 14
    a2 = 2 * spec.num_rx_ant
    y = batch * re * a2 * 4
    h = batch * num_tx * re * a2 * 4 if spec.use_h_hat else 0
    pe = num_tx * re * 2 * 4
    llr = batch * num_tx * re * spec.bits_max * 4 * spec.num_llr_heads
    h_ref = batch * num_tx * re * a2 * 4 if with_h else 0
    return y + h + pe + llr + h_ref


def update_launch_split_per_re_user(spec: ModelSpec, num_it: int) -> dict:
    """The k_update launch's algorithmic FLOPs split by the pipe that executes them:
    the depthwise 3x3 taps run on the VALU (packed f16 FMAs), everything else (pointwise
    1x1 and the dense MLPs of the fused tails) on the MFMA pipe."""
    v1, v2 = spec.state_units
    dw = 2 * 9 * (spec.update_in_ch + v1 + v2)
    total = launch_flops_per_re_user(spec, num_it)["state_update"]
    return {"depthwise_valu": dw, "dense_mfma": total - dw, "total": total}


def mixed_bound_tflops(spec: ModelSpec, num_it: int, mfma_tflops: float = 2500.0,
                       valu_tflops: float = 157.3) -> float:
    """Roofline of the k_update launch when each FLOP runs on its own pipe at that pipe's
    peak and the two pipes overlap perfectly: total / (dense / MFMA peak + depthwise /
    VALU peak).  The VALU peak is the f32 vector peak; packed f16 FMAs issue at the same
    wave-instruction rate on gfx950 (tools/ubench/valu_occ.hip)."""
    s = update_launch_split_per_re_user(spec, num_it)
    return s["total"] / (s["dense_mfma"] / mfma_tflops + s["depthwise_valu"] / valu_tflops)


# MI355X peaks (MI355X_MICROARCH.md "Chip-level parameters")
PEAK_TFLOPS = {"f16": 2500.0, "f32x": 78.6}   # dense f16 MFMA; f64 MFMA (spec, = FP32/2)
PEAK_HBM_GBS = 8000.0
PEAK_VALU_TFLOPS = 157.3                       # f32 vector peak (= packed f16 issue rate)
