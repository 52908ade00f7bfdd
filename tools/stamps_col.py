"""Diagnostic: per-phase cycles of the whole-column launches (k_init_col, k_update_col), from an
NRX_STAMPS variant library (python tools/build_variants.py stamps=-DNRX_STAMPS, or any path).

usage (GPU box): NRX_STAMP_COL=<launch> python tools/stamps_col.py [lib]
Runs 200 bench forwards (nrx_rt, B = 128, U = 2, 4 PRB; NRX_STAMP_SHAPE="B,U,PRB") with every
stage on the column launches (schedule mask 28): launch 3 i is forward i's StateInit, 3 i + 1 its
aggregation update, 3 i + 2 its readout update.  Prints, per item k of a workgroup (k < 4) and for
waves 0 and 4, the mean over workgroups of each phase's cycles (col_ts in nrx_col.inc), the
weight-staging time and the kernel's wall span / shader clock (s_memrealtime edges).
"""
import ctypes
import os
import sys

os.environ.setdefault("NRX_UPDATE_RR", "28")

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from neural_rx_amd import _lib  # noqa: E402

path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(_lib.LIB_PATH), "diag", "stamps", "libnrx.so")
lib = _lib.load(path)
lib.nrx_debug_col_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
from neural_rx_amd import synth, weights as W  # noqa: E402
from neural_rx_amd.config import get_config, spec_from_config  # noqa: E402
from neural_rx_amd.receiver import CGNNEngine, compute_pe  # noqa: E402

B, U, prbs = (int(x) for x in os.environ.get("NRX_STAMP_SHAPE", "128,2,4").split(","))
cfg = get_config("nrx_rt")
spec = spec_from_config(cfg)
groups = tuple(i % 2 for i in range(U))
sl = synth.generate(B, U, prbs, 4, [4] * U, groups, snr_db=10, seed=3)
eng = CGNNEngine(spec, W.load("nrx_rt"))
# mask bit 32 = the one-launch column forward (k_fwd_col), which needs the one-launch paths on
eng.fused_config(enable=bool(int(os.environ["NRX_UPDATE_RR"]) & 32))
t = lambda a: torch.from_numpy(a).cuda()
pe = t(compute_pe(U, 12 * prbs, (2, 11), groups))
dy, dh, da = t(sl.y), t(sl.h_hat), t(sl.active)
for _ in range(200):
    eng.forward(dy, pe, dh, da, None, 2, "f16")
torch.cuda.synchronize()
n = 256
buf = np.zeros((n, 64), np.uint64)
lib.nrx_debug_col_stamps(buf.ctypes.data, n)
st = buf.astype(np.int64).reshape(n, 4, 8, 2)   # [wg][item k][m][wave 0 / 4]
L = int(os.environ.get("NRX_STAMP_COL", "-1"))
print("launch", L, ["StateInit", "aggregation update", "readout update"][L % 3] if L >= 0 else "")
# m = 5: StateInit: the slot norm is known; UpdateState: the first item's weights are staged
phases = [("pro", 0, 5), ("conv1", 5, 1), ("exch1", 1, 2), ("conv2", 2, 3), ("exch2", 3, 4), ("conv3+epi", 4, 6)]
PRO = os.environ.get("NRX_PRO") == "1"
if PRO:
    # NRX_PRO_STAMPS build: the first item's prologue and conv1 in the item-1 slots (col_upd_item)
    chain = [("kernel start", 0, 7), ("item start", 0, 0), ("z rows issued", 1, 0), ("rest weights issued", 1, 1),
             ("W1 stored", 1, 2), ("barrier", 0, 5), ("step 0 depthwise", 1, 3), ("pass 0 done", 1, 4),
             ("rest weights stored", 1, 5), ("conv1 done", 0, 1)]
    ok = (st[:, 0, 6, 0] != 0) & (st[:, 1, 2, 0] != 0)
    for w in (0, 1):
        print("   wave", 4 * w, " -> ".join(f"{nm} +{(st[ok, k1, m1, w] - st[ok, k0, m0, w]).mean():.0f}"
                                       for (_, k0, m0), (nm, k1, m1) in zip(chain, chain[1:])))
for k in range(1 if PRO else 4):
    s0 = st[:, k, 0, 0]
    if (s0 == 0).all():
        continue
    ok = (s0 != 0) & (st[:, k, 6, 0] != 0)
    tot = st[ok, k, 6, 0] - st[ok, k, 0, 0]
    print(f"item {k}: {ok.sum()} workgroups, item {tot.mean():.0f} cycles (wave 0), min {tot.min()} max {tot.max()}")
    for w in (0, 1):
        print("   wave", 4 * w, "  ".join(f"{nm} {(st[ok, k, b, w] - st[ok, k, a, w]).mean():6.0f}" for nm, a, b in phases))
for k in range(0 if PRO else 3):   # the one-launch forward: gap between a workgroup's consecutive items
    ok = (st[:, k, 6, 0] != 0) & (st[:, k + 1, 0, 0] != 0)
    if ok.any():
        gap = st[ok, k + 1, 0, 0] - st[ok, k, 6, 0]
        w = st[ok, k + 1, 7, 1]   # after the dependency wait (k_fwd_col diagnostic stamp)
        part = f"; to the wait's end {(w - st[ok, k, 6, 0]).mean():.0f}, then {(st[ok, k + 1, 0, 0] - w).mean():.0f}" \
            if (w != 0).all() else ""
        print(f"gap item {k} -> {k + 1} (signal, dequeue, dependency wait): mean {gap.mean():.0f} max {gap.max()} cycles{part}")
stage = st[:, 0, 0, 0] - st[:, 0, 7, 0]
ok = (st[:, 0, 7, 0] != 0) & (st[:, 0, 0, 0] != 0)
if ok.any():
    print(f"weight staging (kernel start -> item 0 start, wave 0): mean {stage[ok].mean():.0f} max {stage[ok].max()} cycles")
rt0, rt1, mt1, mt0 = buf[:, 16 + 14].astype(np.int64), buf[:, 32 + 14].astype(np.int64), \
    buf[:, 48 + 14].astype(np.int64), buf[:, 14].astype(np.int64)
ok = (rt0 > 0) & (rt1 > 0)
if ok.any():
    span = (rt1[ok].max() - rt0[ok].min()) / 100.0
    per = (rt1[ok] - rt0[ok]) / 100.0
    mhz = (mt1[ok] - mt0[ok]) / np.maximum(per, 1e-3)
    print(f"kernel wall span {span:.2f} us (first workgroup start -> last end); per workgroup "
          f"{per.mean():.2f} us mean, {per.min():.2f} min, {per.max():.2f} max; start skew "
          f"{(rt0[ok].max() - rt0[ok].min()) / 100.0:.2f} us; shader clock {mhz.mean():.0f} MHz "
          f"(min {mhz.min():.0f}, max {mhz.max():.0f})")
