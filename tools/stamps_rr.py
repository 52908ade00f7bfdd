"""Diagnostic: per-phase cycles of the register-resident update launch (k_update_rr), from the
NRX_STAMPS variant library (python tools/build_variants.py stamps=-DNRX_STAMPS).

usage (GPU box): NRX_STAMP_RR=<launch> python tools/stamps_rr.py [lib]
Runs 200 bench forwards (nrx_rt, B = 128, U = 2, 4 PRB); launch 2 i is forward i's aggregation
update, 2 i + 1 its readout update.  Prints, per item k of a workgroup (k < 4) and for waves 0
(R = 3) and 4 (R = 2), the mean over workgroups of each phase's cycles (rr_ts in nrx_rr.inc).
"""
import ctypes
import os
import sys

os.environ.setdefault("NRX_UPDATE_RR", "3")   # both update stages register-resident: launches 2 i, 2 i + 1

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from neural_rx_amd import _lib  # noqa: E402

path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(_lib.LIB_PATH), "var", "stamps", "libnrx.so")
lib = _lib.load(path)
lib.nrx_debug_rr_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
from neural_rx_amd import synth, weights as W  # noqa: E402
from neural_rx_amd.config import get_config, spec_from_config  # noqa: E402
from neural_rx_amd.receiver import CGNNEngine, compute_pe  # noqa: E402

# NRX_STAMP_SHAPE = "B,U,PRB" (nrx_rt weights; default the bench shape 128,2,4)
B, U, prbs = (int(x) for x in os.environ.get("NRX_STAMP_SHAPE", "128,2,4").split(","))
cfg = get_config("nrx_rt")
spec = spec_from_config(cfg)
groups = tuple(i % 2 for i in range(U))
sl = synth.generate(B, U, prbs, 4, [4] * U, groups, snr_db=10, seed=3)
eng = CGNNEngine(spec, W.load("nrx_rt"))
t = lambda a: torch.from_numpy(a).cuda()
pe = t(compute_pe(U, 12 * prbs, (2, 11), groups))
dy, dh, da = t(sl.y), t(sl.h_hat), t(sl.active)
for _ in range(200):
    eng.forward(dy, pe, dh, da, None, 2, "f16")
torch.cuda.synchronize()
n = 256
buf = np.zeros((n, 64), np.uint64)
lib.nrx_debug_rr_stamps(buf.ctypes.data, n)
st = buf.astype(np.int64).reshape(n, 4, 8, 2)   # [wg][item k][m][wave 0 / 4]
names = ["conv1", "exch1", "conv2", "exch2", "conv3", "epilogue"]
print("launch", os.environ.get("NRX_STAMP_RR"), "(2 i: aggregation update, 2 i + 1: readout)")
for k in range(4):
    s0 = st[:, k, 0, 0]
    if (s0 == 0).all():
        continue
    ok = s0 != 0
    tot = st[ok, k, 6, 0] - st[ok, k, 0, 0]
    print(f"item {k}: {ok.sum()} workgroups, item {tot.mean():.0f} cycles (wave 0)")
    for w in (0, 1):
        d = np.diff(st[ok, k, :7, w], axis=1)
        print("   wave", 4 * w, "  ".join(f"{nm} {d[:, i].mean():6.0f}" for i, nm in enumerate(names)))
stage = st[:, 0, 0, 0] - st[:, 0, 7, 0]
ok = (st[:, 0, 7, 0] != 0) & (st[:, 0, 0, 0] != 0)
if ok.any():
    print(f"weight staging (kernel start -> item 0 start, wave 0): mean {stage[ok].mean():.0f} max {stage[ok].max()} cycles")
rt0, rt1, mt1, mt0 = buf[:, 16 + 14].astype(np.int64), buf[:, 32 + 14].astype(np.int64), \
    buf[:, 48 + 14].astype(np.int64), buf[:, 14].astype(np.int64)
ok = (rt0 > 0) & (rt1 > 0)
if ok.any():
    # s_memrealtime runs at 100 MHz on every XCD; s_memtime is the XCD's own shader clock
    span = (rt1[ok].max() - rt0[ok].min()) / 100.0
    per = (rt1[ok] - rt0[ok]) / 100.0
    mhz = (mt1[ok] - mt0[ok]) / np.maximum(per, 1e-3)
    print(f"kernel wall span {span:.2f} us (first workgroup start -> last end); per workgroup "
          f"{per.mean():.2f} us mean, {per.min():.2f} min, {per.max():.2f} max; start skew "
          f"{(rt0[ok].max() - rt0[ok].min()) / 100.0:.2f} us; shader clock {mhz.mean():.0f} MHz "
          f"(min {mhz.min():.0f}, max {mhz.max():.0f})")
