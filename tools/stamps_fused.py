"""Diagnostic: per-item phase timeline of the one-launch forward (NRX_STAMPS build).

Stamps (s_memtime, thread 0 of each workgroup, items 0..7 of the workgroup): 0 item start,
1 conv1 start, 2 conv1 end, 3 conv2 end, 4 conv3 epilogue start, 5 item body done,
6 signalled (counter added); slot 7 holds the item's stage + 1.  Prints the mean phase
lengths per item position and stage, in cycles, and the kernel span."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = os.environ.get("NRX_STAMPS_LIB", os.path.join(ROOT, "neural_rx_amd/lib/var/stamps/libnrx.so"))
os.environ["NRX_LIB_PATH"] = LIB
os.environ["NRX_STAMP_FUSED"] = "1"
import torch  # noqa: E402
from neural_rx_amd import _lib, synth, weights as W  # noqa: E402
from neural_rx_amd.config import get_config, spec_from_config  # noqa: E402
from neural_rx_amd.receiver import CGNNEngine, compute_pe  # noqa: E402

lib = _lib.load(LIB)
lib.nrx_debug_fused_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
cfg = get_config("nrx_rt")
spec = spec_from_config(cfg)
B, U = int(os.environ.get("NRX_STAMP_B", 128)), 2
sl = synth.generate(B, U, 4, 4, [4, 4], (0, 1), snr_db=10, seed=3)
eng = CGNNEngine(spec, W.load("nrx_rt"))
t = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
pe = t(compute_pe(U, 48, (2, 11), (0, 1)))
dy, dh, da = t(sl.y), t(sl.h_hat), t(sl.active)
for _ in range(300):
    eng.forward(dy, pe, dh, da, None, 2, "f16")
torch.cuda.synchronize()
n = 256
buf = np.zeros((n, 64), np.uint64)
lib.nrx_debug_fused_stamps(buf.ctypes.data, n)
buf = buf.astype(np.int64).reshape(n, 8, 8)
t0 = buf[:, 0, 0].min()
names = ["prologue", "conv1", "conv2", "conv3", "epilogue", "signal"]
print(f"{'item':>4} {'stage':>5} {'start':>8} " + " ".join(f"{x:>9}" for x in names) + f" {'gap':>7} {'total':>7}")
for i in range(8):
    ok = buf[:, i, 7] > 0
    if not ok.any():
        continue
    for st in sorted(set(buf[ok, i, 7])):
        sel = ok & (buf[:, i, 7] == st)
        v = buf[sel, i, :7]
        d = np.diff(v, axis=1).mean(axis=0)
        nxt = buf[sel, i + 1, 0] if i < 7 else np.zeros(sel.sum(), np.int64)
        gap = (nxt - v[:, 6])[nxt > 0].mean() if (nxt > 0).any() else 0
        print(f"{i:>4} {st - 1:>5} {(v[:, 0] - t0).mean():8.0f} " + " ".join(f"{x:9.0f}" for x in d) +
              f" {gap:7.0f} {(v[:, 6] - v[:, 0]).mean():7.0f}   ({sel.sum()} wgs)")
last = np.where(buf[:, :, 6] > 0, buf[:, :, 6], 0).max(axis=1)
print(f"kernel span {float((last - t0).max()):.0f} cycles (first item start -> last signal), "
      f"mean workgroup end {float((last - t0).mean()):.0f}")
