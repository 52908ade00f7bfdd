"""Diagnostic: per-wave phase timeline of the register-resident kernels (NRX_STAMPS build).

NRX_STAMP_LAUNCH selects the launch (-1: StateInit, 0 / 1: update i).  Phases of the
workgroup's second item (s_memtime, lane 0 of each wave): 0 item start, 1 inputs in (z wait
+ barrier), 2 conv1 done + exchange barrier, 3 conv2 math done, 4 conv3 inputs in + X-free
barrier, 5 conv3 math done, 6 tail-weights barrier, 7 epilogue done."""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from neural_rx_amd import build as _B  # noqa: E402

LIB = os.path.join(ROOT, "neural_rx_amd/lib/var/stamps/libnrx.so")
if not os.path.exists(LIB):
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-DNRX_STAMPS", *_B.SOURCES, "-o", LIB], check=True)
if len(sys.argv) > 1 and sys.argv[1] == "--build-only":
    sys.exit(0)
import torch  # noqa: E402
from neural_rx_amd import _lib  # noqa: E402

lib = _lib.load(LIB)
lib.nrx_debug_rr_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
from neural_rx_amd import synth, weights as W  # noqa: E402
from neural_rx_amd.config import get_config, spec_from_config  # noqa: E402
from neural_rx_amd.receiver import CGNNEngine, compute_pe  # noqa: E402

cfg = get_config("nrx_rt")
spec = spec_from_config(cfg)
B, U, prbs = int(os.environ.get("NRX_STAMP_B", 128)), 2, 4
sl = synth.generate(B, U, prbs, 4, [4, 4], (0, 1), snr_db=10, seed=3)
eng = CGNNEngine(spec, W.load("nrx_rt"))
t = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
pe = t(compute_pe(U, 48, (2, 11), (0, 1)))
dy, dh, da = t(sl.y), t(sl.h_hat), t(sl.active)
for _ in range(200):
    eng.forward(dy, pe, dh, da, None, 2, "f16")
torch.cuda.synchronize()
n = 512
buf = np.zeros((n, 64), np.uint64)
lib.nrx_debug_rr_stamps(buf.ctypes.data, n)
st = buf.astype(np.int64).reshape(n, 32, 2)          # [wg, phase, wave 0 / wave 4]
used = st[:, 21, 0] > 0
st = st[used]
names = {0: "item start", 1: "inputs issued", 2: "inputs waited + barrier", 3: "pe stored + barrier",
         4: "W2 DMA issued", 5: "conv1 math done", 6: "exch written + W2 landed", 7: "barrier",
         8: "W3 DMA issued", 9: "conv2 math done", 10: "barrier", 11: "exch written + W3 landed",
         12: "barrier", 13: "neighbours read + state prefetch", 14: "X-free barrier",
         15: "next z + tail DMA issued", 16: "conv3 math done", 17: "settle", 18: "vmcnt(0)",
         19: "barrier", 20: "next W1 DMA issued", 21: "epilogue done"}
print("launch", os.environ.get("NRX_STAMP_LAUNCH", "0"), "workgroups", int(used.sum()))
base = st[:, 0, 0:1]
rel = st - base[:, :, None]
print(f"{'phase':36s} {'wave0 (R=3)':>12s} {'wave4 (R=2, DMA)':>17s}   (s_memtime ticks from wave 0's item start)")
prev = [0, 0]
for k, nm in names.items():
    ok = (st[:, k, :] > 0).all(axis=1)
    if not ok.any():
        continue
    m = rel[ok, k, :].mean(axis=0)
    print(f"{k:2d} {nm:33s} {m[0]:9.0f} (+{m[0] - prev[0]:5.0f}) {m[1]:9.0f} (+{m[1] - prev[1]:5.0f})")
    prev = [m[0], m[1]]
