"""Diagnostic: per-phase timeline of one forward launch (NRX_STAMPS build), both items of a
paired workgroup.  NRX_STAMP_LAUNCH selects the launch (0, 1: k_update i; -1: k_init).

Stamps (s_memtime, wave 0 lane 0 of each workgroup): 0 start, 24/25 first item's DMA issue,
1 conv1 start, 2 conv1 end, 3 conv2 end, 6 epilogue start, 4 first item end; second item:
26 start, 27 after its wait + barrier, 28 block start, 34 conv1 end, 35 conv2 end, 38
epilogue start, 29 end; 5 kernel end."""
import ctypes
import os
import subprocess
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neural_rx_amd import build as _B  # noqa: E402

LIB = os.environ.get("NRX_STAMPS_LIB", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "neural_rx_amd/lib/var/stamps/libnrx.so"))
if not os.path.exists(LIB):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-DNRX_STAMPS", *_B.SOURCES, "-o", LIB], check=True)
import torch  # noqa: E402
from neural_rx_amd import _lib  # noqa: E402

lib = _lib.load(LIB)
lib.nrx_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
from neural_rx_amd import synth, weights as W  # noqa: E402
from neural_rx_amd.config import get_config, spec_from_config  # noqa: E402
from neural_rx_amd.receiver import CGNNEngine, compute_pe  # noqa: E402

cfg = get_config("nrx_rt")
spec = spec_from_config(cfg)
B, U, prbs = int(os.environ.get("NRX_STAMP_B", 128)), 2, int(os.environ.get("NRX_STAMP_PRBS", 4))
sl = synth.generate(B, U, prbs, 4, [4, 4], (0, 1), snr_db=10, seed=3)
eng = CGNNEngine(spec, W.load("nrx_rt"))
t = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
pe = t(compute_pe(U, 48, (2, 11), (0, 1)))
dy, dh, da = t(sl.y), t(sl.h_hat), t(sl.active)
for _ in range(300):
    eng.forward(dy, pe, dh, da, None, 2, "f16")
torch.cuda.synchronize()
n = 512
buf = np.zeros((n, 64), np.uint64)
lib.nrx_debug_stamps(buf.ctypes.data, n)
buf = buf.astype(np.int64)
used = buf[:, 5] > 0
buf = buf[used]
st0 = buf[:, 0:1]
rel = buf - st0
print("launch", os.environ.get("NRX_STAMP_LAUNCH", "0"), f"workgroups {used.sum()}")
order = [("init: loads issued", 33), ("init: slot norm", 36), ("init: z stored", 37), ("init: w1 stored", 39),
         ("pair: next z DMA issue", 30), ("pair: DMA issued", 31), ("pair: item 1 done", 32),
         ("dma issue start", 24), ("dma issued", 25), ("conv1 start", 1), ("conv1 end", 2), ("conv2 end", 3),
         ("epilogue start", 6), ("item 1 end", 4), ("item 2 start", 26), ("item 2 data in", 27),
         ("item 2 block", 28), ("item 2 conv1 end", 34), ("item 2 conv2 end", 35),
         ("item 2 epilogue", 38), ("item 2 end", 29), ("kernel end", 5)]
prev = 0.0
for name, k in order:
    v = rel[:, k]
    ok = buf[:, k] > 0
    if not ok.any():
        continue
    m = v[ok].mean()
    print(f"  {name:18s} @{m:9.0f}  (+{m - prev:7.0f})  max {v[ok].max():9.0f}")
    prev = m
det = rel[:, 8:23].reshape(-1, 3, 5)
for L in range(3):
    seg = np.diff(det[:, L, :], axis=1)
    print(f"  (last item) conv{L + 1}: math {seg[:, 0].mean():7.0f}  bar1 {seg[:, 1].mean():7.0f}  "
          f"post {seg[:, 2].mean():7.0f}  epi {seg[:, 3].mean():7.0f}")
# per-wave conv1 stamps (last item of the workgroup): 40+w math end, 48+w early rows stored
# (before the layer barrier), 56+w rows 0,1 stored; relative to wave 0's conv1 math start (8)
if (buf[:, 40:64] > 0).any():
    base = buf[:, 8:9]
    for k, name in ((40, "math end"), (48, "pre-barrier"), (56, "rows 0,1 stored")):
        v = (buf[:, k:k + 8] - base).mean(axis=0)
        print(f"  conv1 per wave {name:16s}", " ".join(f"{x:7.0f}" for x in v))
    print(f"  conv1 barrier release (stamp 10) {float((buf[:, 10] - buf[:, 8]).mean()):7.0f}")
