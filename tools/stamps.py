"""Diagnostic: per-phase cycle shares of k_update (NRX_STAMPS build)."""
import ctypes, os, sys, subprocess
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from neural_rx_amd import build as _B
if not os.path.exists("/tmp/libnrx_stamps.so"):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-DNRX_STAMPS", *_B.SOURCES, "-o", "/tmp/libnrx_stamps.so"], check=True)
import torch
from neural_rx_amd import _lib
lib = _lib.load("/tmp/libnrx_stamps.so")
lib.nrx_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
from neural_rx_amd import synth, weights as W
from neural_rx_amd.config import get_config, spec_from_config, dmrs_symbols, user_cdm_groups
from neural_rx_amd.receiver import CGNNEngine, compute_pe
cfg = get_config("nrx_rt"); spec = spec_from_config(cfg)
B, U, prbs = 128, 2, 4
sl = synth.generate(B, U, prbs, 4, [4, 4], (0, 1), snr_db=10, seed=3)
eng = CGNNEngine(spec, W.load("nrx_rt"))
t = lambda a: torch.from_numpy(a).cuda()
pe = t(compute_pe(U, 48, (2, 11), (0, 1)))
dy, dh, da = t(sl.y), t(sl.h_hat), t(sl.active)
for _ in range(300):
    eng.forward(dy, pe, dh, da, None, 2, "f16")
torch.cuda.synchronize()
n = 512
buf = np.zeros((n, 64), np.uint64)
lib.nrx_debug_stamps(buf.ctypes.data, n)
st = buf[:, [0, 1, 2, 3, 6, 4, 5]].astype(np.int64)
d = np.diff(st, axis=1)
names = ["z-load", "conv1", "conv2", "conv3", "epilogue", "tail"]
launch = os.environ.get("NRX_STAMP_LAUNCH", "0")
print("launch", os.environ.get("NRX_STAMP_LAUNCH", "0"), "(k_update i; -1 = k_init)")
tot = st[:, -1] - st[:, 0]
print("cycles per WG (mean):", tot.mean(), " start spread:", st[:, 0].max() - st[:, 0].min())
for i, nm in enumerate(names):
    print(f"  {nm:10s} mean {d[:, i].mean():9.0f}  ({100 * d[:, i].mean() / tot.mean():5.1f}%)  max {d[:, i].max()}")

# conv_layer detail (wave 0): math | barrier1 | post+pre | epilogue (own rows)
det = buf[:, 8:23].astype(np.int64).reshape(n, 3, 5)
for L in range(3):
    seg = np.diff(det[:, L, :], axis=1)
    print(f"  conv{L + 1}: math {seg[:, 0].mean():7.0f}  bar1 {seg[:, 1].mean():7.0f}  "
          f"post {seg[:, 2].mean():7.0f}  epi {seg[:, 3].mean():7.0f}")
z = buf[:, [0, 24, 25, 26, 27, 1]].astype(np.int64)
zd = np.diff(z, axis=1)
print(f"  z-load: issue {zd[:, 0].mean():7.0f}  zero-fill {zd[:, 1].mean():7.0f}  wait+store {zd[:, 2].mean():7.0f}  "
      f"w-store {zd[:, 3].mean():7.0f}  barrier {zd[:, 4].mean():7.0f}")
