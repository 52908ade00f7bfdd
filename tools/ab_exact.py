"""Diagnostic: dump f16 forward outputs of the library named by NRX_LIB_PATH (bench
workload + U = 1 + an inactive user) so that two kernel variants can be compared bit for
bit.  usage: NRX_LIB_PATH=... python tools/ab_exact.py out.npz ; python tools/ab_exact.py --cmp a.npz b.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if sys.argv[1] == "--cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    for k in a.files:
        same = np.array_equal(a[k], b[k])
        print(k, "bit-identical" if same else f"DIFFERENT max|d|={np.abs(a[k] - b[k]).max():.3e}")
    sys.exit(0)

import torch
from neural_rx_amd import synth, weights as W
from neural_rx_amd.config import get_config, spec_from_config, dmrs_symbols, user_cdm_groups
from neural_rx_amd.receiver import CGNNEngine, compute_pe

cfg = get_config("nrx_rt")
spec = spec_from_config(cfg)
eng = CGNNEngine(spec, W.load("nrx_rt"))
out = {}
for tag, B, U, prbs, act in (("b128u2", 128, 2, 4, None), ("b2u1", 2, 1, 4, None),
                             ("b2u2_inactive", 2, 2, 4, [[1, 0], [0, 1]]), ("b3u2_f50", 3, 2, 4, None)):
    groups = user_cdm_groups(cfg, U)
    sl = synth.generate(B, U, prbs, 4, [4] * U, groups, dmrs_symbols(cfg), snr_db=10, seed=5,
                        active=None if act is None else np.array(act, np.float32))
    y, h, F = sl.y, sl.h_hat, 12 * prbs
    if tag.endswith("f50"):
        rng = np.random.default_rng(9)
        F = 50
        y = rng.standard_normal((B, F, 14, 8)).astype(np.float32)
        h = rng.standard_normal((B, U, F, 14, 8)).astype(np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()
    pe = t(compute_pe(U, F, dmrs_symbols(cfg), groups))
    llr, hr = eng.forward(t(y), pe, t(h), t(sl.active), None, 2, "f16")
    torch.cuda.synchronize()
    out[tag + "_llr"] = llr.cpu().numpy()
    out[tag + "_h"] = hr.cpu().numpy()
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1])
