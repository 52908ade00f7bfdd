"""Diagnostic (CPU): error of tools/ab_exact.py dumps against the fp64 oracle on the same
inputs (the b128u2 case on its first 8 slots), so that a kernel variant that is not
bit-identical can be judged on accuracy.  usage: python tools/ab_vs_oracle.py a.npz [b.npz ...]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from neural_rx_amd import synth, weights as W  # noqa: E402
from neural_rx_amd.config import dmrs_symbols, get_config, spec_from_config, user_cdm_groups  # noqa: E402
from neural_rx_amd.receiver import compute_pe  # noqa: E402
from oracle import cgnn_ref  # noqa: E402

cfg = get_config("nrx_rt")
spec = spec_from_config(cfg)
wts = cgnn_ref.split_keras_weights(W.load("nrx_rt"), spec)
ref = {}
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
    n = min(B, 8)
    pe = compute_pe(U, F, dmrs_symbols(cfg), groups)
    o = cgnn_ref.cgnn_forward(y[:n], pe, h[:n], sl.active[:n], np.ones((n, U, 1)), wts, spec, num_it=2)
    ref[tag + "_llr"] = o["llr"][0]
    ref[tag + "_h"] = o["h_hat"]

for path in sys.argv[1:]:
    d = np.load(path)
    print(path)
    for k, r in ref.items():
        g = (d[k][0] if k.endswith("_llr") else d[k])[: r.shape[0]].astype(np.float64)   # llr: [H, B, ...]
        err = g - r
        line = f"  {k:18s} max|d|/max|ref| {np.abs(err).max() / np.abs(r).max():.4f}  rms {np.sqrt((err ** 2).mean() / (r ** 2).mean()):.5f}"
        if k.endswith("_llr"):
            line += f"  flips {np.mean(np.sign(g) != np.sign(r)):.2e}"
        print(line)
