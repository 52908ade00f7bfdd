"""Diagnostic (GPU): where the register-resident update launch departs from the strip kernels.
Runs the bench shape with update_schedule(False / True) at num_it = 1 and 2 and compares the
outputs and the workspace's state planes; prints the first mismatching (slot, user, f, t, channel)
of each plane and a histogram of mismatching f mod 16 and t."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests.helpers import make_case  # noqa: E402
from neural_rx_amd.receiver import CGNNEngine  # noqa: E402

case = make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=12, seed=51)
B, U, F = 128, 2, 48
eng = CGNNEngine(case.spec, case.weights)
eng.fused_config(enable=False)
dev = "cuda:0"
t = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(dev)
args = [t(case.y), t(case.pe), t(case.h_hat), t(case.active), t(case.mcs_mask)]
plane = B * U * F * 14 * 56


def run(rr, num_it):
    eng.update_schedule(rr)
    llr, h = eng.forward(*args, num_it=num_it, precision="f16")
    torch.cuda.synchronize()
    ws = eng._ws["buf"].clone().cpu().numpy()
    off = ((B * 8 + 255) // 256) * 256
    pl = []
    for k in range(5):
        pl.append(ws[off + 2 * plane * k: off + 2 * plane * (k + 1)].view(np.float16).reshape(B if k < 4 else 1, U if k < 4 else U, F, 14, 56)
                  if k < 4 else ws[off + 2 * plane * 4: off + 2 * plane * 4 + 2 * U * F * 14 * 56].view(np.float16).reshape(U, F, 14, 56))
    return llr.cpu().numpy(), h.cpu().numpy(), pl


for num_it in (1, 2):
    a = run(False, num_it)
    b = run(True, num_it)
    print(f"num_it {num_it}: llr maxdiff {np.abs(a[0] - b[0]).max():.4g}  h maxdiff {np.abs(a[1] - b[1]).max():.4g}")
    d = np.argwhere(a[0] != b[0])
    if len(d):
        print("   llr mismatches", len(d), "first", d[:3].tolist(), "f mod 16 hist", np.bincount(d[:, 3] % 16, minlength=16).tolist(),
              "t hist", np.bincount(d[:, 4], minlength=14).tolist())
    for k, name in enumerate(["s_out", "s_in", "a_out", "a", "pe16"]):
        x, y = a[2][k].astype(np.float32), b[2][k].astype(np.float32)
        bad = ~((x == y) | (np.isnan(x) & np.isnan(y)))
        if bad.any():
            w = np.argwhere(bad)
            print(f"   {name}: {bad.sum()} mismatches, max {np.nanmax(np.abs(x - y)):.4g}, first {w[:3].tolist()}")
            print("      f mod 16", np.bincount(w[:, -3] % 16, minlength=16).tolist(), " t", np.bincount(w[:, -2], minlength=14).tolist(),
                  " c//8", np.bincount(w[:, -1] // 8, minlength=7).tolist(), " u", np.bincount(w[:, 1], minlength=U).tolist() if name != "pe16" else "")
        else:
            print(f"   {name}: identical")
