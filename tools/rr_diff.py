"""Bisect the register-resident kernels against the strip kernels (diagnostic): one case,
NRX_RR launch masks 0 (strip kernels) / 1 / 2 / 4 / 7, LLR + h_ref differences per mask and
where they sit (subcarrier f, symbol t, slot, user)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from tests.helpers import make_case
from neural_rx_amd.receiver import CGNNEngine

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
case = make_case("nrx_rt", batch=B, users=2, prbs=4, snr_db=12, seed=22)
eng = CGNNEngine(case.spec, case.weights)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()
res = {}
for mask in (0, 1, 2, 4, 7):
    os.environ["NRX_RR"] = str(mask)
    for nit in (1, 2):
        llr, h = eng.forward(t(case.y), t(case.pe), t(case.h_hat), t(case.active), None, nit, "f16")
        torch.cuda.synchronize()
        res[(mask, nit)] = (llr.cpu().numpy().copy(), h.cpu().numpy().copy())
for nit in (1, 2):
    l0, h0 = res[(0, nit)]
    for mask in (1, 2, 4, 7):
        l, h = res[(mask, nit)]
        d = np.abs(l - l0)[0]          # [B, U, F, T, bits]
        print(f"num_it {nit} mask {mask}: llr maxdiff {d.max():.4g} mean {d.mean():.4g} frac!=0 {(d > 0).mean():.3f}  "
              f"h maxdiff {np.abs(h - h0).max():.4g}", flush=True)
        if d.max() > 0:
            per_f = d.max(axis=(0, 1, 3, 4))
            per_t = d.max(axis=(0, 1, 2, 4))
            per_b = d.max(axis=(1, 2, 3, 4))
            print("   per f:", np.array2string(per_f, precision=2, max_line_width=250))
            print("   per t:", np.array2string(per_t, precision=2, max_line_width=250))
            print("   slots with diff:", int((per_b > 0).sum()), "of", B, " users:", d.max(axis=(0, 2, 3, 4)))
