"""StateInit outputs (state s and act*sp rows left in the workspace) of the RR vs the strip
kernels (diagnostic)."""
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
U, F = 2, 48
sb = ((B * U * F * 14 * 56 * 2) + 255) // 256 * 256
nb = ((B * 8) + 255) // 256 * 256
out = {}
for mask in (0, 1):
    os.environ["NRX_RR"] = str(mask)
    eng.forward(t(case.y), t(case.pe), t(case.h_hat), t(case.active), None, 1, "f16")
    torch.cuda.synchronize()
    ws = eng._ws["buf"].cpu().numpy()
    s = ws[nb:nb + B * U * F * 14 * 56 * 2].view(np.float16).reshape(B, U, F, 14, 56).astype(np.float32)
    a = ws[nb + 2 * sb:nb + 2 * sb + B * U * F * 14 * 56 * 2].view(np.float16).reshape(B, U, F, 14, 56).astype(np.float32)
    out[mask] = (s, a)
for k, name in ((0, "state s"), (1, "act*sp")):
    d = np.abs(out[1][k] - out[0][k])
    print(f"{name}: maxdiff {d.max():.4g} mean {d.mean():.4g} frac!=0 {(d > 0).mean():.4f} max|ref| {np.abs(out[0][k]).max():.3g}")
    print("  per f:", np.array2string(d.max(axis=(0, 1, 3, 4)), precision=3, max_line_width=250))
    print("  per t:", np.array2string(d.max(axis=(0, 1, 2, 4)), precision=3, max_line_width=250))
    print("  per c:", np.array2string(d.max(axis=(0, 1, 2, 3)), precision=3, max_line_width=250))
    idx = np.unravel_index(np.argmax(d), d.shape)
    print("  argmax", idx, out[0][k][idx], out[1][k][idx])
