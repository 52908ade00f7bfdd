"""Diagnostic: forwards of the bench workload issued on one stream vs alternated over N streams
(one engine -- handle + workspace -- per stream, so forwards in flight share nothing).  Kernels of
consecutive forwards may then overlap at the launch boundaries (a kernel's last waves and the next
kernel's dispatch).  usage (GPU box): python tools/stream_pipe.py [streams] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from neural_rx_amd import synth, weights as W  # noqa: E402
from neural_rx_amd.config import get_config, spec_from_config  # noqa: E402
from neural_rx_amd.receiver import CGNNEngine, compute_pe  # noqa: E402

NS = int(sys.argv[1]) if len(sys.argv) > 1 else 2
K = int(sys.argv[2]) if len(sys.argv) > 2 else 400
B, U, prbs = 128, 2, 4
cfg = get_config("nrx_rt")
spec = spec_from_config(cfg)
groups = (0, 1)
sl = synth.generate(B, U, prbs, 4, [4] * U, groups, snr_db=10, seed=3)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()
pe = t(compute_pe(U, 12 * prbs, (2, 11), groups))
y, h, act = t(sl.y), t(sl.h_hat), t(sl.active)


def run(ns, steps):
    engs = [CGNNEngine(spec, W.load("nrx_rt")) for _ in range(ns)]
    outs = [e.alloc_outputs(B, U, 12 * prbs) for e in engs]
    sts = [torch.cuda.Stream() for _ in range(ns)]
    def go(n):
        for i in range(n):
            j = i % ns
            engs[j].forward(y, pe, h, act, None, 2, "f16", out=outs[j], stream=sts[j].cuda_stream)
    go(200)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    go(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    llr = [o[0].cpu().numpy() for o in outs]
    for e in engs:
        e.close()
    return steps * B / dt, llr


for rep in range(3):
    v1, l1 = run(1, K)
    vn, ln = run(NS, K)
    same = all(np.array_equal(l1[0], x) for x in ln)
    print(f"rep {rep}: 1 stream {v1:.0f} slots/s, {NS} streams {vn:.0f} slots/s ({vn / v1 - 1:+.1%}), outputs equal: {same}",
          flush=True)
