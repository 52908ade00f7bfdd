"""Feasibility probe: does a memory-bound kernel on a second stream run beside the RR update
launches (one 512-thread workgroup per CU, ~240 VGPRs per wave: 2 waves per SIMD)?

Times (a) the forward alone, (b) an HBM-bound torch elementwise stream alone, (c) both issued
on two streams, (d) both on one stream.  (c) ~ max(a, b) means the second stream's waves found
room on the CUs; (c) ~ (d) means no concurrency."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from neural_rx_amd import synth, weights as W  # noqa: E402
from neural_rx_amd.config import get_config, spec_from_config  # noqa: E402
from neural_rx_amd.receiver import CGNNEngine, compute_pe  # noqa: E402

B, U, prbs = 6, 8, 273
cfg = get_config("nrx_rt")
spec = spec_from_config(cfg)
groups = tuple(i % 2 for i in range(U))
sl = synth.generate(B, U, prbs, 4, [4] * U, groups, snr_db=10, seed=3)
eng = CGNNEngine(spec, W.load("nrx_rt"))
t = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
pe = t(compute_pe(U, 12 * prbs, (2, 11), groups))
dy, dh, da = t(sl.y), t(sl.h_hat), t(sl.active)
out = eng.alloc_outputs(B, U, 12 * prbs)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
x = torch.empty(100 * 1024 * 1024, dtype=torch.float32, device="cuda").uniform_()
y = torch.empty_like(x)


def fwd(n):
    for _ in range(n):
        eng.forward(dy, pe, dh, da, None, 2, "f16", out=out)


def mem(n):
    for _ in range(n):
        torch.mul(x, 1.0001, out=y)


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


NF, NM = 20, 60
with torch.cuda.stream(sa):
    fwd(3)
    mem(3)
torch.cuda.synchronize()
for rep in range(2):
    with torch.cuda.stream(sa):
        ta = timed(lambda: fwd(NF))
        tb = timed(lambda: mem(NM))
        td = timed(lambda: (fwd(NF), mem(NM)))

    def both():
        with torch.cuda.stream(sa):
            fwd(NF)
        with torch.cuda.stream(sb):
            mem(NM)
    tc = timed(both)
    print(f"rep {rep}: forward alone {ta:.2f} ms, memory stream alone {tb:.2f} ms, "
          f"two streams {tc:.2f} ms, one stream {td:.2f} ms; overlap saved {ta + tb - tc:.2f} ms")
