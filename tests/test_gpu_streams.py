"""The throughput pipeline bench.py runs: consecutive batches alternated over two HIP streams, one
engine (handle + workspace + outputs) per stream, so that a kernel's last waves overlap the next
batch's launch.  Batches in flight share no buffer, so every batch's LLRs / h_ref must equal, bit
for bit, the same batch run alone on one stream."""
import numpy as np
import pytest

from tests.helpers import make_case, run_engine

pytestmark = pytest.mark.gpu


def test_two_stream_pipeline_equals_one_stream():
    import torch
    from neural_rx_amd.receiver import CGNNEngine
    cases = [make_case("nrx_rt", batch=128, users=2, prbs=4, snr_db=8 + i, seed=90 + i) for i in range(4)]
    ref_eng = CGNNEngine(cases[0].spec, cases[0].weights)
    try:
        refs = [run_engine(c, "f16", ref_eng) for c in cases]
    finally:
        ref_eng.close()
    engs = [CGNNEngine(cases[0].spec, cases[0].weights) for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, np.float32)).cuda()
    try:
        ins = [(dev(c.y), dev(c.pe), dev(c.h_hat), dev(c.active), None if c.mcs_mask is None else dev(c.mcs_mask))
               for c in cases]
        outs = [engs[i % 2].alloc_outputs(128, 2, 48) for i in range(len(cases))]
        torch.cuda.synchronize()
        for rep in range(3):   # several rounds back to back: batches of both streams in flight
            for i, (y, pe, h, a, m) in enumerate(ins):
                engs[i % 2].forward(y, pe, h, a, m, cases[i].num_it, "f16", out=outs[i],
                                    stream=streams[i % 2].cuda_stream)
        torch.cuda.synchronize()
        for i, ref in enumerate(refs):
            assert np.array_equal(outs[i][0].cpu().numpy(), ref["llr_raw"]), i
            assert np.array_equal(outs[i][1].cpu().numpy(), ref["h_hat"]), i
    finally:
        for e in engs:
            e.close()
