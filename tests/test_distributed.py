"""Data-parallel slot sharding + counter all-reduce, world_size 2 over gloo (CPU)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from neural_rx_amd.parallel import ErrorCounters, count_errors, shard_range


def test_shard_range_partitions():
    for batch in (1, 7, 128, 1024):
        for world in (1, 2, 3, 8):
            spans = [shard_range(batch, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == batch
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from neural_rx_amd import parallel, synth
    from tests.helpers import make_case, run_oracle

    full = make_case("nrx_rt", batch=6, users=2, prbs=1, snr_db=12, seed=21)

    def make_slots(lo, hi):
        class S:
            pass
        s = S()
        s.y, s.h_hat = full.y[lo:hi], full.h_hat[lo:hi]
        s.active, s.bits, s.data_mask = full.active[lo:hi], full.slots.bits[lo:hi], full.slots.data_mask
        s.mask = full.mcs_mask[lo:hi]
        return s

    def receiver(s):
        # the numpy oracle stands in for the engine: this test checks the plumbing
        from oracle import cgnn_ref
        w = cgnn_ref.split_keras_weights(full.weights, full.spec)
        return cgnn_ref.cgnn_forward(s.y, full.pe, s.h_hat, s.active, s.mask, w, full.spec)["llr"][0]

    c = parallel.evaluate_sharded(receiver, make_slots, 6, rank, world)
    q.put((rank, c.as_array().tolist()))
    dist.destroy_process_group()


def test_gloo_two_ranks_match_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0] == res[1]
    # single-process reference count over the whole batch
    from tests.helpers import make_case, run_oracle
    full = make_case("nrx_rt", batch=6, users=2, prbs=1, snr_db=12, seed=21)
    llr = run_oracle(full)["llr"][0]
    c = count_errors(llr, full.slots.bits[..., :4], full.slots.data_mask, full.active)
    assert res[0] == c.as_array().tolist()
    assert c.bits == 6 * 2 * 12 * 12 * 4
