"""The data-parallel evaluation loop as product code: two ranks on one GPU (needs an MI355X).

Reference analogue: Sionna ``sim_ber(distribute="all")`` (scripts/evaluate.py:61,
193-202) -- every replica runs the receiver on its own slots and the error counters are
summed.  Here two processes share device 0 (gloo carries the counter reduction, since
RCCL needs one device per rank) and each runs the real ``evaluate.sim_ber``: GPU slot
generator -> CGNN engine (libnrx.so) -> ``nrx_count_errors``, with the counters reduced
every ``sync_every`` batches.  The summed counters must equal ONE process evaluating the
same global slot indices (batch 2B per Monte-Carlo iteration): every draw of the
generator is a function of the global slot index and the engine's output for a slot does
not depend on the batch it runs in.

The ranks are spawned when this module is set up.  The file name sorts before every other
GPU test module, so the pytest process has not initialised the GPU yet at that point
(children are started as fresh interpreters, never by replacing a GPU process).
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

B = 32          # slots per rank per Monte-Carlo iteration
MAX_IT = 5      # not a multiple of SYNC: the last window is partial
SYNC = 2
EBNO = [2.0, 6.0]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_sim(world_batch):
    from neural_rx_amd import weights as W
    from neural_rx_amd.config import get_config
    from neural_rx_amd.evaluate import sim_ber
    from neural_rx_amd.generator import GenParams, SlotGenerator
    from neural_rx_amd.receiver import CGNNEngine, spec_for
    cfg = get_config("nrx_rt")
    eng = CGNNEngine(spec_for(cfg), W.load(cfg.label), device=0)
    gen = SlotGenerator(GenParams.from_config(cfg, num_tx=2, num_prbs=4, seed=99), device=0)
    res = sim_ber(eng, gen, EBNO, world_batch, max_mc_iter=MAX_IT, num_target_block_errors=10 ** 9,
                  early_stop=False, num_it=cfg.num_nrx_iter_eval, precision="f16", sync_every=SYNC)
    return res.counts, res.mc_iters


def _rank(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        counts, iters = _run_sim(B)
        q.put((rank, counts, iters, None))
        dist.destroy_process_group()
    except Exception as e:          # report instead of hanging the parent
        q.put((rank, None, None, repr(e)))


@pytest.fixture(scope="module")
def two_ranks():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        out = [q.get(timeout=300) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return {r: (c, i, err) for r, c, i, err in out}


def test_two_ranks_on_one_gpu_match_single_process(two_ranks):
    for r in (0, 1):
        assert two_ranks[r][2] is None, two_ranks[r][2]
    c0, i0, _ = two_ranks[0]
    c1, i1, _ = two_ranks[1]
    assert c0 == c1 and i0 == i1 == [MAX_IT] * len(EBNO)
    single, iters = _run_sim(2 * B)
    assert iters == [MAX_IT] * len(EBNO)
    assert c0 == single, (c0, single)
    # bits counted: every data RE of every active (slot, user) over both points
    tot = np.asarray(single)
    assert (tot[:, 3] > 0).all() and (tot[:, 1] > 0).all()
