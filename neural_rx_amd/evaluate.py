"""Monte-Carlo evaluation of the neural receiver, all on the GPU.

The counterpart of the reference's ``scripts/evaluate.py`` NRX leg (evaluate.py:154-207:
``E2E_Model`` + ``load_weights`` + ``num_it = num_nrx_iter_eval`` + Sionna ``sim_ber``),
with the pieces that exist here: the GPU slot generator (``generator.SlotGenerator``),
the CGNN engine, the GPU error counters, and -- across ranks -- one RCCL
``all_reduce(SUM)`` of the int64 counters every ``sync_every`` Monte-Carlo iterations
(the analogue of ``sim_ber(distribute="all")``, evaluate.py:61).  Between those
reductions nothing leaves the device: the counters accumulate in HBM and the host runs
ahead, so a sharded run pays one collective + one host sync per window, not per batch.  Counts are uncoded (no LDPC here): BER
of hard decisions on the LLRs and the fraction of (slot, user) grids with any bit error.

sim_ber semantics kept: per Eb/N0 point iterate until ``max_mc_iter`` or until
``num_target_block_errors`` block errors (tested at each reduction, so a point may run
up to ``sync_every - 1`` batches past the target); ``early_stop`` ends the sweep at the first
point without errors; ``target_bler`` ends it once the BLER falls below the target.

    python -m neural_rx_amd.evaluate -config_name nrx_rt -num_tx_eval 2 \
        -ebno_db 0 2 4 6 8 -batch_size 128 -max_mc_iter 50
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import time
from typing import List, Optional, Sequence

import numpy as np

from .config import dmrs_symbols, get_config
from .generator import GenParams, SlotGenerator, count_errors, ebno_to_no
from .receiver import CGNNEngine, compute_pe, spec_for


@dataclasses.dataclass
class SimResult:
    ebno_db: List[float]
    ber: List[float]
    bler: List[float]
    counts: List[List[int]]          # per point [bit_errors, bits, block_errors, blocks]
    mc_iters: List[int]
    seconds: float
    slots: int

    def as_dict(self):
        return dataclasses.asdict(self)


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def sim_ber(engine: CGNNEngine, gen: SlotGenerator, ebno_dbs: Sequence[float], batch_size: int,
            max_mc_iter: int = 100, num_target_block_errors: int = 100, target_bler: Optional[float] = None,
            early_stop: bool = True, num_it: Optional[int] = None, precision: str = "f16",
            verbose: bool = False, sync_every: int = 8) -> SimResult:
    """Sionna ``sim_ber`` loop on the GPU (this rank's shard of every Monte-Carlo batch:
    global slot ``(it * world + rank) * batch_size + b``).  The counters are reduced
    over ranks (and copied to the host) every ``sync_every`` batches and at the end of a
    point; every rank runs the same number of batches, so the collectives pair up."""
    import torch
    dist = _dist()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    # gloo (CPU tests, or ranks sharing one device) reduces host tensors; nccl = RCCL
    host_reduce = dist is not None and dist.get_backend() != "nccl"
    sync_every = max(1, int(sync_every))
    p = gen.p
    dev = torch.device(f"cuda:{gen.device}")
    pe = torch.from_numpy(compute_pe(p.num_tx, p.num_subcarriers, p.dmrs_symbols, p.cdm_group)).to(dev)
    spec = engine.spec
    llr_out = engine.alloc_outputs(batch_size, p.num_tx, p.num_subcarriers, want_h=False)
    res = SimResult([], [], [], [], [], 0.0, 0)
    t0 = time.perf_counter()
    point_seed = 0
    for ebno in ebno_dbs:
        no = ebno_to_no(float(ebno), len(p.dmrs_symbols))
        counts = torch.zeros((p.num_tx, 4), dtype=torch.int64, device=dev)
        total = np.zeros(4, np.int64)
        it = 0
        while it < max_mc_iter:
            off = ((point_seed * max_mc_iter + it) * world + rank) * batch_size
            sb = gen(batch_size, no, slot_offset=off)
            mcs_mask = sb.mcs_mask if spec.num_mcs > 1 else None
            llr, _ = engine.forward(sb.y, pe, sb.h_hat, sb.active, mcs_mask=mcs_mask, num_it=num_it,
                                    precision=precision, out=llr_out, want_h=False)
            count_errors(llr, sb.bits, sb.active, sb.mcs, p.mcs_bits, p.dmrs_symbols, counts=counts)
            it += 1
            if it % sync_every and it < max_mc_iter:
                continue
            # the one-launch forward's error word: a timed-out or incomplete forward raises here
            # instead of entering the counts (include/nrx.h nrx_fused_status)
            engine.check()
            tot = counts.sum(0)
            if host_reduce:
                tot = tot.cpu()
            if dist:
                dist.all_reduce(tot)
            total = tot.cpu().numpy()
            if total[2] >= num_target_block_errors:
                break
        ber = total[0] / total[1] if total[1] else float("nan")
        bler = total[2] / total[3] if total[3] else float("nan")
        res.ebno_db.append(float(ebno))
        res.ber.append(float(ber))
        res.bler.append(float(bler))
        res.counts.append([int(v) for v in total])
        res.mc_iters.append(it)
        res.slots += it * batch_size * world
        if verbose and rank == 0:
            print(f"EbNo {ebno:6.2f} dB  BER {ber:.4e}  BLER(uncoded) {bler:.4e}  "
                  f"bit errors {total[0]}  blocks {total[3]}  iters {it}", flush=True)
        point_seed += 1
        if early_stop and total[0] == 0:
            break
        if target_bler is not None and bler < target_bler:
            break
    torch.cuda.synchronize(dev)
    res.seconds = time.perf_counter() - t0
    return res


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("-config_name", default="nrx_rt")
    ap.add_argument("-num_tx_eval", type=int, default=None, help="active DMRS ports per slot")
    ap.add_argument("-num_prbs", type=int, default=None)
    ap.add_argument("-ebno_db", type=float, nargs="+", default=None)
    ap.add_argument("-batch_size", type=int, default=128)
    ap.add_argument("-max_mc_iter", type=int, default=100)
    ap.add_argument("-num_target_block_errors", type=int, default=500)
    ap.add_argument("-target_bler", type=float, default=None)
    ap.add_argument("-var_mcs", action="store_true", help="draw the MCS of every (slot, user)")
    ap.add_argument("-precision", default="f16")
    ap.add_argument("-seed", type=int, default=1234)
    ap.add_argument("-sync_every", type=int, default=8, help="MC batches per counter all-reduce")
    ap.add_argument("-gpu", type=int, default=None)
    ap.add_argument("-out", default=None, help="write the result JSON here")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = a.gpu if a.gpu is not None else local
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{device}"))
    cfg = get_config(a.config_name)
    spec = spec_for(cfg)
    from . import weights as W
    engine = CGNNEngine(spec, W.load(cfg.label), device=device)
    u = cfg.max_num_tx
    params = GenParams.from_config(cfg, num_tx=u, num_prbs=a.num_prbs, var_mcs=a.var_mcs, seed=a.seed)
    params.num_active = a.num_tx_eval or u
    gen = SlotGenerator(params, device=device)
    ebno = a.ebno_db if a.ebno_db is not None else list(np.arange(-2.0, 8.0, 1.0))
    res = sim_ber(engine, gen, ebno, a.batch_size, a.max_mc_iter, a.num_target_block_errors, a.target_bler,
                  num_it=cfg.num_nrx_iter_eval, precision=a.precision, verbose=True, sync_every=a.sync_every)
    if rank == 0:
        d = res.as_dict()
        d.update(config=cfg.label, num_tx_eval=params.num_active, dmrs_symbols=list(dmrs_symbols(cfg)),
                 world=world, slots_per_s=res.slots / res.seconds)
        print(json.dumps(d))
        if a.out:
            with open(a.out, "w") as f:
                json.dump(d, f)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
