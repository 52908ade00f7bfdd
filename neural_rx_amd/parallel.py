"""Data parallelism for the receiver: slots shard over ranks, RCCL only for statistics.

The reference's only parallel mode is Sionna's ``sim_ber(distribute="all")`` (a TF
MirroredStrategy, scripts/evaluate.py:61, 76-82, 199): every replica runs the
receiver on its own slots and the error counters are summed.  Here each process owns
one GPU and a contiguous shard of the slot batch; the forward pass has no collective;
after a measurement window one ``all_reduce(SUM)`` of four int64 counters
``[bit_errors, bits, block_errors, blocks]`` (and a MAX of the elapsed time) crosses
the ranks -- over RCCL/xGMI (backend "nccl") on MI355X, or gloo on CPU for tests.
"""
from __future__ import annotations

import dataclasses
from typing import Callable, Optional, Tuple

import numpy as np


def shard_range(batch: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous split of ``batch`` slots over ``world`` ranks (sizes differ by <= 1)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, rem = divmod(batch, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


@dataclasses.dataclass
class ErrorCounters:
    bit_errors: int = 0
    bits: int = 0
    block_errors: int = 0
    blocks: int = 0

    def add(self, other: "ErrorCounters"):
        self.bit_errors += other.bit_errors
        self.bits += other.bits
        self.block_errors += other.block_errors
        self.blocks += other.blocks

    @property
    def ber(self) -> float:
        return self.bit_errors / self.bits if self.bits else float("nan")

    @property
    def bler(self) -> float:
        return self.block_errors / self.blocks if self.blocks else float("nan")

    def as_array(self) -> np.ndarray:
        return np.array([self.bit_errors, self.bits, self.block_errors, self.blocks], np.int64)


def count_errors(llr: np.ndarray, bits: np.ndarray, data_mask: np.ndarray,
                 active: Optional[np.ndarray] = None) -> ErrorCounters:
    """Uncoded hard-decision errors (Sionna LLR sign: > 0 decides 1).  A block is one
    (slot, user) codeword-less resource grid here (uncoded BLER proxy).
    llr/bits: [B, U, F, T, bits]."""
    hard = (llr[:, :, :, data_mask] > 0)
    ref = bits[:, :, :, data_mask].astype(bool)
    err = hard != ref
    if active is not None:
        keep = active > 0
        err = err[keep]
        nbits = int(np.prod(err.shape))
        blk = err.reshape(err.shape[0], -1).any(axis=1)
    else:
        nbits = int(err.size)
        blk = err.reshape(err.shape[0] * err.shape[1], -1).any(axis=1)
    return ErrorCounters(int(err.sum()), nbits, int(blk.sum()), int(blk.size))


def all_reduce_counters(c: ErrorCounters, device=None) -> ErrorCounters:
    """SUM the counters over the default process group (no-op when not initialised)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return c
    t = torch.tensor(c.as_array(), dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    v = t.cpu().numpy()
    return ErrorCounters(int(v[0]), int(v[1]), int(v[2]), int(v[3]))


def all_reduce_max(x: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def evaluate_sharded(receiver: Callable, make_slots: Callable, batch: int, rank: int, world: int,
                     device=None) -> ErrorCounters:
    """One data-parallel evaluation window: this rank generates/receives its shard of the
    batch (``make_slots(lo, hi)`` -> object with y/h_hat/active/bits/data_mask), runs
    ``receiver(slots) -> llr [B,U,F,T,bits]`` on it and the counters are summed over
    ranks.  Mirrors sim_ber's replica loop (evaluate.py:193-202)."""
    lo, hi = shard_range(batch, world, rank)
    local = ErrorCounters()
    if hi > lo:
        slots = make_slots(lo, hi)
        llr = np.asarray(receiver(slots))
        nb = llr.shape[-1]
        local = count_errors(llr, slots.bits[..., :nb], slots.data_mask, slots.active)
    return all_reduce_counters(local, device)
