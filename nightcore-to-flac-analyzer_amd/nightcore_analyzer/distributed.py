"""Multi-GPU execution: one process per GPU (torch.distributed; backend "nccl"
is RCCL on ROCm), pairs sharded in contiguous blocks across ranks.

(nightcore, source) pairs are independent objects, so the data path has no
collective at all (weak scaling); the only communication is
the final gather of the small per-pair results to every rank (or to rank 0),
a few hundred bytes per pair over xGMI.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch.distributed as dist


def shard_range(n_items: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous block [lo, hi) of items for `rank`; sizes differ by at most one."""
    base, extra = divmod(n_items, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_results(local: list, world: int, group=None) -> list:
    """Concatenate every rank's list in rank order (all ranks get the full list)."""
    if world == 1:
        return list(local)
    buf: List[Optional[list]] = [None] * world
    dist.all_gather_object(buf, local, group=group)
    out: list = []
    for part in buf:
        out.extend(part)
    return out


def run_batch_distributed(pairs: Sequence, analyze_fn: Optional[Callable] = None, group=None, **kwargs) -> list:
    """Each rank analyses its block of `pairs`; every rank returns all results
    (AnalysisResult or the exception run() would raise) in input order.
    ``analyze_fn(pairs, **kwargs)`` defaults to pipeline.run_batch."""
    if analyze_fn is None:
        from .pipeline import run_batch as analyze_fn
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    lo, hi = shard_range(len(pairs), world, rank)
    local = analyze_fn(list(pairs[lo:hi]), **kwargs) if hi > lo else []
    return gather_results(local, world, group)
