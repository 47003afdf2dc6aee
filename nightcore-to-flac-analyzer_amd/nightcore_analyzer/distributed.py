"""Multi-GPU execution: one process per GPU (torch.distributed; backend "nccl" is RCCL
on ROCm).

Two ways to split a batch of (nightcore, source) pairs over the ranks:

* **pairs** (``run_batch_distributed``, the default when there are at least as many
  pairs as ranks): pairs are independent objects, so each rank analyses a contiguous
  block of whole pairs with the single-GPU engine and no data-path collective at all
  (weak scaling); only the finished results are gathered to every rank.
  A rank whose analysis raises contributes the exception as the result of each of its
  pairs, so the gather never waits on a rank that died.
* **windows** (``sharded.analyze_sharded``, used when there are fewer pairs than ranks,
  or on request): the 10 s windows and 20 s chunk pairs of the batch are split over
  the ranks, with all-gathers of the per-window records before the nc prior and
  before consensus, so a single pair spans GPUs (north_star).
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


def run_batch_distributed(pairs: Sequence, analyze_fn: Optional[Callable] = None, group=None,
                          shard: Optional[str] = None, **kwargs) -> list:
    """Every rank returns all results (AnalysisResult, or the exception run() raises) in
    input order.  ``shard`` = "pairs" | "windows" | None (windows when there are fewer
    pairs than ranks).  ``analyze_fn(pairs, **kwargs)`` (pair mode) defaults to
    pipeline.run_batch."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    mode = shard or ("windows" if 0 < len(pairs) < world and analyze_fn is None else "pairs")
    if mode == "windows":
        from .engine import Params
        from .pipeline import _load
        from .sharded import run_window_sharded
        quiet = (lambda m: None)
        arrays = [(_load(n, quiet, "nightcore"), _load(s, quiet, "source")) for n, s in pairs]
        keys = ("window_sec", "hop_sec", "energy_gate_db", "silence_strip_db", "src_trim_sec", "auto_align",
                "compute_pitch", "compute_ibi")
        p = Params(**{k: v for k, v in kwargs.items() if k in keys})
        outs = run_window_sharded(arrays, p, group)
        return [o.error if o.error is not None else o.result for o in outs]
    if analyze_fn is None:
        from .pipeline import run_batch as analyze_fn
    lo, hi = shard_range(len(pairs), world, rank)
    try:
        local = analyze_fn(list(pairs[lo:hi]), **kwargs) if hi > lo else []
    except Exception as exc:           # noqa: BLE001 - delivered as this rank's results
        local = [exc] * (hi - lo)
    return gather_results(local, world, group)
