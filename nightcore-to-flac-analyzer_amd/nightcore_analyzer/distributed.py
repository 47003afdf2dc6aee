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


RUN_KWARGS = ("window_sec", "hop_sec", "energy_gate_db", "silence_strip_db", "src_trim_sec", "auto_align",
              "compute_pitch", "compute_ibi", "log")          # pipeline.run_batch's keyword arguments


def run_batch_distributed(pairs: Sequence, analyze_fn: Optional[Callable] = None, group=None,
                          shard: Optional[str] = None, split_offset: float = 0.0, **kwargs) -> list:
    """Every rank returns all results (AnalysisResult, or the exception run() raises) in
    input order.  ``shard`` = "pairs" | "windows" | None (windows when there are fewer
    pairs than ranks).  ``analyze_fn(pairs, **kwargs)`` (pair mode) defaults to
    pipeline.run_batch; window mode takes pipeline.run_batch's keyword arguments (``log``
    receives every pair's lines, prefixed "[pair i] ", after the run).  In both modes a
    failure of the run itself (a file that does not decode, a device error) comes back as
    the result of the pairs it hit — in window mode, where a pair's items span ranks, as
    the result of every pair — instead of raising."""
    if shard not in (None, "pairs", "windows"):
        raise ValueError(f"shard must be 'pairs', 'windows' or None, not {shard!r}")
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    mode = shard or ("windows" if 0 < len(pairs) < world and analyze_fn is None else "pairs")
    if mode == "windows":
        if analyze_fn is not None:
            raise ValueError("analyze_fn applies to pair mode only")
        unknown = sorted(set(kwargs) - set(RUN_KWARGS))
        if unknown:
            raise TypeError(f"run_batch_distributed() got unexpected keyword arguments {unknown}")
        return _run_windows(pairs, group, world, rank, split_offset, **kwargs)
    if analyze_fn is None:
        from .pipeline import run_batch as analyze_fn
    lo, hi = shard_range(len(pairs), world, rank)
    try:
        local = analyze_fn(list(pairs[lo:hi]), **kwargs) if hi > lo else []
    except Exception as exc:           # noqa: BLE001 - delivered as this rank's results
        local = [exc] * (hi - lo)
    return gather_results(local, world, group)


def _run_windows(pairs, group, world, rank, split_offset, log=None, **kw) -> list:
    """Window mode of run_batch_distributed: plan from the files' lengths, decode and
    upload only the pairs this rank touches (sharded.run over DeviceStages)."""
    from .engine import Params, get_engine
    from .io import decoded_length
    from .pipeline import _load, _melodia_hook
    from .sharded import DeviceStages, Exchange, ShardError, analyze_sharded, shard_plan
    p = Params(**kw)
    quiet = (lambda m: None)
    ex = Exchange(group)
    outs, err = None, None
    try:
        lengths = [decoded_length(x) for nc, src in pairs for x in (nc, src)]
        touched = shard_plan(lengths, p, world, split_offset).needed(rank, p.compute_ibi and world > 1)
        arrays = [a for b in touched for a in (_load(pairs[b][0], quiet, "nightcore"),
                                                _load(pairs[b][1], quiet, "source"))]
        if p.compute_pitch:
            # MELODIA where essentia is installed, as run_batch does; the hook is called with
            # global pair indices (sharded.analyze_sharded maps the engine's local ones)
            p.melodia = _melodia_hook({b: (arrays[2 * i], arrays[2 * i + 1]) for i, b in enumerate(touched)})
        eng = get_engine()
        sig = eng.upload_signals(arrays) if arrays else None
    except Exception as exc:           # noqa: BLE001 - carried to every rank below
        err = exc
    try:
        ex.check(err)                  # every rank decoded its pairs, or all stop here
        if sig is None:
            from .engine import DeviceSignals
            import numpy as np
            import torch
            sig = DeviceSignals(torch.zeros(64, device=eng.dev), np.zeros(0, np.int64), np.zeros(0, np.int64))
        outs = analyze_sharded(DeviceStages(eng, sig), p, group, lengths=lengths, local_pairs=touched,
                               split_offset=split_offset)
    except Exception as exc:           # noqa: BLE001 - delivered as every pair's result
        err = exc
    # the same list on every rank: a failed run is every pair's result, with the failing
    # rank's own exception (the others raised ShardError)
    errs = gather_results([err], world, group)
    if any(e is not None for e in errs):
        first = next((e for e in errs if e is not None and not isinstance(e, ShardError)),
                     next(e for e in errs if e is not None))
        return [first] * len(pairs)
    if log is not None:
        for i, o in enumerate(outs):
            for line in o.logs:
                log(f"[pair {i}] {line}")
    return [o.error if o.error is not None else o.result for o in outs]
