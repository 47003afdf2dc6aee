"""Where a window-sharded call's result gather spends its time, per rank: bench.py's own run
(same arguments) with the gather's phases wrapped in wall-clock timers — _StepRecords.add (the
record packing, in the pipeline), _StepRecords.bytes, Exchange.check (the fail-together
collective, which waits for the slowest rank), Exchange.gather_bytes and GatheredOutcomes.table.
Each rank prints every call's phase times (ms) and, at exit, the totals and call counts to stderr.

usage: python -m torch.distributed.run ... tools/gather_phase_probe.py <bench.py arguments>
"""
import atexit
import os
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "nightcore-to-flac-analyzer_amd"))
from nightcore_analyzer import sharded  # noqa: E402

tot = defaultdict(float)
cnt = defaultdict(int)


def wrap(cls, name, tag):
    f = getattr(cls, name)

    def g(*a, **k):
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            tot[tag] += (time.perf_counter() - t) * 1e3
            cnt[tag] += 1
    setattr(cls, name, g)


wrap(sharded._StepRecords, "add", "records.add")
wrap(sharded._StepRecords, "bytes", "records.bytes")
wrap(sharded.Exchange, "check", "exchange.check")
wrap(sharded.Exchange, "gather_bytes", "exchange.gather_bytes")
wrap(sharded.GatheredOutcomes, "table", "outcomes.table")
_inner = sharded._analyze_sharded


def _call(*a, **k):
    before = dict(tot)
    t = time.perf_counter()
    try:
        return _inner(*a, **k)
    finally:
        ms = (time.perf_counter() - t) * 1e3
        d = {n: tot[n] - before.get(n, 0.0) for n in tot}
        print(f"rank {os.environ.get('RANK', '0')} call offset={a[5]} gather={a[6]} "
              f"steps={a[7] if len(a) > 7 else k.get('steps')} {ms:.1f} ms: " +
              ", ".join(f"{n} {v:.1f}" for n, v in sorted(d.items()) if v > 0), file=sys.stderr, flush=True)


sharded._analyze_sharded = _call


@atexit.register
def report():
    rank = os.environ.get("RANK", "0")
    print(f"rank {rank} phases (ms total, calls): " +
          ", ".join(f"{k} {tot[k]:.1f}/{cnt[k]}" for k in sorted(tot)), file=sys.stderr, flush=True)


if __name__ == "__main__":
    import bench
    sys.argv = ["bench.py"] + sys.argv[1:]
    bench.main()
