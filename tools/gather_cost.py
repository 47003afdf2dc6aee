#!/usr/bin/env python3
"""Host cost of the window-sharded outcome gather (analyze_sharded gather=True): the 64
outcomes of one config-3 batch rendered (logs), pickled, and unpickled world-1 times, as
all_gather_object does on every rank; plus the pickled size and what dominates it.
    python3 tools/gather_cost.py [world]"""
import pickle
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))


def main():
    import bench
    from nightcore_analyzer import engine as E
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    p = E.Params(compute_ibi=False)
    eng.analyze(signals=sig, params=p)
    from nightcore_analyzer.sharded import _dumps_outcomes
    for rep in range(3):
        outs = eng.analyze(signals=sig, params=p)
        t0 = time.perf_counter()
        blob = _dumps_outcomes(list(enumerate(outs)))
        t1 = time.perf_counter()
        for _ in range(world - 1):
            pickle.loads(blob)
        t2 = time.perf_counter()
        print(f"rep {rep} (round 5, unrendered lines): pickle {1e3 * (t1 - t0):.2f} ms ({len(blob) / 1e6:.2f} MB), "
              f"unpickle x{world - 1} {1e3 * (t2 - t1):.2f} ms", flush=True)
        t0 = time.perf_counter()
        for o in outs:
            o.logs
        t1 = time.perf_counter()
        blob = pickle.dumps(list(enumerate(outs)), protocol=pickle.HIGHEST_PROTOCOL)
        t2 = time.perf_counter()
        for _ in range(world - 1):
            pickle.loads(blob)
        t3 = time.perf_counter()
        print(f"rep {rep} (rendered, as all_gather_object did): logs {1e3 * (t1 - t0):.2f} ms, pickle {1e3 * (t2 - t1):.2f} ms ({len(blob) / 1e6:.2f} MB), "
              f"unpickle x{world - 1} {1e3 * (t3 - t2):.2f} ms", flush=True)
    o = outs[0]
    parts = {"result": o.result, "logs": o.logs, "error": o.error}
    parts.update({f"detail.{k}": v for k, v in o.detail.items()})
    sizes = sorted(((len(pickle.dumps(v, protocol=pickle.HIGHEST_PROTOCOL)), k, type(v).__name__) for k, v in parts.items()),
                   reverse=True)
    print("one outcome, pickled bytes by part:", sizes[:20])
    print("log lines", len(o.logs), "detail keys", list(o.detail))


if __name__ == "__main__":
    main()
