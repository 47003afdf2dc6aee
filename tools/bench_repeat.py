#!/usr/bin/env python3
"""The bench's timed call (Engine.analyze_batches over K copies of the config-3 batch) repeated R
times in one process after the bench's own warmup: separates a cold first call from the steady
state.   usage: tools/bench_repeat.py [K] [R]"""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))


def main():
    import torch
    import bench
    from nightcore_analyzer import engine as E
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    params = E.Params(compute_ibi=False)
    for _ in range(3):
        eng.analyze(signals=sig, params=params)
    eng.analyze_batches([sig] * 2, params)
    eng.kernel_profile(4)
    import os
    keep = []                                   # NC_KEEP=1: hold every call's outcomes
    for r in range(R):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = eng.analyze_batches([sig] * K, params)
        if os.environ.get("NC_KEEP") == "1":
            keep.append(out)
        del out
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / K * 1e3
        eng.kernel_times()
        print(f"call {r}: {ms:.3f} ms per step ({K} steps)", flush=True)
    eng.kernel_profile(False)


if __name__ == "__main__":
    main()
