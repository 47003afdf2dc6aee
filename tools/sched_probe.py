#!/usr/bin/env python3
"""Host phase times (engine.host_stats) of the config-3 workload for a few pair-group
schedules: separates host stalls (launch / assemble) from device time (wait)."""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))


def main():
    import gc
    import os
    if os.environ.get("PROBE_NO_GC") == "1":
        gc.disable()
    import torch
    import bench
    from nightcore_analyzer import engine as E
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    params = E.Params(compute_ibi=False)
    for arg in sys.argv[1:] or ["8,24,24,8", "32", "4,24,24,12"]:
        gp = [int(v) for v in arg.split(",")] if "," in arg else int(arg)
        for _ in range(2):
            eng.analyze(signals=sig, params=params, group_pairs=gp)
        torch.cuda.synchronize()
        eng.host_stats = {}
        t0 = time.perf_counter()
        for _ in range(5):
            eng.analyze(signals=sig, params=params, group_pairs=gp)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 5 * 1e3
        hs = {k: round(v / 5 * 1e3, 2) for k, v in eng.host_stats.items()}
        eng.host_stats = None
        print(f"{arg:>14s}: {ms:7.3f} ms/step  {hs}", flush=True)


if __name__ == "__main__":
    main()
