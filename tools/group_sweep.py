#!/usr/bin/env python3
"""Step time of the config-3 workload (64 x 3-min pairs) against the engine's pair-group
size (the unit of host/device pipelining and of kernel batch size)."""
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
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    params = E.Params(compute_ibi=False)
    for arg in (sys.argv[1:] or ["8", "16", "24", "32", "64"]):
        gp = [int(v) for v in arg.split(",")] if "," in arg else int(arg)
        for _ in range(2):
            eng.analyze(signals=sig, params=params, group_pairs=gp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            eng.analyze(signals=sig, params=params, group_pairs=gp)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 5 * 1e3
        print(f"group_pairs {arg:>14s}: {ms:7.3f} ms/step  {3968 / ms * 1e3:9.0f} windows/s", flush=True)


if __name__ == "__main__":
    main()
