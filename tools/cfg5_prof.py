#!/usr/bin/env python3
"""Config 5 (one 60-min pair, run() with the hop-64 IBI pass) for a rocprofv3 kernel trace:
    rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/cfg5_prof.py"""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))


def main():
    import torch
    import bench
    import os
    from nightcore_analyzer import _native
    from nightcore_analyzer import engine as E
    if os.environ.get("CFG5_LIB"):  # a tools/var_build.sh variant
        _native._LIB_PATH = Path(os.environ["CFG5_LIB"]).resolve()
    nc, src = bench.make_pairs(1, 3600.0, 5000, 1)[0]
    eng = E.get_engine(0)
    sig = eng.upload_signals([nc, src])
    eng.analyze(signals=sig, params=E.Params(compute_ibi=True))
    torch.cuda.synchronize()
    eng.host_stats = {}
    t0 = time.perf_counter()
    eng.analyze(signals=sig, params=E.Params(compute_ibi=True))
    torch.cuda.synchronize()
    print("config5 s", time.perf_counter() - t0, {k: round(v, 4) for k, v in eng.host_stats.items()})


if __name__ == "__main__":
    main()
