#!/usr/bin/env python3
"""cProfile of the engine's host side on the bench workload (64 x 3-min pairs):
where the ~12 ms per step outside the kernels goes.  Writes gpurun_out/host.pstats
and prints the top entries by cumulative and own time."""
import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from nightcore_analyzer import engine as E  # noqa: E402


def main():
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    flat = [a for nc, src in pairs for a in (nc, src)]
    sig = eng.upload_signals(flat)
    params = E.Params(compute_ibi=False)
    for _ in range(2):
        eng.analyze(signals=sig, params=params)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        eng.analyze(signals=sig, params=params)
    torch.cuda.synchronize()
    print("step ms", (time.perf_counter() - t0) / 5 * 1e3)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        eng.analyze(signals=sig, params=params)
    torch.cuda.synchronize()
    pr.disable()
    out = REPO / "gpurun_out"
    out.mkdir(exist_ok=True)
    pr.dump_stats(str(out / "host.pstats"))
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(35)
        print(s.getvalue())


if __name__ == "__main__":
    main()
