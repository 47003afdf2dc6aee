#!/usr/bin/env python3
"""Cost of the kernel-span profiling (nc_profile mode 2) on the pipelined config-3 step:
10 steps as one analyze_batches call, profiling off / on, alternated over rounds."""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))


def main(rounds=4):
    import torch
    import bench
    from nightcore_analyzer import engine as E
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    params = E.Params(compute_ibi=False)
    eng.analyze_batches([sig] * 3, params)
    res = {0: [], 2: []}
    for _ in range(rounds):
        for mode in (0, 2):
            if mode:
                eng.kernel_profile(mode)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.analyze_batches([sig] * 10, params)
            torch.cuda.synchronize()
            res[mode].append((time.perf_counter() - t0) / 10 * 1e3)
            if mode:
                eng.kernel_spans()
                eng.kernel_profile(False)
    for mode, v in res.items():
        print(f"profile mode {mode}: min {min(v):.3f} mean {sum(v) / len(v):.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
