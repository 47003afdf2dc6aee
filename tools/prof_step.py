#!/usr/bin/env python3
"""Every kernel of the config-3 step, for rocprofv3 --kernel-trace --stats: one warm-up call and
K pipelined batches of the bench's 64 pairs (kernel_stats / (K + 1) = per-step totals).
NC_SERIAL_STREAMS=1 runs the three chains on one stream (isolated durations).
    rocprofv3 --kernel-trace --stats -- python3 tools/prof_step.py [K]"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))


def main():
    import torch
    import bench
    from nightcore_analyzer import engine as E
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    params = E.Params(compute_ibi=False)
    eng.analyze(signals=sig, params=params)
    eng.analyze_batches([sig] * K, params)
    torch.cuda.synchronize()
    print("steps", K + 1)


if __name__ == "__main__":
    main()
