#!/usr/bin/env python3
"""Host overhead of the window-sharded entry point against the engine's pipelined batches on
one GPU, one process (no process group: analyze_sharded runs with world 1, every pair
interior): K steps of config 3 (64 x 3-min pairs) each way, alternated.
    python3 tools/win_overhead.py [rounds]"""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))


def main(rounds=3, K=10):
    import torch
    import bench
    from nightcore_analyzer import engine as E
    from nightcore_analyzer.sharded import DeviceStages, analyze_sharded
    pairs = bench.make_pairs_ids(list(range(64)), 180.0, 1000, 16)
    eng = E.get_engine(0)
    flat = [a for pr in pairs for a in pr]
    sig = eng.upload_signals(flat)
    p = E.Params(compute_ibi=False)
    lengths = [n for _ in range(64) for n in bench.synth_lengths(180.0)]
    eng.analyze_batches([sig] * 2, p)
    analyze_sharded(DeviceStages(eng, sig), p, lengths=lengths, gather=False, steps=2)
    for r in range(rounds):
        for name in ("batches", "sharded"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if name == "batches":
                eng.analyze_batches([sig] * K, p)
            else:
                analyze_sharded(DeviceStages(eng, sig), p, lengths=lengths, gather=False, steps=K)
            torch.cuda.synchronize()
            print(f"{name:8s} round {r}: {(time.perf_counter() - t0) / K * 1e3:.2f} ms/step", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
