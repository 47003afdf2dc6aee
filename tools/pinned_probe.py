#!/usr/bin/env python3
"""Does the per-group pinned result arena cost the pipelined step?  Engine._Arena.alloc_host
allocates a fresh pinned buffer for every pair group, and the outcomes keep it (their host
views point into it), so the caching host allocator cannot reuse it within a call.  Times
Engine.analyze_batches (config 3, K steps) as is, with every alloc_host timed, and with the
arenas carved from one pinned slab allocated up front (timing only), alternating.
usage: tools/pinned_probe.py [K] [ROUNDS]"""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import numpy as np
    import torch
    import bench
    from nightcore_analyzer import engine as E
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    params = E.Params(compute_ibi=False)
    orig = E._Arena.alloc_host
    times = []

    def timed(self):
        t = time.perf_counter()
        orig(self)
        times.append(time.perf_counter() - t)

    slab = torch.empty(512 << 20, dtype=torch.uint8, pin_memory=True)
    pos = [0]

    def from_slab(self):
        if getattr(self, "host", None) is None:
            n = (self.nbytes + 4095) & ~4095
            self.host = slab[pos[0]:pos[0] + n][:self.nbytes]
            pos[0] += n

    def run(kind):
        E._Arena.alloc_host = {"fresh": timed, "slab": from_slab}[kind]
        pos[0] = 0
        torch.cuda.synchronize()
        t = time.perf_counter()
        res = eng.analyze_batches([sig] * K, params)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / K * 1e3
        E._Arena.alloc_host = orig
        del res
        return dt

    for k in ("fresh", "slab"):
        run(k)
    best = {"fresh": [], "slab": []}
    for _ in range(R):
        for k in best:
            times.clear()
            best[k].append(run(k))
            if k == "fresh":
                t = np.array(times) * 1e3
                print(f"fresh: {len(t)} pinned arena allocations, {t.sum() / K:.3f} ms per step, "
                      f"max {t.max():.3f} ms, median {np.median(t):.3f} ms", flush=True)
    for k, v in best.items():
        print(f"{k:>6}: {min(v):.3f} ms/step min, {sorted(v)[len(v) // 2]:.3f} median (runs {[round(x, 3) for x in v]})",
              flush=True)


if __name__ == "__main__":
    main()
