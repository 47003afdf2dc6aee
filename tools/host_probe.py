#!/usr/bin/env python3
"""Host side of the pipelined config-3 step (Engine.analyze_batches over K batches): ms per step
with the library's kernel timers off / on, engine.host_stats phases, and a cProfile of the host
path sorted by own time.  Finds what the host does while the device idles at batch boundaries.
usage: tools/host_probe.py [K] [schedule ...]   (schedule: "6,26,26,6", "32", ...)"""
import cProfile
import io
import pstats
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
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    scheds = sys.argv[2:] or ["default"]
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    params = E.Params(compute_ibi=False)

    def run(gp):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.analyze_batches([sig] * K, params, group_pairs=gp)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / K * 1e3

    gif0 = eng.GROUPS_IN_FLIGHT
    for s in scheds:
        # "SCHEDULE@G": that schedule with G pair groups in flight
        sched, _, gif = s.partition("@")
        eng.GROUPS_IN_FLIGHT = int(gif) if gif else gif0
        gp = None if sched == "default" else ([int(v) for v in sched.split(",")] if "," in sched else int(sched))
        for _ in range(2):
            run(gp)
        off, on, on3, on2, on4 = [], [], [], [], []
        for _ in range(3):                       # interleaved: off, events on all, on roofline kernels, spans only
            off.append(run(gp))
            eng.kernel_profile(1)
            on.append(run(gp))
            eng.kernel_profile(3)
            on3.append(run(gp))
            eng.kernel_profile(2)
            on2.append(run(gp))
            eng.kernel_profile(4)
            on4.append(run(gp))
            eng.kernel_profile(False)
        off, on, on3, on2, on4 = min(off), min(on), min(on3), min(on2), min(on4)
        eng.host_stats = {}
        run(gp)
        hs = {k: round(v / K * 1e3, 3) for k, v in eng.host_stats.items()}
        eng.host_stats = None
        print(f"{s:>12s}: {off:7.3f} ms/step (timers off)  {on:7.3f} (events on all)  {on3:7.3f} (events on the "
              f"roofline kernels)  {on2:7.3f} (spans only)  {on4:7.3f} (events on the roofline kernels, no spans)  host {hs}", flush=True)

    eng.GROUPS_IN_FLIGHT = gif0
    gp = None
    eng.host_trace = []
    ms = run(gp)
    tr, eng.host_trace = eng.host_trace, None
    print(f"host trace run: {ms:.3f} ms/step; batches 4-5 (ms from the first mark of batch 4, step between marks):")
    i0 = next(i for i, (_, l) in enumerate(tr) if l == "b4 trim")
    i1 = next((i for i, (_, l) in enumerate(tr) if l == "b6 trim"), len(tr))
    t0 = tr[i0][0]
    for i in range(i0, i1):
        t, l = tr[i]
        print(f"  {(t - t0) * 1e3:8.3f}  +{(tr[i + 1][0] - t) * 1e3 if i + 1 < len(tr) else 0:7.3f}  {l}")
    pr = cProfile.Profile()
    pr.enable()
    ms = run(gp)
    pr.disable()
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(45)
    print(f"cProfile run: {ms:.3f} ms/step")
    print(out.getvalue())
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("cumulative").print_stats(40)
    print(out.getvalue())


if __name__ == "__main__":
    main()
