#!/usr/bin/env python3
"""Device idle of the pipelined config-3 step without a tracer: Engine.analyze_batches over K
batches with every kernel recording its execution span (profile mode 2), then the union of the
spans (nc_profile_read_busy) against their extent.  Variants are timed in rotation.
usage: tools/idle_probe.py [K] [variant ...]
  variant: "default", "SCHEDULE" ("6,26,26,6", "32"), "SCHEDULE@G" (G groups in flight: GROUPS_IN_FLIGHT and, eager, MAX_GROUPS_IN_FLIGHT),
           "...+eager" / "+lazy" (Engine.EAGER_FINISH: assemble a group only once it is complete)"""
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
    variants = sys.argv[2:] or ["default"]
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    params = E.Params(compute_ibi=False)
    gif0, eager0, max0 = eng.GROUPS_IN_FLIGHT, eng.EAGER_FINISH, eng.MAX_GROUPS_IN_FLIGHT

    def setup(v):
        v, _, flag = v.partition("+")
        sched, _, gif = v.partition("@")
        eng.GROUPS_IN_FLIGHT = int(gif) if gif else gif0
        eng.MAX_GROUPS_IN_FLIGHT = int(gif) if gif else max0
        eng.EAGER_FINISH = True if flag == "eager" else (False if flag == "lazy" else eager0)
        return None if sched == "default" else ([int(x) for x in sched.split(",")] if "," in sched else int(sched))

    def run(gp, mode):
        eng.kernel_profile(mode)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.analyze_batches([sig] * K, params, group_pairs=gp)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / K * 1e3
        busy = eng.device_busy() if mode == 2 else None
        eng.kernel_profile(0)
        return ms, busy

    for v in variants:          # warm every variant
        run(setup(v), 0)
    res = {v: {"off": [], "span": [], "idle": []} for v in variants}
    import os
    for _ in range(int(os.environ.get("NC_PROBE_ROUNDS", "3"))):
        for v in variants:
            gp = setup(v)
            res[v]["off"].append(run(gp, 0)[0])
            ms, (b, e, n) = run(gp, 2)
            res[v]["span"].append(ms)
            res[v]["idle"].append(1.0 - b / e)
    for v in variants:
        r = res[v]
        print(f"{v:>18}: {min(r['off']):7.3f} ms/step (no timers; runs {[round(x, 3) for x in r['off']]}), "
              f"{min(r['span']):7.3f} with spans, device idle {[round(100 * x, 2) for x in r['idle']]} %", flush=True)


if __name__ == "__main__":
    main()
