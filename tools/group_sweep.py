#!/usr/bin/env python3
"""Step time of the config-3 workload (64 x 3-min pairs) against the engine's pair-group
schedule (the unit of host/device pipelining and of kernel batch size).
    python3 tools/group_sweep.py [--pipelined] [--rounds R] SCHEDULE ...
SCHEDULE: an int (groups of that size) or a comma list of sizes; "default" = the engine's;
a suffix "@G" runs it with G groups in flight (Engine.GROUPS_IN_FLIGHT).
--pipelined times 10 steps as one Engine.analyze_batches call (bench.py's timed loop);
schedules are alternated over R rounds so that clock drift hits them alike."""
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
    args = sys.argv[1:]
    pipelined = "--pipelined" in args
    rounds = 1
    if "--rounds" in args:
        rounds = int(args[args.index("--rounds") + 1])
        del args[args.index("--rounds"):args.index("--rounds") + 2]
    args = [a for a in args if a != "--pipelined"] or ["8", "16", "24", "32", "64"]
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    params = E.Params(compute_ibi=False)

    gif0 = eng.GROUPS_IN_FLIGHT

    def sched(arg):
        arg, _, gif = arg.partition("@")
        eng.GROUPS_IN_FLIGHT = int(gif) if gif else gif0
        if arg == "default":
            return None
        return [int(v) for v in arg.split(",")] if "," in arg else int(arg)

    def run(gp, k):
        if pipelined:
            eng.analyze_batches([sig] * k, params, group_pairs=gp)
        else:
            for _ in range(k):
                eng.analyze(signals=sig, params=params, group_pairs=gp)

    res = {a: [] for a in args}
    for arg in args:
        run(sched(arg), 2)
    for _ in range(rounds):
        for arg in args:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(sched(arg), 10)
            torch.cuda.synchronize()
            res[arg].append((time.perf_counter() - t0) / 10 * 1e3)
    for arg in args:
        v = res[arg]
        print(f"group_pairs {arg:>14s}: {min(v):7.3f} min {sum(v) / len(v):7.3f} mean ms/step "
              f"{3968 / min(v) * 1e3:9.0f} windows/s  ({'pipelined' if pipelined else 'separate calls'})", flush=True)


if __name__ == "__main__":
    main()
