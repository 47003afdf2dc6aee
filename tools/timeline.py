#!/usr/bin/env python3
"""GPU occupancy of the bench step: runs K analysis steps of the config-3 workload
between two marker kernels (torch.cumsum on a tiny tensor) so that a rocprofv3
--kernel-trace of this script can be cut to exactly the timed steps.

    rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python3 tools/timeline.py
    python3 tools/timeline.py --analyze OUT/run_kernel_trace.csv
"""
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))


def run(steps=5):
    import torch
    import bench
    from nightcore_analyzer import engine as E
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    params = E.Params(compute_ibi=False)
    for _ in range(2):
        eng.analyze(signals=sig, params=params)
    marker = torch.arange(8, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    torch.cumsum(marker, 0)
    t0 = time.perf_counter()
    if "--pipelined" in sys.argv:
        eng.analyze_batches([sig] * steps, params)
    else:
        for _ in range(steps):
            eng.analyze(signals=sig, params=params)
    torch.cumsum(marker, 0)
    torch.cuda.synchronize()
    print("wall ms per step", (time.perf_counter() - t0) / steps * 1e3)
    eng.host_stats = {}
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.analyze(signals=sig, params=params)
    torch.cuda.synchronize()
    print("host phases ms per step:", {k: round(v / steps * 1e3, 3) for k, v in eng.host_stats.items()},
          "wall", round((time.perf_counter() - t0) / steps * 1e3, 3))
    eng.host_stats = None


def analyze(path, steps=5):
    import csv
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "single_scan_kernel" in r["Kernel_Name"] or "cumsum" in r["Kernel_Name"].lower()]
    i0, i1 = marks[-2], marks[-1]
    sel = rows[i0 + 1:i1]
    t_begin, t_end = int(rows[i0]["End_Timestamp"]), int(rows[i1]["Start_Timestamp"])
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel)
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = t_end - t_begin
    per = {}
    for r in sel:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
        per[k] = per.get(k, 0) + int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print(f"span {span / steps / 1e6:.2f} ms/step, GPU busy (union) {busy / steps / 1e6:.2f} ms/step "
          f"({100 * busy / span:.1f} %), kernels {len(sel) // steps}/step")
    for k, v in sorted(per.items(), key=lambda x: -x[1])[:16]:
        print(f"  {k:48s} {v / steps / 1e6:7.3f} ms/step")
    # one step in detail: start / end (us from the step start) and queue of every kernel
    n1 = len(sel) // steps
    q = "Queue_Id" if "Queue_Id" in sel[0] else ("Stream_Id" if "Stream_Id" in sel[0] else None)
    t00 = int(sel[0]["Start_Timestamp"])
    print("step 0 detail (us):")
    for r in sel[:n1]:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
        print(f"  q{r.get(q, '?') if q else '?':>3} {(int(r['Start_Timestamp']) - t00) / 1e3:9.1f} "
              f"{(int(r['End_Timestamp']) - t00) / 1e3:9.1f}  {k}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run()
