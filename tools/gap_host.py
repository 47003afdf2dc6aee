#!/usr/bin/env python3
"""What the host does while the device idles: device gaps inside the bench's timed region
(cut at its marker launches, as tools/trace_gaps.py) of a rocprofv3 run with
--kernel-trace --memory-copy-trace --hip-runtime-trace, and for each gap the HIP API calls
that overlap it (name, start relative to the gap, duration), longest first.
usage: tools/gap_host.py DIR/run [min_gap_us]   (DIR/run_kernel_trace.csv, ..._hip_api_trace.csv)"""
import csv
import sys
from collections import Counter


def rows(path):
    try:
        return list(csv.DictReader(open(path)))
    except FileNotFoundError:
        return []


def main():
    base = sys.argv[1]
    thr = float(sys.argv[2]) if len(sys.argv) > 2 else 300.0
    kt = sorted(rows(base + "_kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    mc = rows(base + "_memory_copy_trace.csv")
    api = sorted(rows(base + "_hip_api_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in kt]
    ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?")) for r in mc]
    ev.sort()
    marks = [i for i, r in enumerate(kt) if "single_scan_kernel" in r["Kernel_Name"]]
    t0, t_end = int(kt[marks[-2]]["End_Timestamp"]), int(kt[marks[-1]]["Start_Timestamp"])
    reg = [e for e in ev if t0 <= e[0] <= t_end]
    end, idle, gaps = t0, 0, []
    for i, (s, e, name) in enumerate(reg):
        if s > end:
            idle += s - end
            if s - end > thr * 1e3:
                gaps.append((end, s, reg[i - 1][2] if i else "", name))
        end = max(end, e)
    span = t_end - t0
    print(f"timed region {span / 1e6:.3f} ms, device idle (kernels + copies) {idle / 1e6:.3f} ms "
          f"({idle / span:.1%}), {len(gaps)} gaps > {thr:.0f} us")
    tot = Counter()
    for a, b, before, after in gaps:
        print(f"\n{(b - a) / 1e3:8.1f} us at {(a - t0) / 1e6:8.3f} ms: after {before!r} before {after!r}")
        ov = [r for r in api if int(r["Start_Timestamp"]) < b and int(r["End_Timestamp"]) > a]
        ov.sort(key=lambda r: int(r["Start_Timestamp"]) - int(r["End_Timestamp"]))
        for r in ov[:8]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            print(f"    {r['Function'][:40]:40s} start {(s - a) / 1e3:+9.1f} us  dur {(e - s) / 1e3:9.1f} us")
        n = Counter(r["Function"] for r in ov)
        print("    calls in gap:", ", ".join(f"{k} x{v}" for k, v in n.most_common(8)))
        for r in ov:
            s, e = max(int(r["Start_Timestamp"]), a), min(int(r["End_Timestamp"]), b)
            tot[r["Function"]] += e - s
    print("\nAPI time inside gaps (us):", {k: round(v / 1e3, 1) for k, v in tot.most_common(12)})


if __name__ == "__main__":
    main()
