#!/usr/bin/env python3
"""Device idle gaps inside the timed region of a rocprofv3 kernel trace (cut at the bench's
marker launches): total idle, and each gap above a threshold with the launches around it.
usage: tools/trace_gaps.py run_kernel_trace.csv [min_gap_us]"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    thr = float(sys.argv[2]) if len(sys.argv) > 2 else 300.0
    idx = [i for i, r in enumerate(rows) if "single_scan_kernel" in r["Kernel_Name"] or "cumsum" in r["Kernel_Name"]]
    reg = rows[idx[-2]:idx[-1] + 1]
    t0 = int(reg[0]["End_Timestamp"])
    t_end = int(reg[-1]["Start_Timestamp"])
    end, idle, gaps = t0, 0, []
    for i in range(1, len(reg)):
        s = int(reg[i]["Start_Timestamp"])
        if s > end:
            idle += s - end
            if s - end > thr * 1e3:
                gaps.append((i, end, s))
        end = max(end, int(reg[i]["End_Timestamp"]))
    span = t_end - t0
    print(f"timed region {span / 1e6:.3f} ms, device idle {idle / 1e6:.3f} ms ({idle / span:.1%}), "
          f"{len(gaps)} gaps > {thr:.0f} us")
    for i, a, b in gaps:
        print(f"  {(b - a) / 1e3:8.1f} us at {(a - t0) / 1e6:8.3f} ms: after {reg[i - 1]['Kernel_Name'][:50]!r} "
              f"before {reg[i]['Kernel_Name'][:50]!r}")


if __name__ == "__main__":
    main()
