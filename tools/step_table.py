#!/usr/bin/env python3
"""Per-step kernel table from a rocprofv3 --stats kernel_stats.csv of tools/prof_step.py:
total ms per step of every kernel (TotalDurationNs / steps), sorted, and their sum.
    python3 tools/step_table.py KERNEL_STATS_CSV STEPS"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = float(sys.argv[2])
    tot = 0.0
    out = []
    for r in rows:
        name = r["Name"].split("(")[0].replace("void ", "")[:70]
        ms = float(r["TotalDurationNs"]) / 1e6 / steps
        out.append((ms, int(r["Calls"]) / steps, name))
        tot += ms
    out.sort(reverse=True)
    for ms, calls, name in out:
        print(f"{ms:8.3f} ms/step {calls:7.1f} calls/step  {name}")
    print(f"{tot:8.3f} ms/step total")


if __name__ == "__main__":
    main()
