#!/usr/bin/env python3
"""Which kernels run together in a pipelined step: from a rocprofv3 --kernel-trace CSV of
tools/timeline.py --pipelined (cut at its two marker launches), the time spent in each set of
concurrently running kernel classes, largest first.
    python3 tools/concurrency.py TRACE.csv [steps]"""
import csv
import sys

CLASSES = [("stft_mel", "S"), ("window_tg", "W"), ("tuning_peaks", "T"), ("decimate3", "D"), ("cqt_mfma_low", "L"),
           ("cqt_mfma_kernel", "H"), ("tempo_beat", "B"), ("trim_blocks", "R"), ("bootstrap", "b"), ("tuning_select", "s")]


def cls(name):
    for key, c in CLASSES:
        if key in name:
            return c
    return "o"


def main(path, steps=5):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "single_scan_kernel" in r["Kernel_Name"] or "cumsum" in r["Kernel_Name"].lower()]
    i0, i1 = marks[-2], marks[-1]
    t_begin, t_end = int(rows[i0]["End_Timestamp"]), int(rows[i1]["Start_Timestamp"])
    ev = []
    for r in rows[i0 + 1:i1]:
        c = cls(r["Kernel_Name"])
        ev.append((int(r["Start_Timestamp"]), 1, c))
        ev.append((int(r["End_Timestamp"]), -1, c))
    ev.sort()
    active = {}
    acc = {}
    t_prev = t_begin
    for t, d, c in ev:
        t = min(max(t, t_begin), t_end)
        key = "".join(sorted(k for k, n in active.items() if n > 0)) or "-"
        acc[key] = acc.get(key, 0) + (t - t_prev)
        t_prev = t
        active[c] = active.get(c, 0) + d
    key = "".join(sorted(k for k, n in active.items() if n > 0)) or "-"
    acc[key] = acc.get(key, 0) + (t_end - t_prev)
    span = t_end - t_begin
    print(f"span {span / steps / 1e6:.3f} ms/step; classes: " + ", ".join(f"{c}={k}" for k, c in CLASSES) + ", o=other")
    for k, v in sorted(acc.items(), key=lambda x: -x[1])[:24]:
        print(f"  {k:12s} {v / steps / 1e6:7.3f} ms/step  {100 * v / span:5.1f} %")
    big = set("SWTDLH")
    only_small = sum(v for k, v in acc.items() if not (set(k) & big))
    mfma = sum(v for k, v in acc.items() if set(k) & set("LH"))
    stft = sum(v for k, v in acc.items() if "S" in k)
    print(f"no big kernel running: {100 * only_small / span:.1f} %; a CQT kernel running: {100 * mfma / span:.1f} %; "
          f"stft_mel running: {100 * stft / span:.1f} %")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
