#!/usr/bin/env python3
"""Reconcile the bench line with rocprofv3: the kernel launches of bench.py's timed region, cut
from a `rocprofv3 --kernel-trace` run of the same command by the two marker launches bench.py
puts around it (torch.cumsum), their average durations per kernel, and the roofline fractions
recomputed from them with the line's own algorithmic bytes and launches per step.

    python3 tools/rocprof_timed.py TRACE_CSV BENCH_JSON OUT_JSON"""
import collections
import csv
import json
import sys

KERNELS = {"stft_mel_kernel": "stft_mel", "cqt_mfma_low_kernel": "cqt_low", "cqt_mfma_kernel": "cqt_high",
           "window_tg_kernel": "window_tg", "tuning_peaks_kernel": "tuning_peaks", "decimate3_kernel": "decimate",
           "trim_blocks_kernel": "trim_blocks"}
HBM_PEAK_GBS = 8000.0


def short(name):
    return name.split("(")[0].replace("void ", "").split("::")[-1].split("<")[0]


def main(trace, bench, out):
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    # torch.cumsum lowers to rocprim's single_scan_kernel on ROCm (the engine's own kernels never
    # use rocprim; bootstrap_rejscan_kernel is not a marker)
    marks = [i for i, r in enumerate(rows) if "single_scan_kernel" in r["Kernel_Name"] or "cumsum" in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit("fewer than two marker launches in the trace")
    i0, i1 = marks[0], marks[1]
    t_lo, t_hi = int(rows[i0]["End_Timestamp"]), int(rows[i1]["Start_Timestamp"])
    dur = collections.defaultdict(list)
    for r in rows[i0 + 1:i1]:
        if int(r["Start_Timestamp"]) >= t_lo and int(r["End_Timestamp"]) <= t_hi:
            k = KERNELS.get(short(r["Kernel_Name"]))
            if k:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    # device occupancy of the timed region: the union of every kernel's [start, end)
    iv = sorted((max(t_lo, int(r["Start_Timestamp"])), min(t_hi, int(r["End_Timestamp"])))
                for r in rows[i0 + 1:i1] if int(r["End_Timestamp"]) > t_lo and int(r["Start_Timestamp"]) < t_hi)
    busy, cs, ce = 0, None, None
    for a, b in iv:
        if ce is None or a > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    if ce is not None:
        busy += ce - cs
    line = json.loads(open(bench).read().strip().splitlines()[-1])
    steps = line["steps"]
    roof = line["roofline"]
    lines = {"stft_mel": roof if roof["kernel"] == "stft_mel" else roof.get("stft_mel"),
             "cqt_chroma": roof if roof["kernel"] == "cqt_chroma" else roof.get("cqt_chroma"),
             "window_tg": roof.get("window_tg")}
    res = {"trace": trace, "bench_line": bench, "timed_region_ns": t_hi - t_lo, "steps": steps,
           "device_busy_frac": busy / max(1, t_hi - t_lo), "kernels_in_region": len(iv),
           "rocprof_ms_per_launch": {k: sum(v) / len(v) for k, v in dur.items()},
           "rocprof_launches_per_step": {k: len(v) / steps for k, v in dur.items()}, "check": {}}
    for tag, ln in lines.items():
        if not ln:
            continue
        if tag == "cqt_chroma":
            if "cqt_low" not in dur or "cqt_high" not in dur:
                continue
            rp = res["rocprof_ms_per_launch"]["cqt_low"] + res["rocprof_ms_per_launch"]["cqt_high"]
        elif tag in dur:
            rp = res["rocprof_ms_per_launch"][tag]
        else:
            continue
        frac = ln["alg_bytes_per_launch"] / (rp * 1e-3) / 1e9 / HBM_PEAK_GBS
        res["check"][tag] = {"line_avg_launch_ms": ln["avg_launch_ms"], "rocprof_avg_launch_ms": rp,
                             "ratio": ln["avg_launch_ms"] / rp, "line_frac": ln["frac"], "rocprof_frac": frac,
                             "line_traffic": ln.get("traffic"), "traffic_source": ln.get("traffic_source")}
    open(out, "w").write(json.dumps(res, indent=1) + "\n")
    print(json.dumps({"device_busy_frac": res["device_busy_frac"], **res["check"]}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
