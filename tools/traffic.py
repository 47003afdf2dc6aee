#!/usr/bin/env python3
"""Per-launch HBM traffic of the bench kernels from the two counter passes of
tools/pmc_traffic.sh, corrected per MI355X_MICROARCH.md (FETCH_SIZE reports half the
bytes of a wide coalesced read on gfx950: hbm = 2 x FETCH_SIZE + WRITE_SIZE, KiB -> B),
written to profiles/<NAME> (default r3_traffic.json) for bench.py's roofline.traffic.
    python3 tools/traffic.py OUTDIR [NAME]"""
import collections
import csv
import json
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
TAGS = {"cqt_mfma_kernel": "cqt_high", "cqt_mfma_low_kernel": "cqt_low", "cqt_mfma_low2_kernel": "cqt_low",
        "cqt_tail_kernel": "cqt_tail",
        "stft_mel_kernel": "stft_mel", "tuning_peaks_kernel": "tuning_peaks",
        "trim_blocks_kernel": "trim_blocks", "window_tg_kernel": "window_tg", "decimate_kernel": "decimate", "decimate3_kernel": "decimate"}
# algorithmic bytes per step of the config-3 bench: 3968 windows x 882 000 B,
# 896 chunks x 1 764 000 B, 64 pairs of 3 969 000 + 3 175 200 samples x 4 B for the trim pass;
# the octave chain reads levels 0 and 3 and writes levels 1-6 once per 441 000-sample chunk
# (441 000 + 55 125 read, 220 500 + 110 250 + 55 125 + 27 563 + 13 782 + 6 891 written, f32)
# the CQT is two launches per chroma call (octaves 0-2, octaves 3-6): their bytes per call
# are summed into "cqt_chroma", the unit bench.py times (the sum of the two kernels' times);
# the frame tail (cqt_tail) is listed on its own
CQT_PARTS = ("cqt_low", "cqt_high")
ALG_STEP = {"cqt_chroma": 896 * 1764000, "stft_mel": 3968 * 882000, "trim_blocks": 64 * (3969000 + 3175200) * 4,
            "decimate": 896 * 4 * (441000 + 55125 + 220500 + 110250 + 55125 + 27563 + 13782 + 6891)}


def per_dispatch(d: Path, counter: str):
    vals = collections.defaultdict(list)
    for f in d.rglob("*counter_collection.csv"):
        acc = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]
            if name in TAGS:
                acc[(TAGS[name], r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (tag, _), v in acc.items():
            vals[tag].append(v)
    return vals


# the access form each kernel's reads / writes mostly use (tools/calib_fetch.hip kernel names):
# FETCH_SIZE / WRITE_SIZE are divided by that form's measured scale (profiles/r6_fetch_calibration.json)
FORMS = {"stft_mel": ("stream_read<float2>", "stream_write<float>"),
         "tuning_peaks": ("stream_read<float2>", "stream_write<float>"),
         "window_tg": ("stream_read<float2>", "stream_write<float>"),
         "trim_blocks": ("stream_read<float4>", "stream_write<float>"),
         "decimate": ("stream_read<float4>", "stream_write<float4>"),
         "cqt_low": ("stream_read<float4>", "stream_write<float>"),      # dwordx4 blocks; slices by LDS-DMA
         "cqt_high": ("lds_dma_read", "stream_write<float>"),            # slices by LDS-DMA; images dwordx4
         "cqt_tail": ("stream_read<float4>", "stream_write<float>")}


def _scales(calib):
    if not calib:
        return None
    c = json.loads(Path(calib).read_text())
    return c.get("read_scale", {}), c.get("write_scale", {})


def main(out, name=None, calib=None):
    out = Path(out)
    sc = _scales(calib)
    fetch = per_dispatch(out / "FETCH_SIZE", "FETCH_SIZE")
    write = per_dispatch(out / "WRITE_SIZE", "WRITE_SIZE")
    sys.path.insert(0, str(REPO))
    from bench import build_provenance     # kernel-source / library hashes and the commit
    prov = build_provenance()
    commit = prov["commit"]
    kern = {}
    # two trim launches per analyze call (engine.Engine.analyze: the first pair group's files,
    # then the rest): the profiled run's call count, hence launches per step of every kernel
    # (the pair-group schedule sets how many launches one step makes)
    calls = max(1, len(fetch.get("trim_blocks", [])) // 2)
    for tag in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(tag, [0])) / max(1, len(fetch.get(tag, [])))
        w = sum(write.get(tag, [0])) / max(1, len(write.get(tag, [])))
        k = {"launches": len(fetch.get(tag, [])), "fetch_size_kib_raw": round(f, 2), "write_size_kib": round(w, 2),
             "hbm_bytes_per_launch": int(round((2 * f + w) * 1024))}
        if sc is not None and tag in FORMS:
            rf, wf = FORMS[tag]
            rs, ws = sc[0].get(rf, 0.5), sc[1].get(wf, 1.0)
            k["calibration"] = {"read_form": rf, "read_scale": rs, "write_form": wf, "write_scale": ws}
            k["hbm_bytes_per_launch"] = int(round((f / rs + w / ws) * 1024))
        k["launches_per_step"] = round(k["launches"] / calls, 3)
        if tag in ALG_STEP and fetch.get(tag):
            # mean over launches of unequal groups: per-step bytes / launches per step
            k["alg_bytes_per_launch"] = int(ALG_STEP[tag] * calls / len(fetch[tag]))
        kern[tag] = k
    present = [t for t in CQT_PARTS if t in kern]
    if len(present) == len(CQT_PARTS):
        n_calls = kern["cqt_low"]["launches"]  # one of each per chroma call
        per_call = lambda key: sum(kern[t][key] * kern[t]["launches"] / n_calls for t in present)
        k = {"launches": n_calls, "parts": present,
             "fetch_size_kib_raw": round(per_call("fetch_size_kib_raw"), 2),
             "write_size_kib": round(per_call("write_size_kib"), 2),
             "hbm_bytes_per_launch": int(per_call("hbm_bytes_per_launch")),
             "launches_per_step": kern["cqt_low"]["launches_per_step"],
             "alg_bytes_per_launch": int(ALG_STEP["cqt_chroma"] * calls / n_calls)}
        kern["cqt_chroma"] = k
    doc = {"workload": "config3-64pairs", "commit": commit, "src_sha": prov["src_sha"], "lib_sha": prov["lib_sha"],
           "analyze_calls": calls,
           "command": "tools/pmc_traffic.sh: rocprofv3 --pmc FETCH_SIZE, then a separate --pmc WRITE_SIZE pass, "
                      "--output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ibi "
                      "--no-config5 (means over every launch; the engine's default pair-group schedule)",
           "correction": "hbm_bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950 FETCH_SIZE reports half "
                         "the bytes of a wide coalesced read (MI355X_MICROARCH.md; calibrated with "
                         "tools/calib_fetch.hip: a 1 GiB stream read reports 0.500 GiB)",
           "kernels": kern}
    if sc is not None:
        doc["correction"] = ("hbm_bytes = FETCH_SIZE / read_scale + WRITE_SIZE / write_scale (KiB -> bytes), the "
                             "scales of each kernel's dominant access form measured by tools/calib_fetch.hip "
                             f"({Path(calib).name}; per kernel under 'calibration')")
    name = name or "r3_traffic.json"
    (REPO / "profiles" / name).write_text(json.dumps(doc, indent=1) + "\n")
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
