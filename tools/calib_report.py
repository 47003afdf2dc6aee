#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE scale per access form from two rocprofv3 counter passes over
tools/calib_fetch (every kernel moves exactly 1 GiB): counter bytes / true bytes, averaged
over the kernel's launches -> JSON (profiles/r6_fetch_calibration.json).  tools/traffic.py
divides each engine kernel's counters by the scale of the form it uses.
    python3 tools/calib_report.py OUTDIR OUT.json"""
import collections
import csv
import json
import sys
from pathlib import Path

TRUE = float(1 << 30)


def per_kernel(d: Path, counter: str):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in d.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1].strip()
            tmpl = r["Kernel_Name"].split("<")[1].split(">")[0] if "<" in r["Kernel_Name"] else ""
            acc[(name + (f"<{tmpl}>" if tmpl else ""))][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in acc.items()}


def main(out, dst):
    out = Path(out)
    fetch = per_kernel(out / "FETCH_SIZE", "FETCH_SIZE")
    write = per_kernel(out / "WRITE_SIZE", "WRITE_SIZE")
    doc = {"true_bytes_per_kernel": int(TRUE), "unit": "counter KiB x 1024 / true bytes",
           "read_scale": {k: round(v * 1024 / TRUE, 4) for k, v in sorted(fetch.items()) if "read" in k},
           "write_scale": {k: round(v * 1024 / TRUE, 4) for k, v in sorted(write.items()) if "write" in k},
           "how": "rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE, over tools/calib_fetch (1 GiB per kernel "
                  "from a cold 1 GiB buffer; two repetitions averaged)"}
    Path(dst).write_text(json.dumps(doc, indent=1) + "\n")
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:3])
