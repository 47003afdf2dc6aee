#!/usr/bin/env python3
"""Summarise rocprofv3 output directories written by tools/prof_kernels.py runs:
    python3 tools/pmc_report.py DIR [DIR ...]
DIR may hold run_kernel_stats.csv (--stats) and/or run_counter_collection.csv (--pmc).
Per kernel: average duration; stall split (SQ_WAIT_ANY / SQ_WAIT_INST_ANY /
SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES), LDS bank-conflict share, VALU and LDS
instructions per dispatch, FETCH/WRITE per dispatch when collected."""
import collections
import csv
import sys
from pathlib import Path


def report(d: Path) -> None:
    st = d / "run_kernel_stats.csv"
    if st.exists():
        print(f"== {d} (kernel stats)")
        for r in list(csv.DictReader(open(st)))[:12]:
            print(f"  {r['Name'][:56]:56s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e3:9.1f} us")
    pc = d / "run_counter_collection.csv"
    if pc.exists():
        print(f"== {d} (counters)")
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        n = collections.Counter()
        for r in csv.DictReader(open(pc)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[(k, r["Counter_Name"])] += 1
        for k, v in agg.items():
            cyc = v.get("SQ_WAVE_CYCLES", 0.0)
            parts = []
            if cyc > 5e7:
                parts.append(f"wait {100 * v['SQ_WAIT_ANY'] / cyc:4.1f}% inst {100 * v['SQ_WAIT_INST_ANY'] / cyc:4.1f}% "
                             f"active {100 * v['SQ_ACTIVE_INST_ANY'] / cyc:4.1f}%")
                parts.append(f"ldsconf {100 * v['SQ_LDS_BANK_CONFLICT'] / max(1.0, v['SQ_LDS_IDX_ACTIVE']):4.1f}%")
                nd = n[(k, "SQ_INSTS_VALU")]
                parts.append(f"valu/disp {v['SQ_INSTS_VALU'] / nd:.3g} lds/disp {v['SQ_INSTS_LDS'] / nd:.3g}")
            if v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) > 0 and v.get("GRBM_GUI_ACTIVE", 0.0) > 0:
                # MFMA pipe busy cycles summed over the chip's 1024 SIMDs, against the dispatches'
                # GPU-active cycles (MI355X_MICROARCH.md: 16 per 16x16x32 f16 MFMA).  GRBM_GUI_ACTIVE
                # comes summed over the 8 XCDs (3 x 0.49 ms of stft_mel read 2.63e7 cycles), hence / 8
                nd = n[(k, "SQ_VALU_MFMA_BUSY_CYCLES")]
                parts.append(f"mfma busy {100 * v['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * v['GRBM_GUI_ACTIVE'] / 8):4.1f}% "
                             f"mfma/disp {v.get('SQ_INSTS_MFMA', 0.0) / nd:.4g}")
            for c in ("FETCH_SIZE", "WRITE_SIZE"):
                if c in v and v[c] > 1e4:
                    parts.append(f"{c} {v[c] / n[(k, c)]:.4g} KiB/disp")
            if parts:
                print(f"  {k:40s} " + " | ".join(parts))


if __name__ == "__main__":
    for a in sys.argv[1:]:
        report(Path(a))
