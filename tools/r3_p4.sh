#!/bin/bash
# piptrack compaction + XCD-ordered CQT: rotated timings, FETCH_SIZE of the chroma path per build, parity tests
set -o pipefail
O=gpurun_out/p4
R=$GRAFT_REPO_ROOT
mkdir -p $O
export TMPDIR=/tmp
VB_TUNING=1 timeout -k 10 300 python3 tools/var_bench.py tools/var/base/libncgpu.so tools/var/pip1/libncgpu.so tools/var/xcd/libncgpu.so tools/var/nomelw/libncgpu.so tools/var/nohann/libncgpu.so > $O/t1.log 2>&1 || { echo "var failed"; tail -20 $O/t1.log; exit 1; }
grep -v amdgpu.ids $O/t1.log
for v in base xcd; do
  cd /tmp && NCGPU_LIB=$R/tools/var/$v/libncgpu.so timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/f_$v -o run -- python3 $R/tools/prof_kernels.py chroma > $R/$O/f_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $R/$O/f_$v.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, collections, glob
for v in ("base", "xcd"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/p4/f_{v}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(r["Kernel_Name"].split("(")[0].split("::")[-1], r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, _), x in per.items(): acc[k].append(x)
    print(v, {k: round(2 * sum(x) / len(x) / 1024, 1) for k, x in acc.items() if "cqt" in k or "decim" in k or "tuning" in k}, "MiB per launch (2x FETCH)")
PY
cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/$O/lds -o run -- python3 $R/tools/prof_kernels.py windows > $R/$O/lds.log 2>&1 || { echo "pmc lds failed"; tail -5 $R/$O/lds.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, collections, glob
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob("gpurun_out/p4/lds/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("::")[-1]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    if "stft" in k or "window_tg" in k: print(k, {c: f"{v:.4g}" for c, v in d.items()})
PY
timeout -k 10 400 python -u -m pytest tests/test_gpu_shared_tuning.py tests/test_gpu_chroma.py -x -q --timeout 150 --timeout-method thread > $O/pt.log 2>&1 || { echo "tests failed"; tail -30 $O/pt.log; exit 1; }
tail -2 $O/pt.log
