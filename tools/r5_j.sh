#!/bin/bash
# MELODIA GPU tests, then per-step kernel tables (rocprofv3 --kernel-trace --stats of
# tools/prof_step.py), streams concurrent and serialized.
set -o pipefail
O=gpurun_out/r5j
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_melodia.py > $O/melodia.log 2>&1 || { echo "melodia failed"; tail -30 $O/melodia.log; exit 1; }
tail -3 $O/melodia.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/conc -o run --output-format csv -- python3 $R/tools/prof_step.py 5 > $R/$O/conc.log 2>&1 || { echo "prof conc failed"; tail -10 $R/$O/conc.log; exit 1; }
cd /tmp && NC_SERIAL_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/ser -o run --output-format csv -- python3 $R/tools/prof_step.py 5 > $R/$O/ser.log 2>&1 || { echo "prof ser failed"; tail -10 $R/$O/ser.log; exit 1; }
cd $R
python3 tools/step_table.py $(find $O/ser -name '*kernel_stats.csv' | head -1) 6 > $O/ser_table.txt
python3 tools/step_table.py $(find $O/conc -name '*kernel_stats.csv' | head -1) 6 > $O/conc_table.txt
head -40 $O/ser_table.txt
tail -1 $O/conc_table.txt
