#!/bin/bash
# bootstrap GPU tests, then the serialized per-step kernel table (rocprofv3 --stats of tools/prof_step.py)
set -o pipefail
O=gpurun_out/${1:-r5k}
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bootstrap.py tests/test_gpu_pipeline.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; exit 1; }
tail -2 $O/tests.log
cd /tmp && NC_SERIAL_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/ser -o run --output-format csv -- python3 $R/tools/prof_step.py 5 > $R/$O/ser.log 2>&1 || { echo "prof ser failed"; tail -10 $R/$O/ser.log; exit 1; }
cd $R && python3 tools/step_table.py $(find $O/ser -name '*kernel_stats.csv' | head -1) 6 > $O/ser_table.txt
head -14 $O/ser_table.txt; tail -1 $O/ser_table.txt
