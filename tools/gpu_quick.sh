#!/bin/bash
# Quick GPU iteration: GPU parity tests, isolated kernel stats for the chroma and window
# paths, one bench line without the CPU baseline.   usage: tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-quick}
O=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for t in chroma windows; do
  cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/$t -o run --output-format csv -- python3 $R/tools/prof_kernels.py $t > $R/$O/$t.log 2>&1 || { echo "stats $t failed"; tail -5 $R/$O/$t.log; exit 1; }
done
cd $R && timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 tools/pmc_report.py $O/chroma $O/windows
python3 -c "import json; d=json.load(open('$O/bench.json')); print('value', round(d['value']), 'ms', round(d['ms_per_step'],3), d['kernels_ms_per_step'])"
