#!/bin/bash
# Chroma parity tests, a short bench line and rocprofv3 kernel stats of it (CQT iteration loop).
#   usage: tools/gpu_quick_cqt.sh TAG
set -o pipefail
TAG=${1:-cq}
O=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_chroma.py tests/test_gpu_shared_tuning.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload --no-ibi > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('ms', round(d['ms_per_step'],3), 'value', round(d['value']))
print('kernels', d['kernels_ms_per_step']); print('iso', r['isolated']['kernels_ms_per_step'])"
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload \
  --no-ibi > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo "rocprof failed"; tail -20 $R/$O/prof.err; exit 1; }
head -8 $R/$O/prof/run_kernel_stats.csv | cut -c1-160
