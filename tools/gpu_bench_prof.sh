#!/bin/bash
# One GPU call: the default bench line (CPU baseline included) and a rocprofv3 kernel-trace
# summary of the same step (timed region only, side measurements off).
#   usage: tools/gpu_bench_prof.sh TAG      (writes gpurun_out/TAG/)
set -o pipefail
TAG=${1:-bench}
O=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload \
  --no-ibi > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo "rocprof failed"; tail -20 $R/$O/prof.err; exit 1; }
cd $R && python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('value', round(d['value']), 'ms', round(d['ms_per_step'],3), 'dom', r['kernel'], round(r['avg_launch_ms'],4), round(r['frac'],4), round(r['compute']['frac'],4))
print('kernels', d['kernels_ms_per_step']); print('iso', r['isolated']['kernels_ms_per_step'])
print('upload', d.get('upload_included')); print('cpu', d.get('cpu_baseline'))"
