#!/bin/bash
# Round measurement in one GPU call: PMC traffic passes (-> profiles/r3_traffic.json, copied to
# the output dir), the default bench line (which reads that traffic file), and a rocprofv3
# kernel-stats summary of the timed region.     usage: tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-round}
O=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p $O
export TMPDIR=/tmp
bash tools/pmc_traffic.sh $O/pmc > $O/traffic.log 2>&1 || { echo "traffic failed"; tail -20 $O/traffic.log; exit 1; }
cp profiles/r3_traffic.json $O/
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload \
  --no-ibi > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo "rocprof failed"; tail -20 $R/$O/prof.err; exit 1; }
cd $R && python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('value', round(d['value']), 'ms', round(d['ms_per_step'],3), 'dom', r['kernel'], round(r['avg_launch_ms'],4), round(r['frac'],4), r.get('traffic'))
print('kernels', d['kernels_ms_per_step']); print('iso', r['isolated']['kernels_ms_per_step'])
print('cpu', d.get('cpu_baseline', {}).get('value'))"
head -12 $O/prof/run_kernel_stats.csv | cut -c1-140
