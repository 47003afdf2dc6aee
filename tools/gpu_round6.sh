#!/bin/bash
# Round 6 measurement in one GPU call, from the build under test:
#   1. FETCH_SIZE / WRITE_SIZE calibration of the access forms the kernels use
#      (tools/calib_fetch.hip -> profiles/r6_fetch_calibration.json);
#   2. HBM traffic per launch of the bench's kernels, corrected per kernel with those scales
#      (tools/pmc_traffic.sh -> profiles/r6_traffic.json, which the bench line's roofline reads);
#   3. the default bench line;
#   4. rocprofv3 --kernel-trace --stats of the same bench command cut to its timed region.
# usage: tools/gpu_round6.sh TAG
set -o pipefail
TAG=${1:-r6m}
O=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p $O
export TMPDIR=/tmp
[ -x tools/calib_fetch ] || /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/calib_fetch.hip -o tools/calib_fetch
for c in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $R/$O/calib/$c -o run -- $R/tools/calib_fetch > $R/$O/calib_$c.log 2>&1 || { echo "calib $c failed"; tail -5 $R/$O/calib_$c.log; exit 1; }
done
cd $R && python3 tools/calib_report.py $O/calib profiles/r6_fetch_calibration.json || exit 1
bash tools/pmc_traffic.sh $O/pmc r6_traffic.json profiles/r6_fetch_calibration.json > $O/traffic.log 2>&1 || { echo "traffic failed"; tail -20 $O/traffic.log; exit 1; }
python3 -c "
import json; d=json.load(open('profiles/r6_traffic.json'))
for k, v in d['kernels'].items(): print(k, v['hbm_bytes_per_launch'], v.get('alg_bytes_per_launch'), v.get('calibration'))"
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo "rocprof failed"; tail -20 $R/$O/prof.err; exit 1; }
cd $R && python3 tools/rocprof_timed.py $O/prof/run_kernel_trace.csv $O/prof_bench.json $O/rocprof_timed.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('value', round(d['value']), 'ms', round(d['ms_per_step'],3), 'dom', r['kernel'], round(r['avg_launch_ms'],4), round(r['frac'],4), r.get('traffic'))
print('kernels', d['kernels_ms_per_step'])"
head -16 $O/prof/run_kernel_stats.csv | cut -c1-140
