#!/bin/bash
# Round measurement in one GPU call, from the final build (the evidence the
# bench line cites, from the same session):
#   1. HBM traffic per launch: rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE (-> profiles/r5_traffic.json,
#      which the bench line's roofline.traffic reads);
#   2. issue / LDS / MFMA counter passes of stft_mel and the CQT on the kernel-isolation driver;
#   3. the default bench line;
#   4. rocprofv3 --kernel-trace --stats of the same bench command (less the host-only CPU baseline
#      leg), cut to its timed region by tools/rocprof_timed.py: per-kernel averages and the
#      roofline fractions recomputed from them beside the profiled run's own line.
# Round 5 adds the GPU suite and smoke at the end.
# usage: tools/gpu_round5.sh TAG (run tools/stamp_commit.sh first)
set -o pipefail
TAG=${1:-r5final}
O=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p $O
export TMPDIR=/tmp
bash tools/pmc_traffic.sh $O/pmc r5_traffic.json > $O/traffic.log 2>&1 || { echo "traffic failed"; tail -20 $O/traffic.log; exit 1; }
cp profiles/r5_traffic.json $O/
bash tools/pmc_passes.sh $O/issue windows chroma > $O/issue.log 2>&1 || { echo "issue passes failed"; tail -20 $O/issue.log; exit 1; }
python3 tools/pmc_report.py $O/issue/windows/stats $O/issue/windows/p1 $O/issue/windows/p2 $O/issue/windows/p3 \
  $O/issue/chroma/stats $O/issue/chroma/p1 $O/issue/chroma/p2 $O/issue/chroma/p3 > $O/issue_report.body 2>&1
{ echo "# build: $(python3 -c 'import json, bench; print(json.dumps(bench.build_provenance()))')"; cat $O/issue_report.body; } > $O/issue_report.txt
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- \
  python3 $R/bench.py --no-cpu-baseline > $R/$O/prof_bench.json 2> $R/$O/prof.err || { echo "rocprof failed"; tail -20 $R/$O/prof.err; exit 1; }
cd $R && python3 tools/rocprof_timed.py $O/prof/run_kernel_trace.csv $O/prof_bench.json $O/rocprof_timed.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('value', round(d['value']), 'ms', round(d['ms_per_step'],3), 'dom', r['kernel'], round(r['avg_launch_ms'],4), round(r['frac'],4), r.get('traffic'))"
head -14 $O/prof/run_kernel_stats.csv | cut -c1-140
cat $O/issue_report.txt | head -40
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|passed|failed" $O/pytest_gpu.log | tail -30; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
