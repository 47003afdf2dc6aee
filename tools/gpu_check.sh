#!/bin/bash
# One GPU session: parity tests, smoke, bench line, rocprofv3 kernel stats of the same bench command.
# usage: tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-run}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-ibi --no-config5 > $GRAFT_REPO_ROOT/$O/prof_bench.json 2> $GRAFT_REPO_ROOT/$O/prof.err || { echo "rocprof failed"; tail -20 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
cat $GRAFT_REPO_ROOT/$O/prof_bench.json
find $GRAFT_REPO_ROOT/$O/prof -name '*kernel_stats.csv' | head -3
