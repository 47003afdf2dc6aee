#!/bin/bash
# GPU suite, smoke and the default bench line from the current tree.   usage: tools/r5_check.sh TAG
set -o pipefail
TAG=${1:-r5check}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|passed|failed" $O/pytest_gpu.log | tail -30; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('value', round(d['value']), 'ms', round(d['ms_per_step'],3), 'idle', d.get('device_idle_frac'), 'dom', r['kernel'], round(r['avg_launch_ms'],4), round(r['frac'],4))
print('iso', r['isolated']['kernels_ms_per_step'])"
