#!/bin/bash
# One GPU session: the GPU suite, smoke, a short bench line.   usage: tools/r3_check.sh TAG
set -o pipefail
TAG=${1:-check}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -30; tail -5 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print('value', round(d['value']), 'ms', round(d['ms_per_step'],3), 'dom', r['kernel'], round(r['avg_launch_ms'],4), round(r['frac'],4))
print('kernels', d['kernels_ms_per_step']); print('iso', r['isolated']['kernels_ms_per_step'])
c=r.get('cqt_chroma') or {}; print('cqt', c.get('avg_launch_ms'), c.get('parts_ms'), c.get('compute'))"
