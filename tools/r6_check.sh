#!/bin/bash
# Round 6 GPU session: GPU suite + smoke, the vmcnt ordering probe, kernel variants
# in the rotated timer (tools/var/*), and the default bench line.
# usage: tools/r6_check.sh TAG
set -o pipefail
TAG=${1:-r6}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|passed|failed" $O/pytest_gpu.log | tail -30; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -x tools/probe/vmcnt_order ]; then
  timeout -k 10 120 ./tools/probe/vmcnt_order 40 > $O/vmcnt_order.txt 2>&1 || { echo "vmcnt probe failed"; cat $O/vmcnt_order.txt; exit 1; }
  cat $O/vmcnt_order.txt
fi
if ls tools/var/*/libncgpu.so > /dev/null 2>&1; then
  timeout -k 10 400 python3 -u tools/var_bench.py tools/var/*/libncgpu.so > $O/var_bench.txt 2>&1 || { echo "var bench failed"; tail -20 $O/var_bench.txt; exit 1; }
  cat $O/var_bench.txt
fi
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print('value', round(d['value']), 'ms', round(d['ms_per_step'],3), 'dom', r['kernel'], round(r['avg_launch_ms'],4), round(r['frac'],4))
print('kernels', d['kernels_ms_per_step'])
print('upload', {k: (round(v, 3) if isinstance(v, float) else v) for k, v in d.get('upload_included', {}).items() if k != 'how'})"
