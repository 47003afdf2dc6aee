#!/bin/bash
# The round's closing GPU session from one build: the GPU suite and smoke, then the round
# measurement (tools/gpu_round4.sh: PMC traffic, issue passes, bench line, rocprofv3 of the same
# bench command cut to its timed region).   usage: tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-r4final}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_round4.sh $TAG
