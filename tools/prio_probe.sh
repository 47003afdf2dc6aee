#!/bin/bash
# Stream-priority probe: the chroma/tail side streams at several NC_STREAM_PRIO settings,
# alternated so that box drift hits every setting alike.   usage: tools/prio_probe.sh TAG
set -o pipefail
TAG=${1:-prio}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do
  for p in 0,0 -1,0 -1,-1 0,-1; do
    NC_STREAM_PRIO=$p timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-ibi --no-config5 \
      --no-spectral --no-resample > $O/bench_${p}_$rep.json 2> $O/bench_${p}_$rep.err || { echo "bench $p failed"; tail -5 $O/bench_${p}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${p}_$rep.json')); print('prio $p rep $rep', round(d['value']), round(d['ms_per_step'], 3))"
  done
done
