#!/bin/bash
# bench.py step time of the in-tree library against tools/var/<name>/libncgpu.so, alternating.
# usage: tools/r3_ab_bench.sh TAG VARIANT
set -o pipefail
TAG=${1:-ab}; VAR=${2:-base}
O=gpurun_out/$TAG
mkdir -p $O
LIB=nightcore-to-flac-analyzer_amd/nightcore_analyzer/_lib/libncgpu.so
cp $LIB $O/cur.so
for r in 1 2; do
  for v in cur $VAR; do
    if [ $v = cur ]; then cp $O/cur.so $LIB; else cp tools/var/$VAR/libncgpu.so $LIB; fi
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload > $O/$v.$r.json 2> $O/$v.$r.err || { echo "bench $v failed"; tail -5 $O/$v.$r.err; cp $O/cur.so $LIB; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$v.$r.json').read().strip().splitlines()[-1]); print('$v', $r, round(d['ms_per_step'],3), {k: round(v,2) for k,v in d['kernels_ms_per_step'].items()})"
  done
done
cp $O/cur.so $LIB
