#!/bin/bash
# Alternating runs of the default bench command (`python bench.py`, as the driver runs it) under
# environment variants on one box.   usage: tools/ab_full.sh TAG ROUNDS "name:VAR=val ..."
set -o pipefail
TAG=${1:-abf}; ROUNDS=${2:-3}; SPECS=${3:-"base"}
O=gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for spec in $SPECS; do
    name=${spec%%:*}; vars=""
    [ "$name" != "$spec" ] && vars=${spec#*:} && vars=${vars//,/ }
    env $vars timeout -k 10 400 python3 -u bench.py > $O/${name}_$r.json 2> $O/${name}_$r.err || { echo "bench $name failed"; tail -5 $O/${name}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/${name}_$r.json')); r=d['roofline']; i=r['isolated']
print('$name round $r', round(d['value']), 'windows/s', round(d['ms_per_step'],3), 'ms/step; stft_mel', round(r['avg_launch_ms'],4), 'ms/launch in pipeline, frac', round(r['frac'],4), '; isolated', round(i['kernels_ms_per_step']['stft_mel'],3), 'ms/step; idle', round(d['device_idle_frac'],4))"
  done
done
