#!/bin/bash
# The N-rank bench path rehearsed on one GPU (NC_BENCH_REHEARSE=1: gloo, ranks share the device):
# window-sharded (the --gpus N default) with 64 pairs per rank, so N = 8 is BASELINE config 4's
# 512-pair batch.   usage: tools/rehearse_n.sh OUTDIR N [extra bench args]
set -o pipefail
O=$1; N=$2; shift 2
mkdir -p $O
NC_BENCH_REHEARSE=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 5 --warmup 2 \
  --no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload "$@" > $O/n$N.json 2> $O/n$N.err \
  || { echo "rehearsal N=$N failed"; tail -20 $O/n$N.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/n$N.json').read().strip().splitlines()[-1])
print('N=$N', round(d['value']), 'windows/s', round(d['ms_per_step'], 2), 'ms/step', d['config']['parallelism'], d['data'][-40:])
print('  modes', {k: (round(v['value']), round(v['ms_per_step'], 2)) for k, v in (d.get('modes') or {}).items()})"
