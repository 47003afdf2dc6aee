#!/bin/bash
# Round 6 A/B session: (1) window energies from the trim's block sums against the round-5 per-frame
# STFT energies (NC_BLOCK_ENERGY=0), alternating bench runs; (2) CU-partitioned chains
# (tools/cu_split_ab.sh); (3) one rank's N > 1 step with the record gather (tools/rank_step_probe.py).
# usage: tools/r6_ab.sh TAG
set -o pipefail
TAG=${1:-r6ab}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for e in 0 1; do
    NC_BLOCK_ENERGY=$e timeout -k 10 300 python3 -u bench.py --steps 30 --no-cpu-baseline --no-ibi --no-config5 \
      --no-spectral --no-resample --no-upload > $O/en${e}_$r.json 2> $O/en${e}_$r.err || { echo "bench en$e failed"; tail -5 $O/en${e}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/en${e}_$r.json')); k=d['kernels_ms_per_step']; i=d['roofline']['isolated']['kernels_ms_per_step']
print('block_energy=$e round $r', round(d['ms_per_step'],3), 'ms/step; stft_mel', round(d['roofline']['avg_launch_ms'],4), 'ms/launch in pipeline,', round(i['stft_mel'],3), 'ms/step isolated; frac', round(d['roofline']['frac'],4))"
  done
done
bash tools/cu_split_ab.sh $TAG/cu 2 "none 128 160 96 128:low" || exit 1
timeout -k 10 300 python3 -u tools/rank_step_probe.py 10 3 > $O/rank_step_probe.txt 2>&1 || { echo "rank probe failed"; tail -10 $O/rank_step_probe.txt; exit 1; }
cat $O/rank_step_probe.txt
