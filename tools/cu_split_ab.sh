#!/bin/bash
# the window chain and the chroma chain on complementary CU sets
# (NC_CU_SPLIT, hipExtStreamCreateWithCUMask; the persistent STFT / tuning grids sized to
# them) against the shared-CU default, alternating bench runs on one box.
# usage: tools/cu_split_ab.sh TAG ROUNDS "SPEC1 SPEC2 ..."   (SPEC = k[:form], "none" = default)
set -o pipefail
TAG=${1:-r6cu}; ROUNDS=${2:-2}; SPECS=${3:-"none 128 160 96 128:low"}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq 1 $ROUNDS); do
  for spec in $SPECS; do
    if [ "$spec" = none ]; then
      env_=""
    else
      k=${spec%%:*}
      env_="NC_CU_SPLIT=$spec NC_STFT_CUS=$k NC_CHROMA_CUS=$((256 - k))"
    fi
    env $env_ timeout -k 10 300 python3 -u bench.py --steps 20 --no-cpu-baseline --no-ibi --no-config5 --no-spectral \
      --no-resample --no-upload > $O/b_${spec/:/_}_$r.json 2> $O/b_${spec/:/_}_$r.err || { echo "bench $spec failed"; tail -5 $O/b_${spec/:/_}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b_${spec/:/_}_$r.json')); k=d['kernels_ms_per_step']
print('$spec', 'round $r', round(d['ms_per_step'],3), 'ms/step', {x: round(k[x],3) for x in ('stft_mel','cqt_low','cqt_high','window_tg','tuning_peaks','decimate') if x in k})"
  done
done
