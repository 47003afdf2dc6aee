#!/bin/bash
# Round 6 A/B session, alternating short bench runs of environment variants on one box:
#   blocks0 = NC_BLOCK_ENERGY=0: the round-5 per-frame STFT energies (round 6: from the trim's block sums);
#   dynN    = NC_STFT_DYN=N: stft_mel's waves take runs of N frames from a counter (default: static ranges);
# then the CU-partitioned chains (tools/cu_split_ab.sh) and one rank's N > 1 step with the record
# gather (tools/rank_step_probe.py).
# usage: tools/r6_ab.sh TAG [ROUNDS] [SPECS]   SPEC = name:VAR=val[,VAR=val]  ("base" = no variables)
# NO_PMC / NO_CU / NO_RANK skip the XCD counter pass, the CU split and the rank probe
set -o pipefail
TAG=${1:-r6ab}; ROUNDS=${2:-2}; SPECS=${3:-"base blocks0:NC_BLOCK_ENERGY=0 dyn128:NC_STFT_DYN=128 dyn512:NC_STFT_DYN=512 xcd:NCGPU_LIB=$GRAFT_REPO_ROOT/tools/var/xcd/libncgpu.so"}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq 1 $ROUNDS); do
  for spec in $SPECS; do
    name=${spec%%:*}; vars=""
    [ "$name" != "$spec" ] && vars=${spec#*:} && vars=${vars//,/ }
    env $vars timeout -k 10 300 python3 -u bench.py --steps 30 --no-cpu-baseline --no-ibi --no-config5 \
      --no-spectral --no-resample --no-upload > $O/${name}_$r.json 2> $O/${name}_$r.err || { echo "bench $name failed"; tail -5 $O/${name}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/${name}_$r.json')); i=d['roofline']['isolated']['kernels_ms_per_step']
print('$name round $r', round(d['ms_per_step'],3), 'ms/step; stft_mel', round(d['roofline']['avg_launch_ms'],4), 'ms/launch in pipeline,', round(i['stft_mel'],3), 'ms/step isolated; frac', round(d['roofline']['frac'],4), 'idle', round(d['device_idle_frac'],4))"
  done
done
if [ -z "$NO_PMC" ] && [ -f tools/var/xcd/libncgpu.so ]; then   # cqt_low bytes with the XCD-contiguous order
  NCGPU_LIB=$GRAFT_REPO_ROOT/tools/var/xcd/libncgpu.so bash tools/pmc_traffic.sh $O/pmc_xcd xcd_probe_traffic.json > $O/pmc_xcd.log 2>&1 || { echo "xcd pmc failed"; tail -5 $O/pmc_xcd.log; exit 1; }
  python3 -c "
import json; d=json.load(open('profiles/xcd_probe_traffic.json'))['kernels']
print('xcd probe traffic', {k: d[k]['hbm_bytes_per_launch'] for k in ('cqt_low', 'cqt_high', 'stft_mel') if k in d})"
fi
if [ -z "$NO_CU" ]; then
  bash tools/cu_split_ab.sh $TAG/cu 2 "none 128 160 96 128:low" || exit 1
fi
if [ -z "$NO_RANK" ]; then
  timeout -k 10 300 python3 -u tools/rank_step_probe.py 10 3 > $O/rank_step_probe.txt 2>&1 || { echo "rank probe failed"; tail -10 $O/rank_step_probe.txt; exit 1; }
  cat $O/rank_step_probe.txt
fi
