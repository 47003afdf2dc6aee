#!/bin/bash
# stft_mel with its waves kept together (SM_SYNC_: a workgroup barrier every N frame groups) against
# the free-running waves: the rotated timer (tools/var_bench.py), stft_mel's HBM traffic per launch
# in the bench (tools/pmc_traffic.sh with NCGPU_LIB per variant) and alternating bench runs.
# Build first (here): tools/var_build.sh sync4:stft.hip:-DSM_SYNC_=4 ...
# usage: tools/stft_sync_ab.sh TAG "VARIANTS" ["EXTRA var_bench libs"]   (VARIANTS: tools/var/<name>; base = the product)
set -o pipefail
TAG=${1:-r6sync}; VARS=${2:-"sync1 sync4"}; EXTRA=${3:-}
O=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p $O
export TMPDIR=/tmp
BASE=nightcore-to-flac-analyzer_amd/nightcore_analyzer/_lib/libncgpu.so
libs="$BASE"; for v in $VARS; do libs="$libs tools/var/$v/libncgpu.so"; done
for e in $EXTRA; do libs="$libs tools/var/$e/libncgpu.so"; done
timeout -k 10 500 python3 -u tools/var_bench.py $libs > $O/var_bench.txt 2>&1 || { echo "var bench failed"; tail -20 $O/var_bench.txt; exit 1; }
cat $O/var_bench.txt
for v in base $VARS; do
  lib=$R/$BASE; [ $v != base ] && lib=$R/tools/var/$v/libncgpu.so
  NCGPU_LIB=$lib bash tools/pmc_traffic.sh $O/pmc_$v stft_sync_${v}_traffic.json > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/pmc_$v.log; exit 1; }
  python3 -c "
import json; d=json.load(open('profiles/stft_sync_${v}_traffic.json'))['kernels']['stft_mel']
print('$v stft_mel traffic per launch', d['hbm_bytes_per_launch'], 'alg', d.get('alg_bytes_per_launch'))"
done
specs="base"; for v in $VARS; do specs="$specs $v:NCGPU_LIB=$R/tools/var/$v/libncgpu.so"; done
NO_PMC=1 NO_CU=1 NO_RANK=1 bash tools/r6_ab.sh $TAG/ab 2 "$specs"
