#!/bin/bash
# determinism + bit-identity of CQT variants against the in-tree build, then the rotated timer
# usage: tools/r5_det.sh TAG "DET_VARIANTS" "TIMING_ONLY_VARIANTS"
set -o pipefail
TAG=${1:-r5d}
O=gpurun_out/$TAG
mkdir -p $O
IN=nightcore-to-flac-analyzer_amd/nightcore_analyzer/_lib/libncgpu.so
V=""
for v in $2; do
  V="$V tools/var/$v/libncgpu.so"
  timeout -k 10 120 python3 -u tools/det_check.py tools/var/$v/libncgpu.so $IN > $O/det_$v.txt 2>&1 || { echo "det $v failed"; tail -20 $O/det_$v.txt; exit 1; }
  grep -v amdgpu.ids $O/det_$v.txt | grep -v "^_lib"
done
for v in $3; do V="$V tools/var/$v/libncgpu.so"; done
timeout -k 10 400 python3 -u tools/var_bench.py $IN $V > $O/vb.txt 2>&1 || { echo "vb failed"; tail -20 $O/vb.txt; exit 1; }
grep -v amdgpu.ids $O/vb.txt | tail -12 | sed -e 's/checksum onset.*chroma/chroma/' -e "s/'stft_mel'.*'decimate'/.. 'decimate'/"
