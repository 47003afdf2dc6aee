#!/bin/bash
# Rotated A/B of libncgpu.so variants against the in-tree build, with a determinism /
# bit-identity check of the first variant.   usage: tools/r5_var.sh TAG VARIANT...
set -o pipefail
TAG=${1:-r5v}; shift
O=gpurun_out/$TAG
mkdir -p $O
IN=nightcore-to-flac-analyzer_amd/nightcore_analyzer/_lib/libncgpu.so
V=""
for v in "$@"; do V="$V tools/var/$v/libncgpu.so"; done
timeout -k 10 180 python3 -u tools/det_check.py tools/var/$1/libncgpu.so $IN > $O/det.txt 2>&1 || { echo "det failed"; tail -20 $O/det.txt; exit 1; }
tail -4 $O/det.txt
timeout -k 10 400 python3 -u tools/var_bench.py $IN $V > $O/vb.txt 2>&1 || { echo "vb failed"; tail -20 $O/vb.txt; exit 1; }
cat $O/vb.txt | tail -14
