#!/bin/bash
# Round 5: the one-tile-per-wave octave 0-2 CQT (NC_CQL2) against the in-tree build:
# determinism and bit-identity (tools/det_check.py), unaligned chunks (var_bench checksums),
# the chroma GPU tests through the variant, and the rotated timer.
# usage: tools/r5_cql2.sh TAG VARIANT...
set -o pipefail
TAG=${1:-r5c}; shift
O=gpurun_out/$TAG
mkdir -p $O
IN=nightcore-to-flac-analyzer_amd/nightcore_analyzer/_lib/libncgpu.so
V=""
for v in "$@"; do V="$V tools/var/$v/libncgpu.so"; done
FIRST=tools/var/$1/libncgpu.so
timeout -k 10 180 python3 -u tools/det_check.py $FIRST $IN > $O/det.txt 2>&1 || { echo "det failed"; tail -20 $O/det.txt; exit 1; }
cat $O/det.txt
VB_CHUNKSHIFT=1 timeout -k 10 240 python3 -u tools/var_bench.py $IN $V > $O/vb_shift1.txt 2>&1 || { echo "vb shift failed"; tail -20 $O/vb_shift1.txt; exit 1; }
NCGPU_LIB=$FIRST timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chroma.py tests/test_gpu_shared_tuning.py > $O/pytest_chroma.txt 2>&1 || { echo "chroma tests failed"; tail -30 $O/pytest_chroma.txt; exit 1; }
tail -3 $O/pytest_chroma.txt
timeout -k 10 300 python3 -u tools/var_bench.py $IN $V > $O/vb.txt 2>&1 || { echo "vb failed"; tail -20 $O/vb.txt; exit 1; }
grep -v "^ " $O/vb_shift1.txt | tail -4
cat $O/vb.txt | tail -6
