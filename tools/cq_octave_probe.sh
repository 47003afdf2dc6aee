#!/bin/bash
# cqt_low per-octave probe in the rotated timer: each octave alone (CQL_ONLY) with and without
# waiting for its next block's loads before the split (C2_NOBW_, outputs wrong), against the
# product library.  Build first (here):
#   tools/var_build.sh o0:cqt.hip:-DCQL_ONLY=0 o0nobw:cqt.hip:"-DCQL_ONLY=0 -DC2_NOBW_=1" \
#     o1:cqt.hip:-DCQL_ONLY=1 o1nobw:cqt.hip:"-DCQL_ONLY=1 -DC2_NOBW_=1 -DC2_NOBW_OCT_=1" allnobw0:cqt.hip:-DC2_NOBW_=1
# usage: tools/cq_octave_probe.sh [TAG]
set -o pipefail
O=gpurun_out/${1:-r6cq}
mkdir -p $O
B=nightcore-to-flac-analyzer_amd/nightcore_analyzer/_lib/libncgpu.so
timeout -k 10 500 python3 -u tools/var_bench.py $B tools/var/o0/libncgpu.so tools/var/o0nobw/libncgpu.so tools/var/o1/libncgpu.so \
  tools/var/o1nobw/libncgpu.so tools/var/allnobw0/libncgpu.so > $O/var_bench.txt 2>&1 || { echo "var bench failed"; tail -20 $O/var_bench.txt; exit 1; }
cat $O/var_bench.txt
