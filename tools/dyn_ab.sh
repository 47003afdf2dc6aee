#!/bin/bash
# The workgroup frame queue (WgFrameQueue: stft_mel, tuning_peaks, spectral_frames take their
# frames one at a time from an LDS counter) against the static interleave (tools/var/static:
# -DSM_DYN_=0 -DTP_DYN_=0) in the rotated timer, then the GPU suite, smoke and the bench line.
# usage: tools/dyn_ab.sh TAG
set -o pipefail
TAG=${1:-r6q}
O=gpurun_out/$TAG
mkdir -p $O
B=nightcore-to-flac-analyzer_amd/nightcore_analyzer/_lib/libncgpu.so
timeout -k 10 400 python3 -u tools/var_bench.py $B tools/var/static/libncgpu.so > $O/var_bench.txt 2>&1 || { echo "var bench failed"; tail -20 $O/var_bench.txt; exit 1; }
cat $O/var_bench.txt
bash tools/r6_check.sh $TAG
