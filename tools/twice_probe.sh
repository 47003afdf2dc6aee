#!/bin/bash
# In-pipeline cost of single kernels: each tools/var/<v> build launches one kernel twice
# (NC_PROBE_TWICE, nc_engine.h); the step's growth over the in-tree build is that launch's
# cost inside the pipelined step.   usage: tools/twice_probe.sh OUTDIR VARIANT...
set -o pipefail
O=$1; shift
mkdir -p $O
for round in 1 2; do
  for v in _lib "$@"; do
    lib=nightcore-to-flac-analyzer_amd/nightcore_analyzer/_lib/libncgpu.so
    [ "$v" != _lib ] && lib=tools/var/$v/libncgpu.so
    NCGPU_LIB=$lib NC_PROBE_ROUNDS=2 timeout -k 10 240 python3 -u tools/idle_probe.py 10 default > $O/$v.$round.txt 2>&1 \
      || { echo "$v failed"; tail -5 $O/$v.$round.txt; exit 1; }
    echo "$v round $round: $(grep 'ms/step' $O/$v.$round.txt)"
  done
done
