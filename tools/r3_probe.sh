#!/bin/bash
# Times tools/var/<name>/libncgpu.so variants in rotation (tools/var_bench.py).  usage: tools/r3_probe.sh TAG name...
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
libs=""
for n in "$@"; do libs="$libs tools/var/$n/libncgpu.so"; done
timeout -k 10 400 python3 tools/var_bench.py $libs > $O/var.log 2>&1 || { echo "var failed"; tail -20 $O/var.log; exit 1; }
grep -v amdgpu.ids $O/var.log
