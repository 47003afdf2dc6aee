#!/bin/bash
# Aligned vs odd-offset windows / chunks for two builds (tools/var/cur, tools/var/odd), then the GPU suite
set -o pipefail
O=gpurun_out/p21
mkdir -p $O
for sh in 0 1; do
  VB_WINSHIFT=$sh VB_CHUNKSHIFT=$sh timeout -k 10 300 python3 tools/var_bench.py tools/var/cur/libncgpu.so tools/var/odd/libncgpu.so tools/var/odd2/libncgpu.so tools/var/odd3/libncgpu.so > $O/s$sh.log 2>&1 || { echo "var failed"; tail -20 $O/s$sh.log; exit 1; }
  echo "shift $sh"; grep -v amdgpu.ids $O/s$sh.log
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pt.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/pt.log | head; tail -5 $O/pt.log; exit 1; }
tail -2 $O/pt.log
