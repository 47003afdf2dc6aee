#!/bin/bash
# CQT fragment scheduling / occupancy variants: rotated timings, determinism, chroma parity, GPU suite
set -o pipefail
O=gpurun_out/p6
mkdir -p $O
V=tools/var
VB_TUNING=1 timeout -k 10 300 python3 tools/var_bench.py $V/cur/libncgpu.so $V/oldlb/libncgpu.so $V/newsched/libncgpu.so $V/newlb/libncgpu.so $V/lowsched/libncgpu.so $V/twb15/libncgpu.so > $O/t1.log 2>&1 || { echo "var failed"; tail -20 $O/t1.log; exit 1; }
grep -v amdgpu.ids $O/t1.log
timeout -k 10 200 python3 tools/det_check.py $V/lowsched/libncgpu.so $V/cur/libncgpu.so > $O/det.log 2>&1 || { echo "det failed"; tail -20 $O/det.log; exit 1; }
grep -v amdgpu.ids $O/det.log | tail -6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pt.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/pt.log | head; tail -5 $O/pt.log; exit 1; }
tail -2 $O/pt.log
