#!/bin/bash
# HBM traffic per launch of the bench's kernels: two rocprofv3 counter passes (FETCH_SIZE, then
# WRITE_SIZE: they do not fit one pass) over the bench command, each under its own limit, then
# tools/traffic.py -> profiles/NAME (default r3_traffic.json).     usage: tools/pmc_traffic.sh OUTDIR [NAME]
set -o pipefail
OUT=$1
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p $R/$OUT
for c in FETCH_SIZE WRITE_SIZE; do
  cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $R/$OUT/$c -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-ibi --no-config5 > $R/$OUT/$c.log 2>&1 || { echo "pass $c failed"; tail -5 $R/$OUT/$c.log; exit 1; }
done
cd $R && python3 tools/traffic.py $OUT ${2:-r3_traffic.json} $3
