#!/bin/bash
# Round 5: where the device idles in the pipelined step. The bench line (timed steps only),
# then the same bench under rocprofv3 with kernel, memory-copy and HIP runtime traces, and
# tools/gap_host.py: each device gap of the timed region with the host API calls inside it.
# usage: tools/r5_gap.sh TAG
set -o pipefail
TAG=${1:-r5gap}
O=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p $O
export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-config5 --no-spectral --no-resample --no-upload"
timeout -k 10 300 python -u bench.py $ARGS > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d $R/$O/tr -o run \
  --output-format csv -- python3 $R/bench.py $ARGS --steps 12 --warmup 2 > $R/$O/tr_bench.json 2> $R/$O/tr.err \
  || { echo "trace failed"; tail -20 $R/$O/tr.err; exit 1; }
cd $R && python3 tools/gap_host.py $O/tr/run 200 > $O/gaps.txt 2>&1
python3 tools/trace_gaps.py $O/tr/run_kernel_trace.csv 200 > $O/kgaps.txt 2>&1
gzip -f $O/tr/*.csv
python3 -c "
import json; d=json.load(open('$O/bench.json')); print('value', round(d['value']), 'ms', round(d['ms_per_step'],3))"
head -60 $O/gaps.txt
