#!/bin/bash
# Where the pipelined step's time goes after a kernel change: concurrency of the timed kernels
# (tools/concurrency_spans.py, untraced spans) and the host side with a few group schedules
# (tools/host_probe.py).   usage: tools/step_probe.sh TAG [schedules...]
set -o pipefail
TAG=${1:-r6sp}; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 -u tools/concurrency_spans.py 10 > $O/concurrency.txt 2>&1 || { echo "concurrency failed"; tail -20 $O/concurrency.txt; exit 1; }
cat $O/concurrency.txt
timeout -k 10 400 python3 -u tools/host_probe.py 10 ${@:-default} > $O/host_probe.txt 2>&1 || { echo "host probe failed"; tail -20 $O/host_probe.txt; exit 1; }
head -60 $O/host_probe.txt
