#!/bin/bash
# Round 6 issue / MFMA passes of the final build (tools/pmc_passes.sh over tools/prof_kernels.py,
# report in gpurun_out/TAG/issue_report.txt) and cqt_low's HBM bytes with the XCD-contiguous order
# (tools/var/xcd, built here first: tools/var_build.sh xcd:cqt.hip:-DC2_XCD_=1).   usage: tools/r6_issue.sh TAG
set -o pipefail
TAG=${1:-r6i}
O=gpurun_out/$TAG
R=$GRAFT_REPO_ROOT
mkdir -p $O
export TMPDIR=/tmp
bash tools/pmc_passes.sh $O/issue windows chroma > $O/issue.log 2>&1 || { echo "issue passes failed"; tail -20 $O/issue.log; exit 1; }
python3 tools/pmc_report.py $O/issue/windows/stats $O/issue/windows/p1 $O/issue/windows/p2 $O/issue/windows/p3 \
  $O/issue/chroma/stats $O/issue/chroma/p1 $O/issue/chroma/p2 $O/issue/chroma/p3 > $O/issue_report.body 2>&1
{ echo "# build: $(python3 -c 'import json, bench; print(json.dumps(bench.build_provenance()))')"; cat $O/issue_report.body; } > $O/issue_report.txt
head -40 $O/issue_report.txt
if [ -f tools/var/xcd/libncgpu.so ]; then
  NCGPU_LIB=$R/tools/var/xcd/libncgpu.so bash tools/pmc_traffic.sh $O/pmc_xcd xcd_probe_traffic.json > $O/pmc_xcd.log 2>&1 || { echo "xcd pmc failed"; tail -5 $O/pmc_xcd.log; exit 1; }
  echo "xcd pmc done"
fi
