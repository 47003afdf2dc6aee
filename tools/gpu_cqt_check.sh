#!/bin/bash
# CQT change check: chroma parity tests, then kernel stats of the chroma path.
set -o pipefail
O=gpurun_out/${1:-cqt}
R=$GRAFT_REPO_ROOT
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_chroma.py tests/test_gpu_shared_tuning.py tests/test_gpu_components.py tests/test_gpu_pipeline.py tests/test_gpu_config5.py > $O/pytest.log 2>&1 || { echo "tests failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$O/chroma -o run --output-format csv -- python3 $R/tools/prof_kernels.py chroma > $R/$O/chroma.log 2>&1 || { echo "stats failed"; tail -5 $R/$O/chroma.log; exit 1; }
cd $R && python3 tools/pmc_report.py $O/chroma/
