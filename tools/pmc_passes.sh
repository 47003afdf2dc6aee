#!/bin/bash
# rocprofv3 counter passes (one --pmc set per run, each under its own time limit) over the
# kernel-isolation driver tools/prof_kernels.py.   usage: tools/pmc_passes.sh OUTDIR target [target ...]
set -o pipefail
OUT=$1; shift
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
P3="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for t in "$@"; do
  cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$OUT/$t/stats -o run --output-format csv -- python3 $R/tools/prof_kernels.py $t > $R/$OUT/$t.stats.log 2>&1 || { echo "stats $t failed"; tail -5 $R/$OUT/$t.stats.log; exit 1; }
  i=1
  for P in "$P1" "$P2" "$P3"; do
    cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $R/$OUT/$t/p$i -o run -- python3 $R/tools/prof_kernels.py $t > $R/$OUT/$t.p$i.log 2>&1 || { echo "pmc pass $i $t failed"; tail -5 $R/$OUT/$t.p$i.log; exit 1; }
    i=$((i+1))
  done
done
echo passes done
