#!/bin/bash
# PMC passes (one counter group per run, per the MI355X guide) over a short bench run.
# Usage: scripts/prof_pmc.sh OUTDIR [bench args...]
set -e
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAVES" "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/$OUT/pmc$i -o run -- python3 $R/bench.py "$@" > $R/$OUT/pmc$i.log 2>&1 || { echo "pmc group $i failed"; tail -5 $R/$OUT/pmc$i.log; exit 1; }
done
echo done
