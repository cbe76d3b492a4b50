#!/bin/bash
# PMC collection for the bench kernels (one counter group per pass, kernel trace off).
# usage: tools_prof.sh OUTDIR [bench args...]
OUT=$1; shift
cd /tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py "$@" > $OUT/pmc$i.log 2>&1 || exit $?
done
