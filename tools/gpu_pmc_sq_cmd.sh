# SQ counters (two PMC passes) for an arbitrary python script: bash tools/gpu_pmc_sq_cmd.sh NAME script.py [args]
set -o pipefail
NAME=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- \
      python3 -u "$GRAFT_REPO_ROOT/$@" > "$OUT/pmc$i.out" 2> "$OUT/pmc$i.err" || exit $?
done
