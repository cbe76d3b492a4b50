# PMC passes over harness binaries: bash tools/probe/pmc.sh p_old p_new ...
# (SQ instruction mix / waits / LDS conflicts, then FETCH_SIZE and WRITE_SIZE, one group per run)
set -o pipefail
R=$GRAFT_REPO_ROOT
for b in "$@"; do
  OUT=$R/gpurun_out/pmc_$b
  mkdir -p $OUT
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- $R/tools/probe/$b 10000000 2 > "$OUT/pmc$i.log" 2>&1 ) || exit 1
  done
  echo "== $b"; python3 tools/probe/pmc_means.py $OUT
done
