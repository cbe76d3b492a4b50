#!/bin/bash
# PMC passes for the bench kernels (one counter group per rocprofv3 run, no tracing
# domains combined with --pmc).  usage: profiles/collect_pmc.sh OUTDIR [bench args...]
# Then: python profiles/pmc_summary.py OUTDIR  -> per-kernel table + pmc_traffic.json
set -o pipefail
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err" || exit $?
done
