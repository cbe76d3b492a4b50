# LDS-atomic / LDS-issue stall counters per kernel for one bench config (one PMC pass of
# 8 SQ counters, no tracing domains):  bash tools/gpu_pmc_lds.sh NAME [bench args...]
# Summarise with: python3 tools/pmc_lds_summary.py gpurun_out/pmc_lds_NAME
set -o pipefail
N=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_lds_$N
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$OUT/p" -o run --output-format csv -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-compact --no-verify --steps 2 --warmup 1 "$@" > "$OUT/p.json" 2> "$OUT/p.err"
