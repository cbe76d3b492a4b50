#!/bin/bash
# HBM traffic of one bench workload: the two PMC passes roofline.traffic needs (FETCH_SIZE;
# WRITE_SIZE, one counter group per rocprofv3 run, no tracing domains), summarised into
# profiles/pmc_traffic.json (one entry per workload; bench.py looks its own up) and a copy
# under gpurun_out/.  usage: tools/gpu_pmc_traffic.sh NAME [bench args...]
set -o pipefail
NAME=$1; shift
OUT=$(realpath -m "gpurun_out/pmc_$NAME")
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$OUT"
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- \
      python3 "$ROOT/bench.py" --no-cpu-baseline --no-writer --steps 3 --warmup 1 "$@" > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err") || exit $?
done
python3 "$ROOT/profiles/pmc_summary.py" "$OUT" --write "$ROOT/profiles/pmc_traffic.json" > "$OUT/summary.txt" && \
cp "$ROOT/profiles/pmc_traffic.json" "$ROOT/gpurun_out/pmc_traffic.json"
