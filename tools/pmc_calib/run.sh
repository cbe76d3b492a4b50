#!/bin/bash
# PMC byte calibration: one rocprofv3 pass per counter (FETCH_SIZE, WRITE_SIZE)
# over tools/pmc_calib/pmc_calib, then the counter / known-bytes ratio per access shape.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$(realpath -m "gpurun_out/pmc_calib")
mkdir -p "$OUT"
"$ROOT/tools/pmc_calib/pmc_calib" > "$OUT/known.txt" || exit $?
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/pmc$i" -o run --output-format csv -- \
      "$ROOT/tools/pmc_calib/pmc_calib" > "$OUT/pmc$i.txt" 2> "$OUT/pmc$i.err") || exit $?
done
python3 "$ROOT/tools/pmc_calib/summary.py" "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
