#!/bin/bash
# C4 / C5 one --share of 8 (the per-rank workload of the 8-GPU runs) with full-size parity
# against the reference's fixtures (tests/golden/fullsize.json C4S / C5S).   bash tools/r04_share.sh
set -o pipefail
mkdir -p gpurun_out
for c in C4 C5; do
  timeout -k 10 400 python bench.py --config $c --share 8 --no-cpu-baseline --no-writer > gpurun_out/r04_share_$c.json 2> gpurun_out/r04_share_$c.err || exit 1
done
