#!/bin/bash
# round 6: the PMC traffic entries (FETCH_SIZE / WRITE_SIZE passes, profiles/pmc_traffic.json) of the
# four workloads on the default line, at HEAD's kernel sources.  usage: bash tools/r06_pmc.sh
set -o pipefail
X="--no-cli-fullsize --no-compact --no-host-chunks --secondary none --tertiary none --quaternary none"
bash tools/gpu_pmc_traffic.sh r06_C2 $X || exit $?
bash tools/gpu_pmc_traffic.sh r06_C3 --config C3 $X || exit $?
bash tools/gpu_pmc_traffic.sh r06_C4 --config C4 $X || exit $?
bash tools/gpu_pmc_traffic.sh r06_C5 --config C5 $X || exit $?
