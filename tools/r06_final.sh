#!/bin/bash
# round 6's closing measurements at HEAD's kernel sources.
#   bash tools/r06_final.sh pmc        the PMC traffic entries (FETCH_SIZE / WRITE_SIZE passes,
#                                      profiles/pmc_traffic.json) of the four workloads on the line
#   bash tools/r06_final.sh line NAME  the default line (python bench.py, as the driver runs it),
#                                      kernel traces of C2 / C3 / C4 / C5 and smoke(), under gpurun_out/NAME*
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
if [ "$1" = pmc ]; then
  X="--no-cli-fullsize --no-compact --no-host-chunks --secondary none --tertiary none --quaternary none"
  bash tools/gpu_pmc_traffic.sh r06_C2 $X || exit $?
  bash tools/gpu_pmc_traffic.sh r06_C3 --config C3 $X || exit $?
  bash tools/gpu_pmc_traffic.sh r06_C4 --config C4 $X || exit $?
  bash tools/gpu_pmc_traffic.sh r06_C5 --config C5 $X || exit $?
  exit 0
fi
N=$2
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py > gpurun_out/${N}_bench.json 2> gpurun_out/${N}_bench.err || exit $?
X="--no-cpu-baseline --no-writer --no-compact --no-cli-fullsize --no-host-chunks --secondary none --tertiary none --quaternary none"
for c in C2 C3 C4 C5; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${N}_prof_$c \
    -o run --output-format csv -- python3 $R/bench.py --config $c --steps 3 --warmup 1 $X \
    > $R/gpurun_out/${N}_prof_$c.json 2> $R/gpurun_out/${N}_prof_$c.err) || exit $?
  python3 tools/kstats.py gpurun_out/${N}_prof_$c/run_kernel_stats.csv > gpurun_out/${N}_prof_$c.txt || exit $?
done
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${N}_smoke.txt 2>&1
