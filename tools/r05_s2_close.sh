#!/bin/bash
# round 5, second session, closing part 1: PMC traffic of C2 / C3 / C4 (roofline.traffic) at the
# working tree's sources, kernel traces of the C2, C3, C4 and C5 bench lines, smoke().
#   bash tools/r05_s2_close.sh NAME
set -o pipefail
N=${1:-r05_s2_close}
mkdir -p gpurun_out
X="--no-compact --no-verify --no-cli-fullsize --secondary none --tertiary none"
bash tools/gpu_pmc_traffic.sh C2 $X || exit 1
bash tools/gpu_pmc_traffic.sh C3 --config C3 $X || exit 1
bash tools/gpu_pmc_traffic.sh C4 --config C4 $X || exit 1
bash tools/gpu_prof.sh ${N} --no-cli-fullsize --secondary none --tertiary none || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}/run_kernel_stats.csv > gpurun_out/${N}_kernel_stats.txt || exit 1
bash tools/gpu_prof.sh ${N}_c3 --config C3 --no-cli-fullsize || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}_c3/run_kernel_stats.csv > gpurun_out/${N}_c3_kernel_stats.txt || exit 1
bash tools/gpu_prof.sh ${N}_c4 --config C4 --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}_c4/run_kernel_stats.csv > gpurun_out/${N}_c4_kernel_stats.txt || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${N}_smoke.txt 2>&1 || exit 1
bash tools/gpu_prof.sh ${N}_c5 --config C5 --no-compact --steps 2 || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}_c5/run_kernel_stats.csv > gpurun_out/${N}_c5_kernel_stats.txt
