#!/bin/bash
# round 5, second session: kernel traces of the C2, C3 and C4 bench lines at HEAD (no PMC passes).
#   bash tools/r05_s2_traces.sh NAME
set -o pipefail
N=${1:-r05_s2_traces}
mkdir -p gpurun_out
bash tools/gpu_prof.sh ${N} --no-cli-fullsize --secondary none --tertiary none || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}/run_kernel_stats.csv > gpurun_out/${N}_kernel_stats.txt || exit 1
bash tools/gpu_prof.sh ${N}_c3 --config C3 --no-cli-fullsize || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}_c3/run_kernel_stats.csv > gpurun_out/${N}_c3_kernel_stats.txt || exit 1
bash tools/gpu_prof.sh ${N}_c4 --config C4 --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}_c4/run_kernel_stats.csv > gpurun_out/${N}_c4_kernel_stats.txt
