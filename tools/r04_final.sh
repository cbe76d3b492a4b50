#!/bin/bash
# round-4 closing measurement at HEAD (after tools/r04_gputest.sh): PMC traffic of C2 and C3
# (roofline.traffic), the default bench line (cpu_baseline, parity, writer), its kernel trace,
# C3's kernel trace, smoke().    bash tools/r04_final.sh NAME
set -o pipefail
N=${1:-r04_final}
mkdir -p gpurun_out
bash tools/gpu_pmc_traffic.sh C2 --secondary none --no-compact --no-verify || exit 1
bash tools/gpu_pmc_traffic.sh C3 --config C3 --no-compact --no-verify || exit 1
timeout -k 10 500 python bench.py > gpurun_out/${N}_bench.json 2> gpurun_out/${N}_bench.err || exit 1
bash tools/gpu_prof.sh ${N} --secondary none || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}/run_kernel_stats.csv > gpurun_out/${N}_kernel_stats.txt || exit 1
bash tools/gpu_prof.sh ${N}_c3 --config C3 || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}_c3/run_kernel_stats.csv > gpurun_out/${N}_c3_kernel_stats.txt || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${N}_smoke.txt 2>&1
