# round-3 closing measurement at HEAD: PMC traffic of C2 and C3 (roofline.traffic), the
# default bench line, its kernel trace, smoke().   KC_COMMIT=<sha> bash tools/r03_final2.sh NAME
set -o pipefail
N=${1:-r03_final2}
mkdir -p gpurun_out
bash tools/gpu_pmc_traffic.sh C2 --secondary none --no-compact --no-verify || exit 1
bash tools/gpu_pmc_traffic.sh C3 --config C3 --no-compact --no-verify || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${N}_bench.json 2> gpurun_out/${N}_bench.err || exit 1
bash tools/gpu_prof.sh ${N} || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}/run_kernel_stats.csv > gpurun_out/${N}_kernel_stats.txt || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${N}_smoke.txt 2>&1
