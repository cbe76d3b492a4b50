# PMC traffic (fresh source digest) and kernel traces of the C4 / C5 shares
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_pmc_traffic.sh C4s --config C4 --share 8 --no-compact --no-verify || exit 1
bash tools/gpu_pmc_traffic.sh C5s --config C5 --share 8 --no-compact --no-verify || exit 1
bash tools/gpu_prof.sh r04_c4s --config C4 --share 8 --no-compact --no-verify || exit 1
python3 tools/kstats.py gpurun_out/prof_r04_c4s/run_kernel_stats.csv > gpurun_out/r04_c4s_kernel_stats.txt || exit 1
bash tools/gpu_prof.sh r04_c5s --config C5 --share 8 --no-compact --no-verify || exit 1
python3 tools/kstats.py gpurun_out/prof_r04_c5s/run_kernel_stats.csv > gpurun_out/r04_c5s_kernel_stats.txt
