# fused pass: phase 1 alone vs both phases (kernel trace), C3
set -o pipefail
mkdir -p gpurun_out
KC_FUSE_PHASES=1 bash tools/gpu_prof.sh r04_ph1 --config C3 --no-compact --no-verify --steps 3 || exit 1
python3 tools/kstats.py gpurun_out/prof_r04_ph1/run_kernel_stats.csv > gpurun_out/r04_ph1_kstats.txt
KC_FUSE_PHASES=1 KC_FUSE_R=65536 bash tools/gpu_prof.sh r04_ph1b --config C3 --no-compact --no-verify --steps 3 || exit 1
python3 tools/kstats.py gpurun_out/prof_r04_ph1b/run_kernel_stats.csv > gpurun_out/r04_ph1b_kstats.txt
KC_FUSE_R=65536 bash tools/gpu_prof.sh r04_ph2b --config C3 --no-compact --no-verify --steps 3 || exit 1
python3 tools/kstats.py gpurun_out/prof_r04_ph2b/run_kernel_stats.csv > gpurun_out/r04_ph2b_kstats.txt
