# round 5: the 1024-thread two-word level 1 for big tables (whole C4 on one GPU): deferral tests
# (incl. a 1.4 G-slot table), the C4 bench line with parity, its kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_defer.py \
  > gpurun_out/r05_t8_defer.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config C4 --no-cpu-baseline --no-compact > gpurun_out/r05_t8_c4.json 2> gpurun_out/r05_t8_c4.err || exit $?
bash tools/gpu_prof.sh r05_t8_c4 --config C4 --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_t8_c4/run_kernel_stats.csv > gpurun_out/r05_t8_c4_kernel_stats.txt
