# round 5: scatter kernels' launch bounds from their LDS occupancy (wide keys: no scratch) --
# golden parity of every width, deferral tests, C5 whole / share, C2 unchanged
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_defer.py \
  > gpurun_out/r05_t9_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config C5 --no-cpu-baseline --no-compact --steps 3 > gpurun_out/r05_t9_c5.json 2> gpurun_out/r05_t9_c5.err || exit $?
timeout -k 10 300 python -u bench.py --config C5 --share 8 --no-cpu-baseline --no-compact --no-writer > gpurun_out/r05_t9_c5s.json 2> gpurun_out/r05_t9_c5s.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-compact --no-cli-fullsize --secondary none --tertiary none > gpurun_out/r05_t9_c2.json 2> gpurun_out/r05_t9_c2.err || exit $?
bash tools/gpu_prof.sh r05_t9_c5 --config C5 --no-compact --steps 2 || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_t9_c5/run_kernel_stats.csv > gpurun_out/r05_t9_c5_kernel_stats.txt
