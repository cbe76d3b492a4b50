# round 5: the sharded-path GPU tests after the merge-timing / owner-sizing changes in Python
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu tests/test_gpu_sharded.py \
  tests/test_gpu_sharded_mp.py tests/test_gpu_sharded_fullsize.py tests/test_bench_launch.py > gpurun_out/r05_t12_tests.log 2>&1
