# round 5: deferred level 3 -- correctness, then C4 / C5 at full size on one GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_defer.py \
  "tests/test_gpu_parity.py::test_device_image_path_and_small_batches" \
  "tests/test_gpu_parity.py::test_segment_overflow_spills_or_falls_back" > gpurun_out/r05_t2_tests.log 2>&1 && \
timeout -k 10 600 python -u bench.py --config C4 --no-cpu-baseline > gpurun_out/r05_t2_c4.json 2> gpurun_out/r05_t2_c4.err && \
timeout -k 10 600 python -u bench.py --config C5 --no-cpu-baseline --steps 3 > gpurun_out/r05_t2_c5.json 2> gpurun_out/r05_t2_c5.err
