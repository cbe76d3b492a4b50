# round 5, first GPU pass: the output digest on every golden case (partitioned path), the
# two-process sharded digest, the launcher on a one-GPU box, full-size digests, default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "host_chunks and partitioned" > gpurun_out/r05_t1_parity.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_sharded_mp.py tests/test_bench_launch.py "tests/test_gpu_fullsize.py::test_bench_job_equals_reference_output" \
  > gpurun_out/r05_t1_rest.log 2>&1 && \
timeout -k 10 900 python -u bench.py > gpurun_out/r05_b1.json 2> gpurun_out/r05_b1.err
