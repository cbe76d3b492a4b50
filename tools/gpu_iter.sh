set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bloom or Bloom or -b" > gpurun_out/gpu_bloom.log 2>&1 && \
timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
