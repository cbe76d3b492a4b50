# round 5: the whole GPU suite after the deferral + hygiene changes, then C4 / C5 at full size
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  > gpurun_out/r05_t3_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config C4 --no-cpu-baseline > gpurun_out/r05_t3_c4.json 2> gpurun_out/r05_t3_c4.err && \
KC_DEBUG=1 timeout -k 10 300 python -u bench.py --config C5 --no-cpu-baseline --steps 3 > gpurun_out/r05_t3_c5.json 2> gpurun_out/r05_t3_c5.err
