# round 5: deferred level 3 with record-sized slots and the deferral-aware path choice (C5 on one
# GPU), then the default bench line, the sharded Bloom job at one rank and the PMC calibration
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_defer.py \
  > gpurun_out/r05_t7_defer.log 2>&1 || exit $?
export KC_DEBUG=1
timeout -k 10 300 python -u bench.py --config C4 --no-cpu-baseline --no-compact > gpurun_out/r05_t7_c4.json 2> gpurun_out/r05_t7_c4.err && \
timeout -k 10 300 python -u bench.py --config C5 --no-cpu-baseline --no-compact --steps 3 > gpurun_out/r05_t7_c5.json 2> gpurun_out/r05_t7_c5.err || exit $?
unset KC_DEBUG
bash tools/r05_t4.sh
