# round 5: C4 / C5 at full size on one GPU -- the table from the distinct estimate vs from -s, the
# deferred level 3 decisions on stderr (KC_DEBUG)
set -o pipefail
mkdir -p gpurun_out
export KC_DEBUG=1
timeout -k 10 300 python -u bench.py --config C4 --no-cpu-baseline --no-compact > gpurun_out/r05_t5_c4e.json 2> gpurun_out/r05_t5_c4e.err && \
timeout -k 10 300 python -u bench.py --config C4 --no-cpu-baseline --no-compact --s-table --steps 2 > gpurun_out/r05_t5_c4s.json 2> gpurun_out/r05_t5_c4s.err && \
timeout -k 10 300 python -u bench.py --config C5 --no-cpu-baseline --no-compact --steps 3 > gpurun_out/r05_t5_c5e.json 2> gpurun_out/r05_t5_c5e.err && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_sharded_fullsize.py > gpurun_out/r05_t5_shfull.log 2>&1
