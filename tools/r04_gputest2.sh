# the rest of the GPU suite after test_gpu_sharded.py::test_route_hint_keeps_owner_counts
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_sharded_mp.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider -k "route_hint or not test_gpu_sharded.py" \
    > gpurun_out/r04_gputest2.log 2>&1
