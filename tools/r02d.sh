set -o pipefail
mkdir -p gpurun_out
KC_REUSE_DEBUG=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bloom_at_scale or level1_reuse" -s > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?"; grep -E "reuse|passed|failed|Error|assert" gpurun_out/gpu_tests.log | head -40
