# Round 4, first GPU call: the fused Bloom + counting pass -- its tests, the C3 full-size
# parity (two steps on one context), then C3 bench lines fused / unfused and a kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/r04_fused_tests.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 600 --timeout-method thread \
    -k "C3" > gpurun_out/r04_fullsize_c3.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline --no-compact --steps 10 > gpurun_out/r04_c3_fused.json \
    2> gpurun_out/r04_c3_fused.err || exit 1
KC_FUSE=0 timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline --no-compact --no-verify --steps 10 \
    > gpurun_out/r04_c3_unfused.json 2> gpurun_out/r04_c3_unfused.err || exit 1
KC_FUSE_GATE=global timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline --no-compact --no-verify --steps 10 \
    > gpurun_out/r04_c3_fused_gglobal.json 2> gpurun_out/r04_c3_fused_gglobal.err || exit 1
KC_FUSE_R=65536 timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline --no-compact --no-verify --steps 10 \
    > gpurun_out/r04_c3_fused_r64k.json 2> gpurun_out/r04_c3_fused_r64k.err || exit 1
bash tools/gpu_prof.sh r04_c3 --config C3 --no-compact --no-verify || exit 1
python3 tools/kstats.py gpurun_out/prof_r04_c3/run_kernel_stats.csv > gpurun_out/r04_c3_kstats.txt
