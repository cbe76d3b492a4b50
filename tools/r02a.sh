set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
for c in C3 C2S; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --secondary none > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit 1; done
bash tools/gpu_prof.sh C2 --config C2 --secondary none
