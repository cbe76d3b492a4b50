set -o pipefail
mkdir -p gpurun_out
bash tools/probe/run.sh p_old p_new || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --secondary none > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bench_c2.json'));print(d['value']/1e9, d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
