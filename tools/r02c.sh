set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/gpu_tests.log
bash tools/gpu_prof.sh C3 --config C3 --secondary none || exit 1
python3 tools/kstats.py gpurun_out/prof_C3/run_kernel_stats.csv | head -24
cat gpurun_out/prof_C3.json | python3 -c "import json,sys;d=json.load(sys.stdin);print(d['value']/1e9, d['ms_per_step'], d['kernel_ms'])"
