# round-2 final measurement call: smoke, the default bench line (C2 + c3 + CPU baselines +
# compact), the skewed preset, a kernel trace of the default bench (GPU tests: run separately)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/f_smoke.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/f_bench.json 2> gpurun_out/f_bench.err || exit 1
timeout -k 10 300 python bench.py --config C2S --no-cpu-baseline --no-compact > gpurun_out/f_bench_C2S.json 2>> gpurun_out/f_bench.err || exit 1
bash tools/gpu_prof.sh r02final --no-compact
