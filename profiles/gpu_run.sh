set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && \
timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof.err && \
cd $GRAFT_REPO_ROOT && bash profiles/collect_pmc.sh gpurun_out/pmc --steps 3 --warmup 1
