# one GPU iteration: bash tools/gpu_iter.sh "<pytest -k expr or ALL>" [bench configs...]
# pytest (GPU tests) -> bench.py per config -> kernel-trace profile of the first config
set -o pipefail
K=$1; shift
mkdir -p gpurun_out
if [ "$K" = "ALL" ]; then KARG=(); else KARG=(-k "$K"); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "${KARG[@]}" > gpurun_out/gpu_tests.log 2>&1 || exit 1
for c in "$@"; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit 1
done
if [ $# -gt 0 ]; then bash tools/gpu_prof.sh $1 --config $1; fi
