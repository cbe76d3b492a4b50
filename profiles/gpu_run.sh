# One GPU call that produces a round's evidence (bash profiles/gpu_run.sh):
# GPU tests, bench lines (C2 default with the CPU baseline, C3, per-GPU shares of C4 and
# C5), kernel-trace profiles of C2 and C3, and the PMC traffic passes of C2.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && \
timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && \
timeout -k 10 200 python bench.py --config C4 --reads 12500000 --slots 1250000000 --no-cpu-baseline > gpurun_out/bench_c4s.json 2> gpurun_out/bench_c4s.err && \
timeout -k 10 200 python bench.py --config C5 --reads 125000 --slots 1250000000 --no-cpu-baseline > gpurun_out/bench_c5s.json 2> gpurun_out/bench_c5s.err && \
bash tools/gpu_prof2.sh C2 "--config C2" C3 "--config C3" && \
bash profiles/collect_pmc.sh gpurun_out/pmc --steps 3 --warmup 1
