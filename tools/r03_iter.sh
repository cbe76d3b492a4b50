# one GPU iteration (round 3): bash tools/r03_iter.sh "<pytest -k expr>" NAME
# GPU parity subset (partitioned paths + full-size reference parity) -> kernel-trace profile of bench.py
set -o pipefail
mkdir -p gpurun_out
K=${1:-partitioned or skew or overflow or bloom or reused or bench_job}
N=${2:-r03}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bloom.py tests/test_gpu_fullsize.py -x -q \
    --timeout 400 --timeout-method thread -m gpu -k "$K" > gpurun_out/t_$N.log 2>&1
rc=$?; tail -3 gpurun_out/t_$N.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh $N || exit 1
python3 tools/kstats.py gpurun_out/prof_$N/run_kernel_stats.csv | grep -E "k_p1|k_p2f|k_p3|k_b3|k_emit|k_tile_summary"
head -c 700 gpurun_out/prof_$N.json
