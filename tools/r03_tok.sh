# round-3 tokenizer iteration: GPU parity subset -> bench -> kernel trace -> LDS stall PMC
#   bash tools/r03_tok.sh NAME
set -o pipefail
N=${1:-tok}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "partitioned or cli or fastq or gzip or bench_job or fullsize" > gpurun_out/gpu_tests_$N.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$N.json 2> gpurun_out/bench_$N.err || exit 1
bash tools/gpu_prof.sh $N || exit 1
python3 tools/kstats.py gpurun_out/prof_$N/run_kernel_stats.csv > gpurun_out/prof_${N}_stats.txt || exit 1
bash tools/gpu_pmc_lds.sh $N || exit 1
python3 tools/pmc_lds_summary.py gpurun_out/pmc_lds_$N > gpurun_out/pmc_lds_$N.txt
