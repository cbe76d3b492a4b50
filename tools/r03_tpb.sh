# A/B of the tokenizer's tiles per workgroup (KC_TOK_TPB) on one box: parity subset at the
# default, then the default bench line (C2 + c3) and a kernel trace per setting
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "partitioned or cli or fastq or gzip or bench_job or fullsize" > gpurun_out/gpu_tests_tpb.log 2>&1 || exit 1
for v in 1 2 4 1 2 4; do
  KC_TOK_TPB=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-compact --no-verify > gpurun_out/bench_tpb$v.json 2>> gpurun_out/bench_tpb.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_tpb$v.json').read().strip().splitlines()[-1]); print('TPB', $v, round(d['ms_per_step'],3), round(d['c3']['ms_per_step'],3))" >> gpurun_out/tpb_ab.txt
done
for v in 1 2 4; do
  KC_TOK_TPB=$v bash tools/gpu_prof.sh tpb$v --secondary none --no-compact --no-verify || exit 1
  python3 tools/kstats.py gpurun_out/prof_tpb$v/run_kernel_stats.csv | grep -E "k_emit|k_tile_summary" >> gpurun_out/tpb_ab.txt
done
# coarse-bin bits of the counting pass (C2: 8 by the geometry rule)
for f in 7 8 9 7 8 9; do
  KC_F1BITS=$f timeout -k 10 200 python bench.py --no-cpu-baseline --no-compact --no-verify --secondary none > gpurun_out/bench_f1_$f.json 2>> gpurun_out/bench_tpb.err || exit 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_f1_$f.json').read().strip().splitlines()[-1]); print('F1BITS', $f, round(d['ms_per_step'],3), d['roofline']['kernel_ms'])" >> gpurun_out/tpb_ab.txt
done
