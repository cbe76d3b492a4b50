# tokenizer summary tiles per workgroup (KC_TSUM_TPB 1 / 2 / 4) on the C2 line, parity subset first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "partitioned or cli or fastq or gzip or device_image" > gpurun_out/r04ab5_tests.log 2>&1 || exit 1
for v in 1 4 2 1 4 2; do
  KC_TSUM_TPB=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-compact --no-verify --no-writer --secondary none \
      --steps 10 > gpurun_out/r04ab5_$v.json 2>> gpurun_out/r04ab5.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04ab5_$v.json').read().strip().splitlines()[-1]); print('TPB $v', round(d['ms_per_step'],3), d['kernel_ms'])" >> gpurun_out/r04ab5.txt
done
bash tools/gpu_prof.sh r04ab5_c2 --no-compact --no-verify --no-writer --secondary none || exit 1
python3 tools/kstats.py gpurun_out/prof_r04ab5_c2/run_kernel_stats.csv > gpurun_out/r04ab5_c2_kstats.txt
