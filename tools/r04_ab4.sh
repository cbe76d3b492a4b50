# owner-sharded Bloom + k_b3 prefetch + Bloom table from new_in_second: tests, then C3 variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_bloom.py tests/test_gpu_sharded.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/r04ab4_tests.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded_mp.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04ab4_tests_mp.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "bloom or reuse or Bloom" > gpurun_out/r04ab4_tests2.log 2>&1 || exit 1
for v in off fused f32k ref; do
  case $v in off) E="";; fused) E="KC_FUSE=1";; f32k) E="KC_FGEO_R=32768";; ref) E="KC_BF_TABLE=reference";; esac
  env $E timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline --no-compact --no-writer --steps 10 \
      > gpurun_out/r04ab4_$v.json 2>> gpurun_out/r04ab4.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04ab4_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],3), d['roofline']['kernel_ms'], d['table_slots'], d.get('parity',{}).get('match'))" >> gpurun_out/r04ab4.txt
done
bash tools/gpu_prof.sh r04ab4_off --config C3 --no-compact --no-verify --no-writer || exit 1
python3 tools/kstats.py gpurun_out/prof_r04ab4_off/run_kernel_stats.csv > gpurun_out/r04ab4_off_kstats.txt
KC_FGEO_R=32768 bash tools/gpu_prof.sh r04ab4_f32k --config C3 --no-compact --no-verify --no-writer || exit 1
python3 tools/kstats.py gpurun_out/prof_r04ab4_f32k/run_kernel_stats.csv > gpurun_out/r04ab4_f32k_kstats.txt
