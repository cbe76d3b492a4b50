# round-4 changes on the GPU: tests of the new paths, then C3 / C2 A/B lines and kernel traces
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_bloom.py tests/test_gpu_sharded.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/r04ab6_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_sharded_mp.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04ab6_tests_mp.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "bloom or reuse or Bloom or planner or cli" > gpurun_out/r04ab6_tests2.log 2>&1 || exit 1
for v in off f32k ref; do
  case $v in off) E="";; f32k) E="KC_FGEO_R=32768";; ref) E="KC_BF_TABLE=reference";; esac
  env $E timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline --no-compact --no-writer --steps 10 \
      > gpurun_out/r04ab6_c3_$v.json 2>> gpurun_out/r04ab6.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04ab6_c3_$v.json').read().strip().splitlines()[-1]); print('C3 $v', round(d['ms_per_step'],3), d['roofline']['kernel_ms'], d['table_slots'], d.get('parity',{}).get('match'))" >> gpurun_out/r04ab6.txt
done
for v in 1 4 2; do
  KC_TSUM_TPB=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-compact --no-verify --no-writer --secondary none \
      --steps 10 > gpurun_out/r04ab6_c2_$v.json 2>> gpurun_out/r04ab6.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04ab6_c2_$v.json').read().strip().splitlines()[-1]); print('C2 TPB $v', round(d['ms_per_step'],3), d['kernel_ms'])" >> gpurun_out/r04ab6.txt
done
bash tools/gpu_prof.sh r04ab6 --no-compact --no-verify --no-writer || exit 1
python3 tools/kstats.py gpurun_out/prof_r04ab6/run_kernel_stats.csv > gpurun_out/r04ab6_kstats.txt
