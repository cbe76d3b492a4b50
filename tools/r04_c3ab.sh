# C3 A/B of the fused pass: fused (default sizing / 2^16 regions) vs KC_FUSE=0, kernel trace
set -o pipefail
mkdir -p gpurun_out
for v in def r64k off def r64k off; do
  case $v in def) E="";; r64k) E="KC_FUSE_R=65536";; off) E="KC_FUSE=0";; esac
  env $E timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline --no-compact --no-verify --steps 10 \
      > gpurun_out/r04ab_$v.json 2>> gpurun_out/r04ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04ab_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],3), d['roofline']['kernel_ms'], d['table_slots'])" >> gpurun_out/r04ab.txt
done
bash tools/gpu_prof.sh r04_c3b --config C3 --no-compact --no-verify || exit 1
python3 tools/kstats.py gpurun_out/prof_r04_c3b/run_kernel_stats.csv > gpurun_out/r04_c3b_kstats.txt
