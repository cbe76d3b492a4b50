# after the parallel segment prefix: C2 default line + C3 fused / r64k / unfused, kernel traces
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu-baseline --no-compact --no-verify --secondary none --steps 10 > gpurun_out/r04ab2_c2.json 2>> gpurun_out/r04ab2.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r04ab2_c2.json').read().strip().splitlines()[-1]); print('C2', round(d['ms_per_step'],3), d['roofline']['kernel_ms'], round(d['value']/1e9,2))" >> gpurun_out/r04ab2.txt
for v in def r64k off; do
  case $v in def) E="";; r64k) E="KC_FUSE_R=65536";; off) E="KC_FUSE=0";; esac
  env $E timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline --no-compact --no-verify --steps 10 \
      > gpurun_out/r04ab2_$v.json 2>> gpurun_out/r04ab2.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04ab2_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],3), d['roofline']['kernel_ms'], d['table_slots'])" >> gpurun_out/r04ab2.txt
done
bash tools/gpu_prof.sh r04ab2_c2 --no-compact --no-verify --secondary none || exit 1
python3 tools/kstats.py gpurun_out/prof_r04ab2_c2/run_kernel_stats.csv > gpurun_out/r04ab2_c2_kstats.txt
KC_FUSE_R=65536 bash tools/gpu_prof.sh r04ab2_c3 --config C3 --no-compact --no-verify || exit 1
python3 tools/kstats.py gpurun_out/prof_r04ab2_c3/run_kernel_stats.csv > gpurun_out/r04ab2_c3_kstats.txt
KC_FUSE=0 bash tools/gpu_prof.sh r04ab2_c3off --config C3 --no-compact --no-verify || exit 1
python3 tools/kstats.py gpurun_out/prof_r04ab2_c3off/run_kernel_stats.csv > gpurun_out/r04ab2_c3off_kstats.txt
