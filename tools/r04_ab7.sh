# C3 A/B: k_b3 at 1024 threads (lib_ab build), level-1 coarse bins 2^7 of the kept fine geometry
set -o pipefail
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline --no-compact --no-writer --no-verify --steps 10 \
      > gpurun_out/r04ab7_$name.json 2>> gpurun_out/r04ab7.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04ab7_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],3), d['roofline']['kernel_ms'], d['table_slots'])" >> gpurun_out/r04ab7.txt
}
for r in 1 2; do
  run def KC_NONE=1
  run b3nt1024 KC_LIB=$PWD/lib_ab/libkc_b3nt1024.so
  run f1_7 KC_FGEO_F1=7
done
KC_LIB=$PWD/lib_ab/libkc_b3nt1024.so bash tools/gpu_prof.sh r04ab7_b3 --config C3 --no-compact --no-verify --no-writer || exit 1
python3 tools/kstats.py gpurun_out/prof_r04ab7_b3/run_kernel_stats.csv > gpurun_out/r04ab7_b3_kstats.txt
KC_FGEO_F1=7 bash tools/gpu_prof.sh r04ab7_f17 --config C3 --no-compact --no-verify --no-writer || exit 1
python3 tools/kstats.py gpurun_out/prof_r04ab7_f17/run_kernel_stats.csv > gpurun_out/r04ab7_f17_kstats.txt
