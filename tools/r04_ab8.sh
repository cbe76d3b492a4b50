# C2 A/B: one-word keys' windows per thread (KC_RUNW1 = 12: every partitioned level; KC_P1_RUNW1
# = 12 / 8: the segmented level 1 only; k_p1<1,0> spills 64 / 12 / 0 B per lane at 16 / 12 / 8),
# lib_ab builds of every translation unit
set -o pipefail
mkdir -p gpurun_out
run() {  # name, verify flag, env...
  local name=$1 ver=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-compact --no-writer --secondary none $ver --steps 10 \
      > gpurun_out/r04ab8_$name.json 2>> gpurun_out/r04ab8.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04ab8_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],3), d['kernel_ms'], (d.get('parity') or {}).get('match'))" >> gpurun_out/r04ab8.txt
}
run def_v "" KC_NONE=1
run runw12_v "" KC_LIB=$PWD/lib_ab/libkc_runw12.so
run p1w12_v "" KC_LIB=$PWD/lib_ab/libkc_p1w12.so
run p1w8_v "" KC_LIB=$PWD/lib_ab/libkc_p1w8.so
for r in 1 2; do
  run def --no-verify KC_NONE=1
  run runw12 --no-verify KC_LIB=$PWD/lib_ab/libkc_runw12.so
  run p1w12 --no-verify KC_LIB=$PWD/lib_ab/libkc_p1w12.so
  run p1w8 --no-verify KC_LIB=$PWD/lib_ab/libkc_p1w8.so
done
KC_LIB=$PWD/lib_ab/libkc_runw12.so bash tools/gpu_prof.sh r04ab8_w12 --secondary none --no-compact --no-verify || exit 1
python3 tools/kstats.py gpurun_out/prof_r04ab8_w12/run_kernel_stats.csv > gpurun_out/r04ab8_w12_kstats.txt
KC_LIB=$PWD/lib_ab/libkc_p1w8.so bash tools/gpu_prof.sh r04ab8_p1w8 --secondary none --no-compact --no-verify || exit 1
python3 tools/kstats.py gpurun_out/prof_r04ab8_p1w8/run_kernel_stats.csv > gpurun_out/r04ab8_p1w8_kstats.txt
