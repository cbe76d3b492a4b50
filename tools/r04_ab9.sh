# C2 A/B: k_p3's 6-byte records read as 12-byte pairs (KC_P3_PAIRS pairs per thread and round, the
# next round prefetched) against the per-record loads (default); lib_ab builds of the count kernels
set -o pipefail
mkdir -p gpurun_out
run() {  # name, verify flag, env...
  local name=$1 ver=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-compact --no-writer --secondary none $ver --steps 10 \
      > gpurun_out/r04ab9_$name.json 2>> gpurun_out/r04ab9.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04ab9_$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],3), d['kernel_ms'], (d.get('parity') or {}).get('match'))" >> gpurun_out/r04ab9.txt
}
run def_v "" KC_NONE=1
run p3p4_v "" KC_LIB=$PWD/lib_ab/libkc_p3p4.so
run p3p3_v "" KC_LIB=$PWD/lib_ab/libkc_p3p3.so
run p3p2_v "" KC_LIB=$PWD/lib_ab/libkc_p3p2.so
for r in 1 2; do
  run def --no-verify KC_NONE=1
  run p3p4 --no-verify KC_LIB=$PWD/lib_ab/libkc_p3p4.so
  run p3p3 --no-verify KC_LIB=$PWD/lib_ab/libkc_p3p3.so
  run p3p2 --no-verify KC_LIB=$PWD/lib_ab/libkc_p3p2.so
done
for v in def p3p4 p3p2; do
  L=""; [ $v != def ] && L=$PWD/lib_ab/libkc_$v.so
  KC_LIB=$L bash tools/gpu_prof.sh r04ab9_$v --secondary none --no-compact --no-verify || exit 1
  python3 tools/kstats.py gpurun_out/prof_r04ab9_$v/run_kernel_stats.csv > gpurun_out/r04ab9_${v}_kstats.txt || exit 1
done
