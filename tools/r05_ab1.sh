# round 5 A/B: the 1024-thread two-word level 1 everywhere (lib_ab/libkc_p1wide.so, -DKC_AB_P1WIDE=1)
# against the default (big tables only) on C3 (the kept Bloom levels) and the C4 share
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/r05_ab1.txt
: > $OUT
X="--no-cpu-baseline --no-compact --no-cli-fullsize --secondary none --tertiary none --no-writer"
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  KC_LIB=$lib timeout -k 10 300 python bench.py $X "$@" > gpurun_out/r05_ab1_$name.json 2>> gpurun_out/r05_ab1.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_ab1_$name.json').read().strip().splitlines()[-1]); print('$name', '$*', round(d['ms_per_step'],3), d['kernel_ms'], (d.get('parity') or {}).get('match'))" >> $OUT
}
DEF=$PWD/canonical-k-mer-hash-table_amd/lib/libkc.so
WIDE=$PWD/lib_ab/libkc_p1wide.so
for r in 1 2; do
  run def_c3 $DEF --config C3
  run wide_c3 $WIDE --config C3
  run def_c4s $DEF --config C4 --share 8
  run wide_c4s $WIDE --config C4 --share 8
done
KC_LIB=$WIDE bash tools/gpu_prof.sh r05_ab1_wide_c3 --config C3 --no-cli-fullsize --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab1_wide_c3/run_kernel_stats.csv > gpurun_out/r05_ab1_wide_c3_kstats.txt
KC_LIB=$WIDE bash tools/gpu_prof.sh r05_ab1_wide_c4s --config C4 --share 8 --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab1_wide_c4s/run_kernel_stats.csv > gpurun_out/r05_ab1_wide_c4s_kstats.txt
