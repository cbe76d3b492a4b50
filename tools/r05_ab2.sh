# round 5 A/B: k_emit with 1 / 2 / 4 tiles per workgroup (lib_ab/libkc_emit{1,2}.so, default 4), parity first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  > gpurun_out/r05_ab2_tests.log 2>&1 || exit $?
OUT=gpurun_out/r05_ab2.txt
: > $OUT
X="--no-cpu-baseline --no-compact --no-cli-fullsize --secondary none --tertiary none --no-writer"
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  KC_LIB=$lib timeout -k 10 300 python bench.py $X "$@" > gpurun_out/r05_ab2_$name.json 2>> gpurun_out/r05_ab2.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_ab2_$name.json').read().strip().splitlines()[-1]); print('$name', '$*', round(d['ms_per_step'],3), d['kernel_ms'], (d.get('parity') or {}).get('match'))" >> $OUT
}
D4=$PWD/canonical-k-mer-hash-table_amd/lib/libkc.so
D1=$PWD/lib_ab/libkc_emit1.so
D2=$PWD/lib_ab/libkc_emit2.so
for r in 1 2; do
  run e1_c2 $D1
  run e2_c2 $D2
  run e4_c2 $D4
  run e1_c3 $D1 --config C3
  run e4_c3 $D4 --config C3
done
bash tools/gpu_prof.sh r05_ab2_e4 --no-cli-fullsize --secondary none --tertiary none --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab2_e4/run_kernel_stats.csv > gpurun_out/r05_ab2_e4_kstats.txt
KC_LIB=$D1 bash tools/gpu_prof.sh r05_ab2_e1 --no-cli-fullsize --secondary none --tertiary none --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab2_e1/run_kernel_stats.csv > gpurun_out/r05_ab2_e1_kstats.txt
