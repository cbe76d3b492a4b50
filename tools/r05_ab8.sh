# round 5 A/B (8): k_emit with its phases merged over 2 tiles per workgroup (one set of barriers)
# against 4 tiles and against the sequential 2-tile k_emit (lib_ab/libkc_tpb2s.so), all with the
# 1024-thread k_hll (the distinct estimate of the strong presets), against lib_ab/libkc_head.so:
# parity tests, then C2 x2 per variant and the whole C4 job (its local_table.ms is the estimate)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  > gpurun_out/r05_ab8_tests.log 2>&1 || exit 1
OUT=gpurun_out/r05_ab8.txt
: > $OUT
X="--no-cpu-baseline --no-compact --no-cli-fullsize --secondary none --tertiary none --no-writer"
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  KC_LIB=$lib timeout -k 10 300 python bench.py $X "$@" > gpurun_out/r05_ab8_$name.json 2>> gpurun_out/r05_ab8.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_ab8_$name.json').read().strip().splitlines()[-1]); print('$name', '$*', round(d['ms_per_step'],3), d['kernel_ms'], (d.get('local_table') or {}).get('ms'), (d.get('parity') or {}).get('match'))" >> $OUT
}
NEW=$PWD/canonical-k-mer-hash-table_amd/lib/libkc.so
BASE=$PWD/lib_ab/libkc_head.so
T4=$PWD/lib_ab/libkc_tpb4.so
T2S=$PWD/lib_ab/libkc_tpb2s.so
for r in 1 2; do
  run base_c2 $BASE
  run new_c2 $NEW
  run tpb4_c2 $T4
  run tpb2s_c2 $T2S
done
run new_c3 $NEW --config C3
run tpb2s_c3 $T2S --config C3
run new_c4 $NEW --config C4
run base_c4 $BASE --config C4
run new_c5 $NEW --config C5
bash tools/gpu_prof.sh r05_ab8_c2 --no-cli-fullsize --secondary none --tertiary none --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab8_c2/run_kernel_stats.csv > gpurun_out/r05_ab8_c2_kstats.txt
KC_LIB=$T4 bash tools/gpu_prof.sh r05_ab8_c2t --no-cli-fullsize --secondary none --tertiary none --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab8_c2t/run_kernel_stats.csv > gpurun_out/r05_ab8_c2t_kstats.txt
