# round 5 A/B (7): the tokenizer's tile loads in two phases (every tile's dword loads issued before the
# first funnel shift) and as global (not flat) loads; k_emit with 1 and 2 tiles per workgroup.
# Parity tests first, then C2 x3 and C3 against lib_ab/libkc_head.so (the committed sources)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_bloom.py > gpurun_out/r05_ab7_tests.log 2>&1 || exit 1
OUT=gpurun_out/r05_ab7.txt
: > $OUT
X="--no-cpu-baseline --no-compact --no-cli-fullsize --secondary none --tertiary none --no-writer"
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  KC_LIB=$lib timeout -k 10 300 python bench.py $X "$@" > gpurun_out/r05_ab7_$name.json 2>> gpurun_out/r05_ab7.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_ab7_$name.json').read().strip().splitlines()[-1]); print('$name', '$*', round(d['ms_per_step'],3), d['kernel_ms'], (d.get('parity') or {}).get('match'))" >> $OUT
}
NEW=$PWD/canonical-k-mer-hash-table_amd/lib/libkc.so
BASE=$PWD/lib_ab/libkc_head.so
T2=$PWD/lib_ab/libkc_tpb2.so
for r in 1 2 3; do
  run base_c2 $BASE
  run new_c2 $NEW
  run tpb2_c2 $T2
done
for r in 1 2; do
  run base_c3 $BASE --config C3
  run new_c3 $NEW --config C3
  run tpb2_c3 $T2 --config C3
done
bash tools/gpu_prof.sh r05_ab7_c2 --no-cli-fullsize --secondary none --tertiary none --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab7_c2/run_kernel_stats.csv > gpurun_out/r05_ab7_c2_kstats.txt
KC_LIB=$BASE bash tools/gpu_prof.sh r05_ab7_c2b --no-cli-fullsize --secondary none --tertiary none --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab7_c2b/run_kernel_stats.csv > gpurun_out/r05_ab7_c2b_kstats.txt
KC_LIB=$T2 bash tools/gpu_prof.sh r05_ab7_c2t --no-cli-fullsize --secondary none --tertiary none --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab7_c2t/run_kernel_stats.csv > gpurun_out/r05_ab7_c2t_kstats.txt
