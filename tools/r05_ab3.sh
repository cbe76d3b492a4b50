# round 5 A/B: every key width reads its run's symbols from one funnel-shifted register (lib = new,
# lib_ab/libkc_base.so = before); parity first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_defer.py \
  > gpurun_out/r05_ab3_tests.log 2>&1 || exit $?
OUT=gpurun_out/r05_ab3.txt
: > $OUT
X="--no-cpu-baseline --no-compact --no-cli-fullsize --secondary none --tertiary none --no-writer"
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  KC_LIB=$lib timeout -k 10 300 python bench.py $X "$@" > gpurun_out/r05_ab3_$name.json 2>> gpurun_out/r05_ab3.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_ab3_$name.json').read().strip().splitlines()[-1]); print('$name', '$*', round(d['ms_per_step'],3), d['kernel_ms'], (d.get('parity') or {}).get('match'))" >> $OUT
}
NEW=$PWD/canonical-k-mer-hash-table_amd/lib/libkc.so
BASE=$PWD/lib_ab/libkc_base.so
for r in 1 2; do
  run base_c3 $BASE --config C3
  run new_c3 $NEW --config C3
  run base_c4s $BASE --config C4 --share 8
  run new_c4s $NEW --config C4 --share 8
  run base_c5s $BASE --config C5 --share 8
  run new_c5s $NEW --config C5 --share 8
done
run base_c2 $BASE
run new_c2 $NEW
