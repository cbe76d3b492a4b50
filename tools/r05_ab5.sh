# round 5 A/B: loads into format-independent registers (no merge copies after loads) in k_p2f<2>, k_p3, k_b3;
# parity of the whole GPU suite first (table keys, Bloom positions, the sharded paths), then C3 / C4 / C5
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05_ab5_tests.log 2>&1 || exit 1
OUT=gpurun_out/r05_ab5.txt
: > $OUT
X="--no-cpu-baseline --no-compact --no-cli-fullsize --secondary none --tertiary none --no-writer"
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  KC_LIB=$lib timeout -k 10 300 python bench.py $X "$@" > gpurun_out/r05_ab5_$name.json 2>> gpurun_out/r05_ab5.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_ab5_$name.json').read().strip().splitlines()[-1]); print('$name', '$*', round(d['ms_per_step'],3), d['kernel_ms'], (d.get('parity') or {}).get('match'))" >> $OUT
}
NEW=$PWD/canonical-k-mer-hash-table_amd/lib/libkc.so
BASE=$PWD/lib_ab/libkc_ins.so
for r in 1 2; do
  run base_c3 $BASE --config C3
  run new_c3 $NEW --config C3
  run base_c4s $BASE --config C4 --share 8
  run new_c4s $NEW --config C4 --share 8
  run base_c5s $BASE --config C5 --share 8
  run new_c5s $NEW --config C5 --share 8
  run base_c2 $BASE
  run new_c2 $NEW
done
