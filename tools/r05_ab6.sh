# round 5 A/B (2): the format-independent loads with idle lanes reading nearby items, plus k_p2 / k_p1k
# loads before use and the runs merge's group starts in LDS; parity (parity, deferral, sharded, launch
# tests) first, then C2 x3 and C3 / C4 share against lib_ab/libkc_ins.so
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_defer.py tests/test_gpu_sharded.py tests/test_gpu_sharded_mp.py tests/test_gpu_sharded_fullsize.py \
  tests/test_gpu_bloom.py > gpurun_out/r05_ab6_tests.log 2>&1 || exit 1
OUT=gpurun_out/r05_ab6.txt
: > $OUT
X="--no-cpu-baseline --no-compact --no-cli-fullsize --secondary none --tertiary none --no-writer"
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  KC_LIB=$lib timeout -k 10 300 python bench.py $X "$@" > gpurun_out/r05_ab6_$name.json 2>> gpurun_out/r05_ab6.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_ab6_$name.json').read().strip().splitlines()[-1]); print('$name', '$*', round(d['ms_per_step'],3), d['kernel_ms'], (d.get('parity') or {}).get('match'))" >> $OUT
}
NEW=$PWD/canonical-k-mer-hash-table_amd/lib/libkc.so
BASE=$PWD/lib_ab/libkc_ins.so
for r in 1 2 3; do
  run base_c2 $BASE
  run new_c2 $NEW
done
for r in 1 2; do
  run base_c3 $BASE --config C3
  run new_c3 $NEW --config C3
  run base_c4s $BASE --config C4 --share 8
  run new_c4s $NEW --config C4 --share 8
done
bash tools/gpu_prof.sh r05_ab6_c2 --no-cli-fullsize --secondary none --tertiary none --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab6_c2/run_kernel_stats.csv > gpurun_out/r05_ab6_c2_kstats.txt
KC_LIB=$BASE bash tools/gpu_prof.sh r05_ab6_c2b --no-cli-fullsize --secondary none --tertiary none --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab6_c2b/run_kernel_stats.csv > gpurun_out/r05_ab6_c2b_kstats.txt
