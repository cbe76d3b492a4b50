# round 5 A/B (9): the scatter loops without unrolled per-lane scan / bin loops (their hoisted trip
# counts were spilled) and one scatter loop for both two-word store formats (12-byte records or whole
# keys): k_p2f<2> 128 VGPRs + 84 B/lane of scratch -> 108 VGPRs, none; k_p1<1> 64 -> 8 B; k_p1<2> 24-36
# -> 0 B.  Parity tests, then C2 / C3 against lib_ab/libkc_head.so (the committed sources)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_bloom.py tests/test_gpu_defer.py > gpurun_out/r05_ab9_tests.log 2>&1 || exit 1
OUT=gpurun_out/r05_ab9.txt
: > $OUT
X="--no-cpu-baseline --no-compact --no-cli-fullsize --secondary none --tertiary none --no-writer"
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  KC_LIB=$lib timeout -k 10 300 python bench.py $X "$@" > gpurun_out/r05_ab9_$name.json 2>> gpurun_out/r05_ab9.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r05_ab9_$name.json').read().strip().splitlines()[-1]); print('$name', '$*', round(d['ms_per_step'],3), d['kernel_ms'], (d.get('parity') or {}).get('match'))" >> $OUT
}
NEW=$PWD/canonical-k-mer-hash-table_amd/lib/libkc.so
BASE=$PWD/lib_ab/libkc_head.so
for r in 1 2; do
  run base_c2 $BASE
  run new_c2 $NEW
  run base_c3 $BASE --config C3
  run new_c3 $NEW --config C3
done
bash tools/gpu_prof.sh r05_ab9_c3 --config C3 --no-cli-fullsize --secondary none --tertiary none --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab9_c3/run_kernel_stats.csv > gpurun_out/r05_ab9_c3_kstats.txt
bash tools/gpu_prof.sh r05_ab9_c2 --no-cli-fullsize --secondary none --tertiary none --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_r05_ab9_c2/run_kernel_stats.csv > gpurun_out/r05_ab9_c2_kstats.txt
