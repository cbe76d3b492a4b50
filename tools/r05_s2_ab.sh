# round 5 (second session) A/B: working-tree library (lib/libkc.so) against lib_ab/libkc_base.so (HEAD);
# targeted parity tests first, then interleaved bench lines.  usage: tools/r05_s2_ab.sh NAME "tests" "config args" ...
set -o pipefail
mkdir -p gpurun_out
N=$1; T=$2; shift 2
if [ "$T" != "none" ]; then
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu $T \
  > gpurun_out/${N}_tests.log 2>&1 || exit 1
fi
OUT=gpurun_out/${N}.txt
: > $OUT
X="--no-cpu-baseline --no-compact --no-cli-fullsize --secondary none --tertiary none --no-writer"
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  KC_LIB=$lib timeout -k 10 300 python bench.py $X "$@" > gpurun_out/${N}_$name.json 2>> gpurun_out/${N}.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/${N}_$name.json').read().strip().splitlines()[-1]); print('$name', '$*', round(d['ms_per_step'],3), d['kernel_ms'], (d.get('parity') or {}).get('match'))" >> $OUT
}
NEW=$PWD/canonical-k-mer-hash-table_amd/lib/libkc.so
BASE=$PWD/lib_ab/libkc_base.so
for a in "$@"; do for r in 1 2 3; do
  run base $BASE $a || exit 1
  run new $NEW $a || exit 1
done; done
bash tools/gpu_prof.sh ${N}_new --no-cli-fullsize --secondary none --tertiary none --no-compact $1 || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}_new/run_kernel_stats.csv > gpurun_out/${N}_new_kstats.txt
