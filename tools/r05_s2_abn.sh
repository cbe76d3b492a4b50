# round 5 (second session) A/B of several libraries on one box, interleaved:
#   LIBS="base=lib_ab/libkc_base.so new=canonical-k-mer-hash-table_amd/lib/libkc.so ..." \
#   bash tools/r05_s2_abn.sh NAME "tests|none" "bench args" ...
# targeted parity tests (with lib/libkc.so) first; each bench line 2 times per library
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
for a in "$@"; do for r in 1 2; do for nl in $LIBS; do
  name=${nl%%=*}; lib=$PWD/${nl#*=}
  KC_LIB=$lib timeout -k 10 300 python bench.py $X $a > gpurun_out/${N}_$name.json 2>> gpurun_out/${N}.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/${N}_$name.json').read().strip().splitlines()[-1]); print('$name', '$a', round(d['ms_per_step'],3), d['kernel_ms'], (d.get('parity') or {}).get('match'))" >> $OUT
done; done; done
