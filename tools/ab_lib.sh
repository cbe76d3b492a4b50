# same-box A/B of two builds of libkc.so (KC_LIB): the default bench line (C2 + the C3 record)
# alternated twice.  usage: tools/ab_lib.sh OUT_NAME lib_ab/libkc_variant.so
set -o pipefail
NAME=$1; ALT=$2
mkdir -p gpurun_out
for r in 1 2; do
  for lib in canonical-k-mer-hash-table_amd/lib/libkc.so "$ALT"; do
    KC_LIB=$PWD/$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-compact --steps 20 --warmup 3 > gpurun_out/ab.json 2>/dev/null || exit $?
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/ab.json') if l.startswith('{')][0]
print('$lib', 'C2', round(d['value']/1e9,2), d['kernel_ms'], 'C3', round(d['c3']['value']/1e9,2), d['c3'].get('kernel_ms'))" | tee -a gpurun_out/$NAME.txt
  done
done
