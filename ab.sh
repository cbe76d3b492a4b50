# A/B of engine builds on one box: bash ab.sh "libkc libkc_x" K1 [K2 ...]
set -e
L=canonical-k-mer-hash-table_amd/lib
V=$1; shift
for k in "$@"; do for r in 1 2; do
 for v in $V; do
  KC_LIB=$PWD/$L/${v}.so timeout -k 10 300 python bench.py --k $k --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.json 2>gpurun_out/ab_err.log
  echo "k$k $v $(python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print(round(d['value']/1e9,2), d['ms_per_step'])")"
 done; done; done
