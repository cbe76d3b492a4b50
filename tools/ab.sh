# A/B of engine builds on one box, each bench line run twice, interleaved:
#   bash tools/ab.sh "libkc libkc_x" "--config C3" "--k 51" ...
# (builds in canonical-k-mer-hash-table_amd/lib/<name>.so, loaded through KC_LIB)
set -e
L=canonical-k-mer-hash-table_amd/lib
V=$1; shift
mkdir -p gpurun_out
for a in "$@"; do for r in 1 2; do
 for v in $V; do
  KC_LIB=$PWD/$L/${v}.so timeout -k 10 300 python bench.py $a --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.json 2>gpurun_out/ab_err.log
  echo "[$a] $v $(python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print(round(d['value']/1e9,2), round(d['ms_per_step'],3), d['kernel_ms'], d['distinct_per_gpu'])")"
 done; done; done
