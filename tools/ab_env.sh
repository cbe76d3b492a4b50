# same-box A/B of one environment variable: bash tools/ab_env.sh VAR "v1 v2 ..." "bench args"
# ("-" = unset)
set -e
VAR=$1; VALS=$2; ARGS=$3
mkdir -p gpurun_out
for r in 1 2; do
 for v in $VALS; do
  if [ "$v" = "-" ]; then unset $VAR; else export $VAR=$v; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline $ARGS > gpurun_out/abe.json 2>gpurun_out/abe.err
  echo "$VAR=$v [$ARGS] $(python3 -c "import json;d=json.load(open('gpurun_out/abe.json'));print(round(d['value']/1e9,2), round(d['ms_per_step'],3), d['kernel_ms'])")"
 done
done
