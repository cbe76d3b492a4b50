set -o pipefail
mkdir -p gpurun_out
for v in 0 90000 0 90000; do
  KC_P1_LDS_MIN=$v timeout -k 10 200 python3 bench.py --config C4 --reads 12500000 --slots 1250000000 --no-cpu-baseline --no-compact --steps 10 --warmup 2 > gpurun_out/ab_p1_$v.json 2>/dev/null || exit $?
  python3 -c "import json,sys;d=[json.loads(l) for l in open('gpurun_out/ab_p1_$v.json') if l.startswith('{')][0];print('C4s LDS_MIN=$v', round(d['value']/1e9,2), d['kernel_ms'])" | tee -a gpurun_out/ab_p1.txt
done
for v in 0 90000; do
  KC_P1_LDS_MIN=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-compact --secondary none --steps 20 --warmup 3 > gpurun_out/ab_p1c2_$v.json 2>/dev/null || exit $?
  python3 -c "import json,sys;d=[json.loads(l) for l in open('gpurun_out/ab_p1c2_$v.json') if l.startswith('{')][0];print('C2 LDS_MIN=$v', round(d['value']/1e9,2), d['kernel_ms'])" | tee -a gpurun_out/ab_p1.txt
done
