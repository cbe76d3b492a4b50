# A/B of bench.py under environments (kernel trace): bash tools/probe/ab_env_bench.sh NAME "ENV_A" "ENV_B" [-- bench args]
# each environment twice, alternating; ENV is a space-separated list of VAR=value (or "-" for none)
set -o pipefail
R=$GRAFT_REPO_ROOT
N=$1; A=$2; C=$3; shift 3
[ "$1" = "--" ] && shift
mkdir -p $R/gpurun_out
i=0
for rep in 1 2; do
  for E in "$A" "$C"; do
    i=$((i+1))
    EV=$E; [ "$EV" = "-" ] && EV=""
    ( cd /tmp && export TMPDIR=/tmp && env $EV timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_${N}_$i -o run --output-format csv -- \
        python3 $R/bench.py --no-cpu-baseline --no-compact --steps 5 --warmup 2 "$@" > $R/gpurun_out/ab_${N}_$i.json 2> $R/gpurun_out/ab_${N}_$i.err ) || exit 1
    python3 $R/tools/kstats.py $R/gpurun_out/ab_${N}_$i/run_kernel_stats.csv > $R/gpurun_out/ab_${N}_$i.ks
    echo "== $i [$E] $(python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s=f\"{d['ms_per_step']:.3f} ms/step {d['value']/1e9:.2f} G parity={d.get('parity',{}).get('match')} tok={d['kernel_ms']['tokenize']} count={d['kernel_ms']['count']}\"
c=d.get('c3')
if c: s+=f\" | C3 {c['ms_per_step']:.3f} ms {c['value']/1e9:.2f} G parity={c.get('parity',{}).get('match')} tok={c['kernel_ms']['tokenize']} count={c['kernel_ms']['count']}\"
print(s)" $R/gpurun_out/ab_${N}_$i.json)"
    grep -E "k_emit|k_tile_summary|k_p1f?<|k_p2f|k_p3<|k_b3" $R/gpurun_out/ab_${N}_$i.ks | cut -c1-44,101-130
  done
done
