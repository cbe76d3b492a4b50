# A/B of bench.py under environment settings, kernel trace each: bash tools/ab_bench_env.sh "CONFIG" "ENV_A" "ENV_B"
set -o pipefail
R=$GRAFT_REPO_ROOT
CFG=$1; shift
mkdir -p gpurun_out
for rep in 1 2; do
  for E in "$@"; do
    tag=$(echo "$CFG$E" | tr -c 'A-Za-z0-9' '_')
    ( cd /tmp && export TMPDIR=/tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/abb_$tag -o run --output-format csv -- python3 $R/bench.py --config $CFG --no-cpu-baseline --no-compact --no-verify --steps 3 --warmup 1 > $R/gpurun_out/abb_$tag.json 2> $R/gpurun_out/abb_$tag.err ) || exit 1
    echo "== $CFG $E $(python3 -c "import json;d=json.load(open('$R/gpurun_out/abb_$tag.json'));print(round(d['ms_per_step'],3),'ms',round(d['value']/1e9,2),'G')")"
    python3 tools/kstats.py gpurun_out/abb_$tag/run_kernel_stats.csv | grep -E "k_p1<|k_p2f|k_p3<|k_b3|k_emit|k_tile_summary" | grep -v "OutExact\|k_p3<[0-9], false"
  done
done
