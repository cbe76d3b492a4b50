# A/B of one harness binary under two environments: bash tools/probe/ab_env.sh BIN "ENV_A" "ENV_B"
set -o pipefail
R=$GRAFT_REPO_ROOT
B=$1; A=$2; C=$3
for rep in 1 2; do
  for E in "$A" "$C"; do
    tag=$(echo "$E" | tr -c 'A-Za-z0-9' '_')
    ( cd /tmp && export TMPDIR=/tmp && env $E timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_$tag -o run --output-format csv -- $R/tools/probe/$B 10000000 4 > $R/gpurun_out/ab_$tag.log 2>&1 ) || exit 1
    echo "== $E"; grep iter gpurun_out/ab_$tag.log | tail -1
    python3 tools/kstats.py gpurun_out/ab_$tag/run_kernel_stats.csv | grep -E "k_p1<|k_p2f|k_p3<1, true"
  done
done
