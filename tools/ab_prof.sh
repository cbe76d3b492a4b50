# same-box A/B of engine builds with a kernel trace each: bash tools/ab_prof.sh "libA libB" [bench args]
set -o pipefail
L=$GRAFT_REPO_ROOT/canonical-k-mer-hash-table_amd/lib
V=$1; shift
mkdir -p gpurun_out
for r in 1 2; do for v in $V; do
  ( cd /tmp && export TMPDIR=/tmp && KC_LIB=$L/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/abp_$v -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --secondary none --steps 5 --warmup 2 "$@" > $GRAFT_REPO_ROOT/gpurun_out/abp_$v.json 2>$GRAFT_REPO_ROOT/gpurun_out/abp_$v.err ) || exit 1
  echo "== $v r$r $(python3 -c "import json;d=json.load(open('gpurun_out/abp_$v.json'));print(round(d['value']/1e9,2), round(d['ms_per_step'],3), d['kernel_ms'])")"
  python3 tools/kstats.py gpurun_out/abp_$v/run_kernel_stats.csv > gpurun_out/abp_$v.ks; grep -E "k_p1<|k_p2f|k_p3<|k_emit|k_tile_summary" gpurun_out/abp_$v.ks | grep -v "OutExact\|false, true\|false, false, false"
done; done
