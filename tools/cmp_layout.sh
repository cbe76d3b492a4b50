set -o pipefail
mkdir -p gpurun_out
for lay in blocked reference; do
  KC_BLOOM_LAYOUT=$lay timeout -k 10 200 python bench.py --config C3 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/cmp_$lay.json 2> gpurun_out/cmp_$lay.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && KC_BLOOM_LAYOUT=reference timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_ref -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 2 --warmup 1 --config C3 > /dev/null 2>&1
