# run harness binaries under a kernel trace: bash tools/probe/run.sh p_probe p_exp1 ...
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for b in "$@"; do
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/probe_$b -o run --output-format csv -- $R/tools/probe/$b 10000000 4 > $R/gpurun_out/probe_$b.log 2>&1 ) || exit 1
  echo "== $b"; grep iter gpurun_out/probe_$b.log | tail -1
  python3 tools/kstats.py gpurun_out/probe_$b/run_kernel_stats.csv > gpurun_out/probe_$b.ks
  grep -E "k_p1|k_p2f|k_p3<1, true" gpurun_out/probe_$b.ks
done
