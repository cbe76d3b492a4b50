# kernel-trace profiles: bash tools/gpu_prof2.sh NAME "bench args" [NAME "bench args" ...]
# (KC_LIB etc. may be set per entry as VAR=value inside the args string's env prefix "env:")
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
while [ $# -gt 1 ]; do
  N=$1; A=$2; shift 2
  LIBV=""
  case "$N" in *@*) LIBV=${N#*@}; N=${N%@*};; esac
  if [ -n "$LIBV" ]; then export KC_LIB=$GRAFT_REPO_ROOT/canonical-k-mer-hash-table_amd/lib/$LIBV.so; else unset KC_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$N -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 2 --warmup 1 $A > $GRAFT_REPO_ROOT/gpurun_out/prof_$N.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_$N.err || exit 1
done
