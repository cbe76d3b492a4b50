# kernel-trace profile of one bench config: bash tools/gpu_prof.sh NAME [bench args...]
set -o pipefail
N=$1; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$N -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-writer --steps 3 --warmup 1 "$@" > $GRAFT_REPO_ROOT/gpurun_out/prof_$N.json 2>$GRAFT_REPO_ROOT/gpurun_out/prof_$N.err
