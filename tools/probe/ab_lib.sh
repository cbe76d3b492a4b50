# A/B of library builds on bench.py (kernel trace): bash tools/probe/ab_lib.sh NAME LIB... [-- bench args]
# LIB = path of a libkc.so build (KC_LIB), or "default"
set -o pipefail
N=$1; shift
LIBS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" = "--" ] && shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
i=0
for L in "${LIBS[@]}"; do
  i=$((i+1))
  if [ "$L" = default ]; then unset KC_LIB; else export KC_LIB=$R/$L; fi
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ab_${N}_$i -o run --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline --no-compact --no-verify --secondary none --steps 5 --warmup 2 "$@" \
      > $R/gpurun_out/ab_${N}_$i.json 2> $R/gpurun_out/ab_${N}_$i.err ) || exit 1
  python3 $R/tools/kstats.py $R/gpurun_out/ab_${N}_$i/run_kernel_stats.csv > $R/gpurun_out/ab_${N}_$i.ks
  echo "== $i $L $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3), 'ms/step', round(d['value']/1e9,2), 'G')" $R/gpurun_out/ab_${N}_$i.json)"
  grep -E "k_emit|k_tile_summary|k_p1<|k_p2f|k_p3<|k_b3" $R/gpurun_out/ab_${N}_$i.ks | cut -c1-40,101-130
done
