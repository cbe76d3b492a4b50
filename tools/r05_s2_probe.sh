# round 5 (second session): where the level-3 kernels' time goes.  Kernel traces of probe builds
# (not correct results): pb1 = k_b3 without its insertion path (the gate test only), pb2 = k_b3
# loads only, pb3 = k_p3 loads only (no inserts); against the working-tree library
set -o pipefail
mkdir -p gpurun_out
N=r05_s2_probe
X="--no-cli-fullsize --secondary none --tertiary none --no-compact"
prof() {  # name lib args
  local name=$1 lib=$2; shift 2
  KC_LIB=$lib bash tools/gpu_prof.sh ${N}_$name $X "$@" || exit 1
  python3 tools/kstats.py gpurun_out/prof_${N}_$name/run_kernel_stats.csv | grep "kc::" > gpurun_out/${N}_${name}_kstats.txt
}
L=$PWD/lib_ab
prof c2_pb3 $L/libkc_pb3.so
prof c3_new $PWD/canonical-k-mer-hash-table_amd/lib/libkc.so --config C3
prof c3_pb1 $L/libkc_pb1.so --config C3
prof c3_pb2 $L/libkc_pb2.so --config C3
prof c3_pb3 $L/libkc_pb3.so --config C3
