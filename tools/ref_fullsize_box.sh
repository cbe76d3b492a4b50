# The reference CLI at the bench's full C2 / C3 sizes on the GPU box's host cores (VERDICT r2
# item 4): kc_gen seed 42, 10 M x 150 bp, 50 Mbp genome; -t = the core share + 2 (16 hashing
# workers + the IO thread, main.cpp:383); the reference's own timer lines.
# usage: bash tools/ref_fullsize_box.sh [C2|C3 ...]  -> gpurun_out/ref_fullsize_box.txt
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/ref_fullsize_box.txt
W=${TMPDIR:-/tmp}/kc_ref_fullsize
mkdir -p $W
T=$(( ${OMP_NUM_THREADS:-16} + 2 ))
GEN=canonical-k-mer-hash-table_amd/bin/kc_gen
REF=oracle/_ref/kaarme
[ -f $W/C2.fasta ] || $GEN $W/C2.fasta 10000000 150 50000000 -s 42 -e 0.001 || exit 1
cat $W/C2.fasta > /dev/null
echo "host: $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2) nproc $(nproc) share ${OMP_NUM_THREADS:-?} -t $T" >> $OUT
# heartbeat: the reference's progress lines are block-buffered into the log
( while sleep 45; do echo "heartbeat $(date +%s)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for c in "$@"; do
  case $c in
    C2) args="31 -m 2 -s 200000000 -a 1";;
    C3) args="51 -m 2 -b -u 400000000 -a 2";;
  esac
  # the reference's workers occasionally crash it (a reference-side race, more often with more
  # threads): up to three attempts, each recorded
  for t in $T $T 10; do
    start=$(date +%s)
    timeout -k 10 1000 $REF $W/C2.fasta $args -t $t -o $W/$c.out > gpurun_out/ref_$c.log 2>&1
    rc=$?
    end=$(date +%s)
    echo "$c -t $t rc=$rc wall=$((end-start))s $(grep -h 'Time used' gpurun_out/ref_$c.log | tr '\n' ' ') $(grep -h 'Main array slots used' gpurun_out/ref_$c.log)" >> $OUT
    rm -f $W/$c.out
    [ $rc -eq 0 ] && break
  done
done
cat $OUT
