# The reference CLI built without and with -march=x86-64-v4 (oracle/Makefile) on the same
# C2 CPU-baseline sample, alternating, twice each: bash tools/ref_march_ab.sh
set -o pipefail
mkdir -p gpurun_out
T=${TMPDIR:-/tmp}
canonical-k-mer-hash-table_amd/bin/kc_gen $T/s.fa 10000000 150 50000000 -s 42 -e 0.001 --first 0 --count 1000000 || exit 1
cat $T/s.fa > /dev/null
TH=$(( ${OMP_NUM_THREADS:-16} + 2 ))
for r in 1 2; do for b in kaarme kaarme_v4; do
  timeout -k 10 300 oracle/_ref/$b $T/s.fa 31 -m 2 -t $TH -a 0 -s 156001000 > $T/o.txt 2>&1 || { echo "$b exit $?"; continue; }
  echo "$b $(grep 'Time used to build hash table' $T/o.txt)"
done; done
rm -f $T/s.fa
