# round 5: the drop-in CLI on the whole C2 / C3 inputs (page-cached files): the
# reference's timer lines per upload-reader count, and the output digest against fullsize.json
set -o pipefail
mkdir -p gpurun_out
B=canonical-k-mer-hash-table_amd/bin
D=${TMPDIR:-/tmp}/r05cli
mkdir -p $D
timeout -k 10 300 $B/kc_gen $D/c2.fasta 10000000 150 50000000 -s 42 -e 0.001 || exit $?
cat $D/c2.fasta > /dev/null
OUT=gpurun_out/r05_cli.txt
: > $OUT
for rd in 1 2 4 8; do
  for job in "31 -m 2 -s 200000000 -a 1" "51 -m 2 -b -u 400000000 -a 2"; do
    timeout -k 10 120 $B/kaarme $D/c2.fasta $job -t 18 --readers $rd --phases -o $D/out.txt > $D/log.txt 2> $D/err.txt || exit $?
    echo "readers=$rd job=[$job] $(grep -E 'Time used|Input path' $D/log.txt | tr '\n' ' ') phases: $(grep cli: $D/err.txt | tr '\n' ' ')" >> $OUT
    if [ $rd = 1 ]; then
      echo "digest job=[$job] $(timeout -k 10 120 oracle/_ref/kc_digest lines $D/out.txt)" >> $OUT || exit $?
    fi
  done
done
rm -rf $D
