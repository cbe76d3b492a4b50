# drop-in CLI input paths on the C2 1 M-read sample: host chunks (KC_CLI_HOST=1, kc_count_chunk
# staging; KC_COPY_THREADS=1 = single-threaded stage copies) vs the HBM image (readers x slices)
set -o pipefail
T=${TMPDIR:-/tmp}
canonical-k-mer-hash-table_amd/bin/kc_gen $T/s.fa 10000000 150 50000000 -s 42 -e 0.001 --first 0 --count 1000000 || exit 1
cat $T/s.fa > /dev/null
for r in 1 2; do
  for v in "KC_CLI_HOST=1 KC_COPY_THREADS=1" "KC_CLI_HOST=1" "KC_CLI_READERS=16 KC_CLI_SLICE_MB=32" "KC_CLI_READERS=4 KC_CLI_SLICE_MB=8" "KC_CLI_READERS=2 KC_CLI_SLICE_MB=8" "KC_CLI_READERS=8 KC_CLI_SLICE_MB=4"; do
    env $v timeout -k 10 120 canonical-k-mer-hash-table_amd/bin/kaarme $T/s.fa 31 -m 2 -a 0 -s 156001000 > $T/o.txt 2>&1 || exit 1
    echo "$v: $(grep -E 'Time used to build hash table' $T/o.txt)"
  done
done
rm -f $T/s.fa
