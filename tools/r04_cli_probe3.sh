# the drop-in CLI's file -> HBM upload on the C2 CPU-baseline sample (161 MB): reader threads x
# pinned slice size (KC_CLI_READERS, KC_CLI_SLICE_MB), KC_CLI_DEBUG phase times
set -o pipefail
mkdir -p gpurun_out
B=canonical-k-mer-hash-table_amd/bin
F=/tmp/kc_cli_probe.fasta
$B/kc_gen $F 1000000 150 5000000 -s 42 -e 0.001 > /dev/null || exit 1
cat $F > /dev/null
O=gpurun_out/r04_cli_probe3.txt
: > $O
for r in 1 2; do
  for rd in 1 2 3; do
    for sl in 8 16 32; do
      echo "== readers=$rd slice_mb=$sl" >> $O
      KC_CLI_DEBUG=1 KC_CLI_READERS=$rd KC_CLI_SLICE_MB=$sl timeout -k 10 60 $B/kaarme $F 31 -m 2 -s 156001000 -a 0 -t 18 \
          2>&1 | grep -E "Time used to build|cli:" >> $O || exit 1
    done
  done
done
