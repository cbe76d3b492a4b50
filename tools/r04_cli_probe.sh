# the drop-in CLI's timed build on the C2 CPU-baseline sample (161 MB, 1 M x 150 bp): where its
# time goes (KC_CLI_DEBUG phase times: file -> HBM, the counting call, its queued work)
set -o pipefail
mkdir -p gpurun_out
B=canonical-k-mer-hash-table_amd/bin
F=/tmp/kc_cli_probe.fasta
$B/kc_gen $F 1000000 150 5000000 -s 42 -e 0.001 > /dev/null || exit 1
cat $F > /dev/null
O=gpurun_out/r04_cli_probe2.txt
: > $O
for r in 1 2 3; do
  for rd in 2 4; do
    echo "== readers=$rd" >> $O
    KC_CLI_DEBUG=1 KC_CLI_READERS=$rd timeout -k 10 60 $B/kaarme $F 31 -m 2 -s 156001000 -a 0 -t 18 \
        2>&1 | grep -E "Time used to build|cli:" >> $O || exit 1
  done
done
