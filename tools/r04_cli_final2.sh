# the drop-in CLI with its untimed warm-up pass: GPU CLI tests, then build times with and without it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "cli or gzip" > gpurun_out/r04_cli_tests2.txt 2>&1 || exit 1
B=canonical-k-mer-hash-table_amd/bin
F=/tmp/kc_cli_probe.fasta
$B/kc_gen $F 1000000 150 5000000 -s 42 -e 0.001 > /dev/null || exit 1
cat $F > /dev/null
O=gpurun_out/r04_cli_probe4.txt
: > $O
for r in 1 2 3; do
  for w in 0 1; do
    for rd in 1 2; do
      echo "== no_warmup=$w readers=$rd" >> $O
      env $( [ $w = 1 ] && echo KC_CLI_NO_WARMUP=1 ) KC_CLI_DEBUG=1 KC_CLI_READERS=$rd timeout -k 10 60 $B/kaarme $F 31 \
          -m 2 -s 156001000 -a 0 -t 18 2>&1 | grep -E "Time used to build|cli:|Processed" >> $O || exit 1
    done
  done
done
