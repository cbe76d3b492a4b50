#!/bin/bash
# Several bench.py lines in one GPU call, each under its own time limit, stopping at the first
# failure.  usage: tools/bench_set.sh NAME "bench args 1" "bench args 2" ...
# Writes gpurun_out/NAME_<i>.json (the line) and .err (stderr, KC_DEBUG output if set).
set -o pipefail
N=$1; shift
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  echo "[$N $i] bench.py $a"
  timeout -k 10 ${BENCH_TIMEOUT:-420} python3 -u bench.py $a > gpurun_out/${N}_$i.json 2> gpurun_out/${N}_$i.err
  rc=$?
  tail -c 600 gpurun_out/${N}_$i.json; echo
  [ $rc -eq 0 ] || { echo "[$N $i] exit $rc"; tail -20 gpurun_out/${N}_$i.err; exit $rc; }
done
