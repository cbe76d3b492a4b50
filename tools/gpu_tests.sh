#!/bin/bash
# Selected GPU tests (pytest -k expression or ALL), one process, each under its own limit.
# usage: tools/gpu_tests.sh NAME "<pytest -k expr>|ALL" [test files...]
set -o pipefail
N=$1; K=$2; shift 2
mkdir -p gpurun_out
FILES=${@:-tests}
if [ "$K" = "ALL" ]; then KA=(); else KA=(-k "$K"); fi
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest $FILES -m gpu -x -v --timeout 300 --timeout-method thread \
  "${KA[@]}" > gpurun_out/${N}_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${N}_tests.log
exit $rc
