#!/bin/bash
# round-4 closing run at HEAD: the whole GPU suite, PMC traffic of C2 / C3 at the closing sources,
# the default bench line, its kernel traces, smoke().   bash tools/r04_close.sh NAME
set -o pipefail
N=${1:-r04_close}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${N}_gpu_tests.txt 2>&1 || exit 1
bash tools/r04_final.sh $N
