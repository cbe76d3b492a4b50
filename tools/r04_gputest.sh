# the whole GPU suite at HEAD (as the driver runs it), one process
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 900 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r04_gputest.log 2>&1
