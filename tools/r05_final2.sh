# round 5 closing (after the load changes), part 1: the whole GPU suite, then the PMC traffic of C2 / C3 / C4 / C5
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r05_final2_gpu_tests.txt 2>&1 || exit 1
bash tools/r05_final_pmc.sh
