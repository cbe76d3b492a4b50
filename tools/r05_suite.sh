# round 5: the whole GPU suite at HEAD, then smoke()
set -o pipefail
mkdir -p gpurun_out
N=${1:-r05_suite}
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${N}_gpu_tests.txt 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${N}_smoke.txt 2>&1
