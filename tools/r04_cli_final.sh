# the drop-in CLI's GPU tests at HEAD (two upload readers by default), then the readers x slice probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider -k "cli or gzip" > gpurun_out/r04_cli_tests.txt 2>&1 || exit 1
bash tools/r04_cli_probe3.sh
