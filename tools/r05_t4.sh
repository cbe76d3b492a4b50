# round 5: the default bench line (C2 + c3 + c4 records, cli_fullsize, median-of-3 CPU baseline),
# the sharded Bloom job at one rank, and the PMC byte calibration (item 8)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r05_t4_bench.json 2> gpurun_out/r05_t4_bench.err && \
timeout -k 10 300 python -u bench.py --config C3 --force-sharded --no-cpu-baseline --no-cli-fullsize \
  > gpurun_out/r05_t4_c3sharded.json 2> gpurun_out/r05_t4_c3sharded.err && \
timeout -k 10 300 bash tools/pmc_calib/run.sh > gpurun_out/r05_t4_calib.log 2>&1
