#!/bin/bash
# round 6: SKM / estimate / deferral GPU tests, a kernel trace of the whole C4 job, then the two-rank
# C4 line rehearsed on one GPU (super-k-mer exchange over gloo).  usage: bash tools/r06_a.sh
set -o pipefail
bash tools/gpu_tests.sh t2 "skm or size_table or estimate or two_processes or deferred or rehearsed" \
  tests/test_gpu_skm.py tests/test_gpu_parity.py tests/test_gpu_sharded_mp.py tests/test_gpu_defer.py \
  tests/test_bench_launch.py || exit $?
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4e -o run \
  --output-format csv -- python3 $R/bench.py --config C4 --no-cpu-baseline --no-writer --no-compact --no-cli-fullsize \
  --steps 2 --warmup 1 > $R/gpurun_out/prof_c4e.json 2> $R/gpurun_out/prof_c4e.err) || exit $?
python3 tools/kstats.py gpurun_out/prof_c4e/run_kernel_stats.csv > gpurun_out/prof_c4e.txt || exit $?
KC_DEFER=2 timeout -k 10 600 python3 -u bench.py --gpus 2 --rehearse-one-gpu --config C4 --steps 2 --warmup 1 \
  --no-cpu-baseline --no-writer --no-compact --no-cli-fullsize --multi-secondary none \
  > gpurun_out/rehearse_c4.json 2> gpurun_out/rehearse_c4.err
