# round 5: rehearsal of the N > 1 bench line on the one-GPU box (2 ranks on cuda:0 over gloo):
# the default C4 strong line at 20 M reads with its c2 record, then the sharded Bloom job
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --gpus 2 --rehearse-one-gpu --reads 8000000 --steps 2 --warmup 1 \
  --no-cpu-baseline > gpurun_out/r05_t11_n2.json 2> gpurun_out/r05_t11_n2.err || exit $?
timeout -k 10 600 python -u bench.py --gpus 2 --rehearse-one-gpu --config C3 --reads 5000000 --steps 2 --warmup 1 \
  --no-cpu-baseline > gpurun_out/r05_t11_n2_c3.json 2> gpurun_out/r05_t11_n2_c3.err
timeout -k 10 600 python -u bench.py --config C4 --reads 8000000 --steps 2 --warmup 1 --no-cpu-baseline --no-compact \
  --no-writer > gpurun_out/r05_t11_n1.json 2> gpurun_out/r05_t11_n1.err
