# round 5 closing, part 2: the default bench line, kernel traces of C2 / C3 / C4 / C5, the N > 1 rehearsal
# test, smoke()
set -o pipefail
mkdir -p gpurun_out
N=${1:-r05_final}
timeout -k 10 900 python -u bench.py > gpurun_out/${N}_bench.json 2> gpurun_out/${N}_bench.err || exit 1
bash tools/gpu_prof.sh ${N} --no-cli-fullsize --secondary none --tertiary none || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}/run_kernel_stats.csv > gpurun_out/${N}_kernel_stats.txt || exit 1
bash tools/gpu_prof.sh ${N}_c3 --config C3 --no-cli-fullsize || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}_c3/run_kernel_stats.csv > gpurun_out/${N}_c3_kernel_stats.txt || exit 1
bash tools/gpu_prof.sh ${N}_c4 --config C4 --no-compact || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}_c4/run_kernel_stats.csv > gpurun_out/${N}_c4_kernel_stats.txt || exit 1
bash tools/gpu_prof.sh ${N}_c5 --config C5 --no-compact --steps 2 || exit 1
python3 tools/kstats.py gpurun_out/prof_${N}_c5/run_kernel_stats.csv > gpurun_out/${N}_c5_kernel_stats.txt || exit 1
timeout -k 10 700 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_bench_launch.py \
  > gpurun_out/${N}_launch_tests.txt 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${N}_smoke.txt 2>&1
