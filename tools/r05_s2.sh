# round 5, second session: the whole GPU suite at HEAD, smoke(), then the default bench line
set -o pipefail
mkdir -p gpurun_out
N=${1:-r05_s2}
bash tools/r05_suite.sh ${N} || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/${N}_bench.json 2> gpurun_out/${N}_bench.err
