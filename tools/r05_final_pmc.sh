# round 5 closing, part 1: PMC traffic (FETCH_SIZE / WRITE_SIZE passes) of C2, C3, C4, C5 at HEAD's sources
set -o pipefail
mkdir -p gpurun_out
X="--no-compact --no-verify --no-cli-fullsize --secondary none --tertiary none"
bash tools/gpu_pmc_traffic.sh C2 $X || exit 1
bash tools/gpu_pmc_traffic.sh C3 --config C3 $X || exit 1
bash tools/gpu_pmc_traffic.sh C4 --config C4 $X || exit 1
bash tools/gpu_pmc_traffic.sh C5 --config C5 $X --steps 2 || exit 1
