# PMC traffic of the default line's workloads and of the C4 / C5 per-GPU shares at HEAD
#   KC_COMMIT=<sha> bash tools/r03_pmc_all.sh
set -o pipefail
bash tools/gpu_pmc_traffic.sh C2 --secondary none --no-compact --no-verify || exit 1
bash tools/gpu_pmc_traffic.sh C3 --config C3 --no-compact --no-verify || exit 1
bash tools/gpu_pmc_traffic.sh C4s --config C4 --share 8 --no-compact --no-verify || exit 1
bash tools/gpu_pmc_traffic.sh C5s --config C5 --share 8 --no-compact --no-verify || exit 1
