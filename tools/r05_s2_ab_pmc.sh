# round 5 (second session): targeted GPU tests, an interleaved A/B of lib/libkc.so against
# lib_ab/libkc_head.so, then the PMC traffic passes of C2 / C3 / C4 at the working tree's sources
# (kept only if the change is kept).   bash tools/r05_s2_ab_pmc.sh NAME
set -o pipefail
N=$1
LIBS="head=lib_ab/libkc_head.so new=canonical-k-mer-hash-table_amd/lib/libkc.so" bash tools/r05_s2_abn.sh $N \
  "tests/test_gpu_parity.py tests/test_gpu_bloom.py tests/test_gpu_defer.py tests/test_gpu_sharded.py" \
  "--config C3" "--config C4 --share 8" "" || exit 1
X="--no-compact --no-verify --no-cli-fullsize --secondary none --tertiary none"
bash tools/gpu_pmc_traffic.sh C2 $X || exit 1
bash tools/gpu_pmc_traffic.sh C3 --config C3 $X || exit 1
bash tools/gpu_pmc_traffic.sh C4 --config C4 $X
