# round 5: tools/r05_t5.sh (C4 / C5 sizing, the 8-rank C4 merge test) then tools/r05_cli.sh
set -o pipefail
bash tools/r05_t5.sh && bash tools/r05_cli.sh
