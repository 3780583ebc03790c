# Round 5, call 32: config-4 knobs at HEAD (SHA / LZ4 issue priority, SHA waves per CU, depth)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=r05_c4knobs2 bash scripts/abrun.sh scripts/ab_r05_c4knobs2.txt || exit 1
