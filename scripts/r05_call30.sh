# Round 5, call 30: more config-2 knobs at HEAD
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=r05_knobs3 bash scripts/abrun.sh scripts/ab_r05_knobs3.txt || exit 1
