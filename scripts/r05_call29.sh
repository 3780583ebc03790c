# Round 5, call 29: config-2 knobs re-checked with sha_carry as the default
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=r05_knobs2 bash scripts/abrun.sh scripts/ab_r05_knobs2.txt || exit 1
