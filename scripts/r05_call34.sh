# Round 5, call 34: config-2 issue priorities (walk, granule pass, place)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=r05_c2prio bash scripts/abrun.sh scripts/ab_r05_c2prio.txt || exit 1
