# Round 5, call 33: config-4 parse waves per CU (room for a SHA wave beside the parse)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=r05_c4waves bash scripts/abrun.sh scripts/ab_r05_c4waves.txt || exit 1
