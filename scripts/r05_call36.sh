# Round 5, call 36: config-4 place LDS reservation (0 / 4 KiB vs 8 KiB)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=r05_c4place bash scripts/abrun.sh scripts/ab_r05_c4place.txt || exit 1
