# Round 5, call 27: config-2 A/B of the carried SHA window at HEAD (structurizer option on sha.hip)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=r05_carry bash scripts/abrun.sh scripts/ab_r05_carry.txt || exit 1
