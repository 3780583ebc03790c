# Round 5, call 18: the structurizer option per file (sha / index / store on top of lz4 + chunk): config-2 A/B, then
# config 4 on HEAD
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=r05_c2files bash scripts/abrun.sh scripts/ab_r05_c2files.txt || exit 1
TAG=r05_c4head bash scripts/abrun.sh scripts/ab_r05_c4head.txt || exit 1
