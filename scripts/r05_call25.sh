# Round 5, call 25: config-2 streaming-knob re-check at HEAD
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=r05_nt bash scripts/abrun.sh scripts/ab_r05_nt.txt || exit 1
