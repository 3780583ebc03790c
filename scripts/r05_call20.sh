# Round 5, call 20: config-2 place throttle at HEAD; the LZ4 PMC record at HEAD
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=r05_throttle2 bash scripts/abrun.sh scripts/ab_r05_throttle2.txt || exit 1
bash scripts/r05_lz4pmc.sh || exit 1
