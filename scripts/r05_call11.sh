# Round 5, call 11: config-4 knobs after the LZ4 changes; LZ4 PMC record (VALU issue per SIMD-cycle)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=r05_c4knobs bash scripts/abrun.sh scripts/ab_r05_c4knobs.txt || exit 1
bash scripts/r05_lz4pmc.sh || exit 1
