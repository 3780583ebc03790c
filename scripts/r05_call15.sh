# Round 5, call 15: GPU suite on the scalar trims, config-4 A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_m.log 2>&1 || { tail -30 gpurun_out/r05_tests_m.log; exit 1; }
tail -1 gpurun_out/r05_tests_m.log
TAG=r05_lz4i bash scripts/abrun.sh scripts/ab_r05_lz4i.txt || exit 1
