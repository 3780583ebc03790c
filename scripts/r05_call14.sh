# Round 5, call 14: GPU suite on the catch-up if / else, config-4 A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_l.log 2>&1 || { tail -30 gpurun_out/r05_tests_l.log; exit 1; }
tail -1 gpurun_out/r05_tests_l.log
TAG=r05_lz4h bash scripts/abrun.sh scripts/ab_r05_lz4h.txt || exit 1
