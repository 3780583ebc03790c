# Round 5, call 21: the scans + flush moved to stream B (place alone on B2): GPU suite, A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_q.log 2>&1 || { tail -30 gpurun_out/r05_tests_q.log; exit 1; }
tail -1 gpurun_out/r05_tests_q.log
TAG=r05_flushb bash scripts/abrun.sh scripts/ab_r05_flushb.txt || exit 1
