# Round 5, call 19: GPU suite on HEAD with sha.hip's structurizer option, config 2 and config 4 lines
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_p.log 2>&1 || { tail -30 gpurun_out/r05_tests_p.log; exit 1; }
tail -1 gpurun_out/r05_tests_p.log
TAG=r05_head19 bash scripts/abrun.sh scripts/ab_r05_head19.txt || exit 1
