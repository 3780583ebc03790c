# Round 5, call 17: chunk.hip with uniform regions unstructurized: GPU suite, config-2 A/B over the place throttle
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
HDRF_LIB_PATH=hdrf_amd/_build_c/libhdrf.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_o.log 2>&1 || { tail -30 gpurun_out/r05_tests_o.log; exit 1; }
tail -1 gpurun_out/r05_tests_o.log
TAG=r05_c2chunk bash scripts/abrun.sh scripts/ab_r05_c2chunk.txt || exit 1
