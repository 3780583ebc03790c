# Round 5, call 16: the structurizer flag (uniform regions left unstructurized): GPU suite on the lz4-only
# build and on the all-files build, config-4 and config-2 A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_n.log 2>&1 || { tail -30 gpurun_out/r05_tests_n.log; exit 1; }
tail -1 gpurun_out/r05_tests_n.log
HDRF_LIB_PATH=hdrf_amd/_build_all/libhdrf.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_n_all.log 2>&1 || { tail -30 gpurun_out/r05_tests_n_all.log; exit 1; }
tail -1 gpurun_out/r05_tests_n_all.log
TAG=r05_lz4j bash scripts/abrun.sh scripts/ab_r05_lz4j.txt || exit 1
TAG=r05_c2struct bash scripts/abrun.sh scripts/ab_r05_c2struct.txt || exit 1
