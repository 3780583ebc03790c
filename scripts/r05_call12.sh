# Round 5, call 12: GPU suite on the restructured chain loop; LZ4 tests on the unmasked-store build; config-4 A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_j.log 2>&1 || { tail -30 gpurun_out/r05_tests_j.log; exit 1; }
tail -1 gpurun_out/r05_tests_j.log
HDRF_LIB_PATH=hdrf_amd/_build_us/libhdrf.so timeout -k 10 300 python -u -m pytest tests/test_lz4.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_j_us.log 2>&1 || { tail -30 gpurun_out/r05_tests_j_us.log; exit 1; }
tail -1 gpurun_out/r05_tests_j_us.log
TAG=r05_lz4f bash scripts/abrun.sh scripts/ab_r05_lz4f.txt || exit 1
