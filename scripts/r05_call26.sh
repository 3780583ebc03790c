# Round 5, call 26: LZ4 tests on the XOR-commit build, config-4 A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
HDRF_LIB_PATH=hdrf_amd/_build_xor/libhdrf.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "lz4 or compressor or config4 or stream" > gpurun_out/r05_tests_t.log 2>&1 || { tail -30 gpurun_out/r05_tests_t.log; exit 1; }
tail -1 gpurun_out/r05_tests_t.log
TAG=r05_xor bash scripts/abrun.sh scripts/ab_r05_xor.txt || exit 1
