#!/bin/bash
# Round 6, call 7: LZ4 windows of 128 B — byte parity of the LZ4 / compressor-2 / stream tests on the
# variant build, then the config-4 A/B (scripts/ab_r06_lz4win.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
HDRF_LIB_PATH=$R/hdrf_amd/_build_w128/libhdrf.so timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_lz4.py "tests/test_bench_shape.py::test_config4_bench_batches_depth5_full_state" > gpurun_out/r06_tests_c7.log 2>&1 || { tail -40 gpurun_out/r06_tests_c7.log; exit 1; }
tail -1 gpurun_out/r06_tests_c7.log
TAG=r06_lz4win bash scripts/abrun.sh scripts/ab_r06_lz4win.txt || exit 1
