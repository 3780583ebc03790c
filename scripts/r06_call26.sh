#!/bin/bash
# Round 6, call 26: wave-cooperative list / offsets copies (-DHDRF_COOP=1 in hdrf_amd/_build_ab): chunking parity
# subset on that build (and the fused tests, whose stitch shares the copy), then the config-2 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
HDRF_LIB_PATH=$R/hdrf_amd/_build_ab/libhdrf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_bench_shape.py tests/test_fused_front.py > gpurun_out/r06_tests_c26.log 2>&1 || { tail -30 gpurun_out/r06_tests_c26.log; exit 1; }
tail -1 gpurun_out/r06_tests_c26.log
TAG=r06_co bash scripts/abrun.sh scripts/ab_r06_coop.txt
