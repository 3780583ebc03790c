#!/bin/bash
# Round 6, call 28: the walk's SegMeta records stored together (-DHDRF_COOP_META=1 in hdrf_amd/_build_ab2):
# chunking parity subset on that build, then the config-2 A/B (scripts/ab_r06_meta.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
HDRF_LIB_PATH=$R/hdrf_amd/_build_ab2/libhdrf.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -m gpu tests/test_gpu_parity.py tests/test_bench_shape.py > gpurun_out/r06_tests_c28.log 2>&1 || { tail -30 gpurun_out/r06_tests_c28.log; exit 1; }
tail -1 gpurun_out/r06_tests_c28.log
TAG=r06_me bash scripts/abrun.sh scripts/ab_r06_meta.txt
