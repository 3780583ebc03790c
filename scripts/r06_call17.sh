#!/bin/bash
# Round 6, call 17: fused front with loads one step ahead (4 waves per SIMD) and per-block granule passes —
# parity subset with it on, then config 2 default vs fused.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
HDRF_FUSED=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_bench_shape.py > gpurun_out/r06_tests_fz4.log 2>&1 || { tail -30 gpurun_out/r06_tests_fz4.log; exit 1; }
tail -1 gpurun_out/r06_tests_fz4.log
TAG=r06_fv bash scripts/abrun.sh scripts/ab_r06_fused2.txt
