#!/bin/bash
# Round 6, call 19: the GPU suite on the default (two-pass) front after the fused-front changes; the parity
# subset with the fused front (no granule pass, four-segment digest copy); config 2 default vs fused.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests > gpurun_out/r06_tests_c19.log 2>&1 || { tail -30 gpurun_out/r06_tests_c19.log; exit 1; }
tail -1 gpurun_out/r06_tests_c19.log
HDRF_FUSED=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_bench_shape.py > gpurun_out/r06_tests_fz5.log 2>&1 || { tail -30 gpurun_out/r06_tests_fz5.log; exit 1; }
tail -1 gpurun_out/r06_tests_fz5.log
TAG=r06_fu bash scripts/abrun.sh scripts/ab_r06_fused2.txt
