#!/bin/bash
# Round 6, call 15: fused front with one compression site per step — config 2 speed, then the chunking /
# fingerprint parity tests with it on.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=r06_fy bash scripts/abrun.sh scripts/ab_r06_fused2.txt || exit 1
HDRF_FUSED=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_bench_shape.py > gpurun_out/r06_tests_fz2.log 2>&1; rc=$?
tail -3 gpurun_out/r06_tests_fz2.log
exit $rc
