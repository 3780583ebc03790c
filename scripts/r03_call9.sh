#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
HDRF_SHA_RING=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_bench_shape.py tests/test_gpu_parity.py tests/test_config2_shape.py -m gpu > gpurun_out/c9_tests.log 2>&1 || { tail -30 gpurun_out/c9_tests.log; exit 1; }
tail -1 gpurun_out/c9_tests.log
bash scripts/r03_ab.sh HDRF_SHA_RING=1 HDRF_SHA_RING=0 HDRF_SHA_RING=1 HDRF_SHA_RING=0 "HDRF_SHA_RING=1 HDRF_PLACE_LDS=16384"
