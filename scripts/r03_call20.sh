#!/bin/bash
# Round 3: gmax2 (15 VALU per granule, one 16-B store per thread): chunking parity, A/B vs the round-2 pass.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_config2_shape.py tests/test_bench_shape.py -m gpu > gpurun_out/c20_tests.log 2>&1 || { tail -30 gpurun_out/c20_tests.log; exit 1; }
tail -1 gpurun_out/c20_tests.log
NO_PMC=1 TAG=gv bash scripts/r03_ab.sh HDRF_GMAX_V=2 HDRF_GMAX_V=1 HDRF_GMAX_V=2 HDRF_GMAX_V=1 "HDRF_GMAX_V=2 HDRF_SHA_DUAL=1" "HDRF_GMAX_V=2 HDRF_SHA_WPC=6"
