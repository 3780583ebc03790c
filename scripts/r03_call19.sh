#!/bin/bash
# Round 3: sha_dual with one-iteration-ahead window loads: parity (both hashers), A/B on config 2, config 4 knobs.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
HDRF_SHA_DUAL=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_config2_shape.py tests/test_bench_shape.py -m gpu > gpurun_out/c19_tests.log 2>&1 || { tail -30 gpurun_out/c19_tests.log; exit 1; }
tail -1 gpurun_out/c19_tests.log
NO_PMC=1 TAG=dual2 bash scripts/r03_ab.sh HDRF_SHA_DUAL=1 HDRF_SHA_DUAL=0 HDRF_SHA_DUAL=1 HDRF_SHA_DUAL=0 "HDRF_SHA_DUAL=1 HDRF_SHA_WPC=6" "HDRF_SHA_DUAL=1 HDRF_SHA_WPC=8"
bash scripts/r03_call18.sh
NO_PMC=1 TAG=gv bash scripts/r03_ab.sh HDRF_GMAX_V=2 HDRF_GMAX_V=1 HDRF_GMAX_V=2 HDRF_GMAX_V=1
