#!/bin/bash
# Round 3: back stage split (index part on B, store part on B2 after idx_finalize): full GPU suite, then
# A/B: split vs not, with sha_line, place throttle.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/c22_tests.log 2>&1 || { tail -40 gpurun_out/c22_tests.log; exit 1; }
tail -1 gpurun_out/c22_tests.log
NO_PMC=1 TAG=sp bash scripts/r03_ab.sh HDRF_SPLIT_B=1 HDRF_SPLIT_B=0 HDRF_SPLIT_B=1 HDRF_SPLIT_B=0 HDRF_SHA_LINE=1 "HDRF_SHA_LINE=1 HDRF_PLACE_LDS=24576" "HDRF_PLACE_LDS=24576" "HDRF_SHA_LINE=1 HDRF_SPLIT_B=0"
