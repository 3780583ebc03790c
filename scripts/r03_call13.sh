#!/bin/bash
# Round 3: granule pass on its own stream with a deeper pipeline (the pass of batch k+3 can then run
# while batch k+2 walks and stitches), against the defaults; then the node tests (RCCL exchanges on
# the library's back stream) and config 4 with its CPU baseline + LZ4 counters.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
NO_PMC=1 TAG=d4g BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-alone --depth 4" bash scripts/r03_ab.sh HDRF_GMAX_STREAM=1 HDRF_GMAX_STREAM=0 HDRF_GMAX_STREAM=1 || exit 1
NO_PMC=1 TAG=d5g BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-alone --depth 5" bash scripts/r03_ab.sh HDRF_GMAX_STREAM=1 "HDRF_GMAX_STREAM=1 HDRF_SHA_WPC=6" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_node.py -m gpu > gpurun_out/r03_node_tests.log 2>&1 || { tail -30 gpurun_out/r03_node_tests.log; exit 1; }
tail -1 gpurun_out/r03_node_tests.log
bash scripts/r03_call12.sh
