#!/bin/bash
# Round 3: knob sensitivities at HEAD (config 2): SHA waves per CU, granule pass on its own stream,
# place throttle, depth 4; plus the Infinity-Cache probe.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 120 ./tools/_build/mall_probe > gpurun_out/mall_probe.txt 2>&1 || { tail -20 gpurun_out/mall_probe.txt; exit 1; }
cat gpurun_out/mall_probe.txt
NO_PMC=1 TAG=k11 bash scripts/r03_ab.sh HDRF_SHA_WPC=8 HDRF_SHA_WPC=6 HDRF_SHA_WPC=12 HDRF_GMAX_STREAM=1 HDRF_PLACE_LDS=24576 HDRF_PLACE_LDS=65536 HDRF_SHA_WPC=8 || exit 1
NO_PMC=1 TAG=k11d BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-alone --depth 4" bash scripts/r03_ab.sh HDRF_SHA_WPC=8 || exit 1
