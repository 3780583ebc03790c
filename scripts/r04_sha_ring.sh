#!/bin/bash
# Round 4: sha_lring (HDRF_SHA_RING2=1: each 128-B line loaded once into a per-lane LDS ring) —
# parity under the env (GPU parity + bench-shape tests), then config-2 A/B vs the default kernel.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-a}
HDRF_SHA_RING2=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_bench_shape.py > gpurun_out/r04_sharing_tests_$V.log 2>&1 || { tail -30 gpurun_out/r04_sharing_tests_$V.log; exit 1; }
tail -1 gpurun_out/r04_sharing_tests_$V.log
NO_PMC=${NO_PMC:-1} TAG=r04_sharing_$V BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-alone" bash scripts/r03_ab.sh \
  "X=def" "HDRF_SHA_RING2=1" "HDRF_SHA_RING2=1 HDRF_SHA_WPC=6" "X=def" "HDRF_SHA_RING2=1" "HDRF_SHA_RING2=1 HDRF_SHA_WPC=6"
