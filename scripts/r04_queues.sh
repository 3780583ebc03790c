#!/bin/bash
# Round 4: config 2 with more hardware queues than the library's streams need folded (8 default).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
NO_PMC=1 TAG=r04_hwq BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-alone" bash scripts/r03_ab.sh \
  "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=12" "GPU_MAX_HW_QUEUES=16" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=12" "GPU_MAX_HW_QUEUES=16"
