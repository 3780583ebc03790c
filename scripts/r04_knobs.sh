#!/bin/bash
# Round 4: config-2 knob A/B at HEAD (index epochs: no per-step table clear), alternated, no PMC.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
NO_PMC=1 TAG=r04_knobs BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-alone" bash scripts/r03_ab.sh \
  "X=def" "HDRF_SHA_CARRY=1" "HDRF_PLACE_LDS=32768" "HDRF_PLACE_LDS=49152" "X=def" "HDRF_SHA_CARRY=1" "HDRF_PLACE_LDS=32768" "HDRF_PLACE_LDS=49152"
