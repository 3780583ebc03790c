#!/bin/bash
# Round 3: with gmax2 the index + store stream (B) sets the period: place throttle and SHA waves A/B.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
NO_PMC=1 TAG=pl bash scripts/r03_ab.sh HDRF_PLACE_LDS=40960 HDRF_PLACE_LDS=24576 HDRF_PLACE_LDS=16384 HDRF_PLACE_LDS=0 HDRF_PLACE_LDS=40960 HDRF_PLACE_LDS=24576 "HDRF_PLACE_LDS=24576 HDRF_SHA_WPC=6" "HDRF_PLACE_LDS=16384 HDRF_SETPRIO=32"
