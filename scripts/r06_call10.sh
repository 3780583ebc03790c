#!/bin/bash
# Round 6, call 10: place_kernel LDS A/B on config 2 (scripts/ab_r06_placelds.txt), then the GPU suite
# (the X3 reservation now borrows the runs' LDS arrays).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=r06_pl bash scripts/abrun.sh scripts/ab_r06_placelds.txt || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests > gpurun_out/r06_tests_c10.log 2>&1 || { tail -30 gpurun_out/r06_tests_c10.log; exit 1; }
tail -1 gpurun_out/r06_tests_c10.log
