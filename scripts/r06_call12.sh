#!/bin/bash
# Round 6, call 12: SHA long-lane LDS A/B on config 2 (scripts/ab_r06_shalds.txt); the parity tests of the
# SHA stage (long lanes on and off) first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests > gpurun_out/r06_tests_c12.log 2>&1 || { tail -30 gpurun_out/r06_tests_c12.log; exit 1; }
tail -1 gpurun_out/r06_tests_c12.log
TAG=r06_sl bash scripts/abrun.sh scripts/ab_r06_shalds.txt
