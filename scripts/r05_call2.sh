#!/bin/bash
# Round 5 call 2: the whole GPU suite (node-global pipeline rework, reset_async), then the A/B of
# the primed config-2 steps and the place throttle / depth under them.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-b}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_tests_$V.log 2>&1 || { tail -60 gpurun_out/r05_tests_$V.log; exit 1; }
tail -2 gpurun_out/r05_tests_$V.log
TAG=r05_prime bash scripts/abrun.sh scripts/ab_r05_prime.txt
