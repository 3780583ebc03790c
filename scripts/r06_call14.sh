#!/bin/bash
# Round 6, call 14: the fused chunk + fingerprint front (HDRF_FUSED=1, lanehash.hip) — the GPU suite with it
# on, then config 2 default vs fused.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
HDRF_FUSED=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests > gpurun_out/r06_tests_fz1.log 2>&1; rc=$?
tail -5 gpurun_out/r06_tests_fz1.log
[ $rc -eq 0 ] || exit 1
TAG=r06_fz bash scripts/abrun.sh scripts/ab_r06_fused.txt
