#!/bin/bash
# Round 6, call 27: the cooperative copies as the default, A/B on a second box with the roles and order swapped
# (scripts/ab_r06_coop2.txt), after the GPU suite on the new default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests > gpurun_out/r06_tests_c27.log 2>&1 || { tail -30 gpurun_out/r06_tests_c27.log; exit 1; }
tail -1 gpurun_out/r06_tests_c27.log
TAG=r06_cp bash scripts/abrun.sh scripts/ab_r06_coop2.txt
