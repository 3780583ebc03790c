#!/bin/bash
# Round 6, call 13: GPU suite with the wide recipe copy, then its config-2 A/B (scripts/ab_r06_recipe.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests > gpurun_out/r06_tests_c13.log 2>&1 || { tail -30 gpurun_out/r06_tests_c13.log; exit 1; }
tail -1 gpurun_out/r06_tests_c13.log
TAG=r06_rc bash scripts/abrun.sh scripts/ab_r06_recipe.txt
