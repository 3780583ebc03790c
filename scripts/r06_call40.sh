#!/bin/bash
# Round 6, call 40: the lane walk in single-wave workgroups (its LDS per wave: any free slot, freed per wave;
# 4 instead of 3 waves per SIMD): GPU suite, the default line's kernel trace, then the A/B of scripts/ab_r06_walk1.txt.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests > gpurun_out/r06_tests_c40.log 2>&1 || { tail -30 gpurun_out/r06_tests_c40.log; exit 1; }
tail -1 gpurun_out/r06_tests_c40.log
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06_prof_c40 -o run -- \
  python3 $R/bench.py --no-sub --no-cpu --no-corpus-check --steps 10 > $R/gpurun_out/r06_prof_c40.log 2>&1) || { tail -20 gpurun_out/r06_prof_c40.log; exit 1; }
grep '^{' gpurun_out/r06_prof_c40.log | tail -1 | cut -c1-160
TAG=r06_wk1 bash scripts/abrun.sh scripts/ab_r06_walk1.txt
