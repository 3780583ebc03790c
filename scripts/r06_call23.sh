#!/bin/bash
# Round 6, call 23: issue priorities, second box (scripts/ab_r06_prio2.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=r06_pq bash scripts/abrun.sh scripts/ab_r06_prio2.txt
