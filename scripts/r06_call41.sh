#!/bin/bash
# Round 6, call 41: rebalancing after the single-wave walk (scripts/ab_r06_walk1b.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=r06_wk2 bash scripts/abrun.sh scripts/ab_r06_walk1b.txt
