#!/bin/bash
# Round 6, call 11: place LDS reservation sweep on config 2 (scripts/ab_r06_placesweep.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=r06_ps bash scripts/abrun.sh scripts/ab_r06_placesweep.txt
