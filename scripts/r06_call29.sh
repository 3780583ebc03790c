#!/bin/bash
# Round 6, call 29: A/A control of the A/B harness and the SegMeta-store variant with the order swapped
# (scripts/ab_r06_aa.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=r06_aa bash scripts/abrun.sh scripts/ab_r06_aa.txt
