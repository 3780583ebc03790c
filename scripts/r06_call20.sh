#!/bin/bash
# Round 6, call 20: config-2 knob re-check at HEAD (scripts/ab_r06_knobs.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=r06_kn bash scripts/abrun.sh scripts/ab_r06_knobs.txt
