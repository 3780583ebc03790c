#!/bin/bash
# Round 6, call 22: issue priorities on the chunking chain at HEAD (scripts/ab_r06_prio.txt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=r06_pr bash scripts/abrun.sh scripts/ab_r06_prio.txt
