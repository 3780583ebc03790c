#!/bin/bash
# v13: default workload now batches 32 blocks; FETCH/WRITE PMC passes, then bench + rocprof stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/pmc.sh v13 --steps 1 --warmup 1 --no-cpu || exit 1
bash scripts/r01_prof.sh || exit 1
