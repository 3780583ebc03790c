#!/bin/bash
# Round 6, call 21: the kernel trace of the default config-2 line at HEAD (rocprofv3 --kernel-trace --stats),
# whose gmax2 / sha_carry / place averages the line's HIP-event figures are checked against.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06_prof_k3 -o run -- \
  python3 $R/bench.py --no-sub --no-cpu --no-corpus-check --steps 10 > $R/gpurun_out/r06_prof_k3.log 2>&1) || { tail -20 gpurun_out/r06_prof_k3.log; exit 1; }
grep '^{' gpurun_out/r06_prof_k3.log | tail -1 | cut -c1-200
