#!/bin/bash
# Round 4: config-5 whole-block timeline at HEAD (paced CU drain), kernel + memory-copy trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/c5trace3 -o run -- python3 $R/bench.py --workload config5 --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/c5trace3.log 2>&1) || { tail -20 gpurun_out/c5trace3.log; exit 1; }
tail -1 gpurun_out/c5trace3.log | cut -c1-120
