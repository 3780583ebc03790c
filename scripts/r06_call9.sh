#!/bin/bash
# Round 6, call 9: the node-global rank at G = 4 on one GPU (loopback, bench batch shape, index 2^26 per
# rank so four contexts fit): kernel trace, and two global batches (256 x 128 MiB blocks) against the oracle.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06_prof_lb4 -o run -- python3 $R/scripts/node_loopback.py --G 4 --batches 4 --index-log2 26 > $R/gpurun_out/r06_prof_lb4.log 2>&1) || { echo "loopback trace failed"; tail -20 gpurun_out/r06_prof_lb4.log; exit 1; }
grep '^{' gpurun_out/r06_prof_lb4.log | cut -c1-300
timeout -k 10 600 python3 scripts/node_loopback.py --G 4 --batches 4 --index-log2 26 --check 2 > gpurun_out/r06_lb4_check.log 2>&1 || { tail -20 gpurun_out/r06_lb4_check.log; exit 1; }
grep '^{' gpurun_out/r06_lb4_check.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('G4', d['logical_GB_s_one_gpu'], d.get('oracle_check'))"
