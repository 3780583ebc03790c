#!/bin/bash
# Round 3: confirm the carried SHA window (default, untrimmed) against HDRF_SHA_CARRY=0, four pairs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
i=0
for v in "HDRF_SHA_CARRY=0" "X=0" "HDRF_SHA_CARRY=0" "X=0" "HDRF_SHA_CARRY=0" "X=0" "HDRF_SHA_CARRY=0" "X=0"; do
  i=$((i+1))
  env $v timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/c31_$i.json.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/c31_$i.json.log; exit 1; }
  tail -1 gpurun_out/c31_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c2 $v', d['value'], d['roofline']['chains_ms_per_batch'], d['roofline']['batch_period_ms'], 'sha', d['stages']['sha(sha_chunk_kernel)']['avg_launch_ms'], 'gmax', d['stages']['gmax(gmax_kernel)']['avg_launch_ms'])"
done
