#!/bin/bash
# Round 3: config 4 (SHA stream 87 % busy beside the LZ4 passes): SHA issue priority, LZ4 waves per CU,
# dual-chain SHA.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
i=0
for v in "HDRF_SETPRIO=0" "HDRF_SETPRIO=12" "HDRF_LZ4_WAVES=14" "HDRF_SHA_DUAL=1"; do
  i=$((i+1))
  env $v timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/c18_$i.json.log 2>&1 || { echo "variant $v failed"; tail -20 gpurun_out/c18_$i.json.log; exit 1; }
  tail -1 gpurun_out/c18_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== $v', d['value'], d['roofline']['chains_ms_per_batch'])
print('  '.join('%s=%.1f' % (k.split('(')[0], v['avg_launch_ms']) for k, v in d['stages'].items()))"
done
