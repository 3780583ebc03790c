#!/bin/bash
# Round 6, check 6 (HEAD with the single-wave small chunking kernels; its GPU suite ran in call 31): smoke, the default bench line as the
# driver runs it (twice), each with its sub-lines (config 4, config 5 whole blocks, config 5 packets).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
V=${V:-k6}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_$V.log 2>&1 || { tail -20 gpurun_out/r06_smoke_$V.log; exit 1; }
tail -1 gpurun_out/r06_smoke_$V.log
for run in a b; do
  timeout -k 10 900 python -u bench.py > gpurun_out/r06_bench_${V}$run.json.log 2>&1 || { tail -20 gpurun_out/r06_bench_${V}$run.json.log; exit 1; }
  tail -1 gpurun_out/r06_bench_${V}$run.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d['roofline']
print('bench', d['value'], 'period', r.get('batch_period_ms'), 'frac', r.get('frac'), 'pipe', (r.get('pipeline') or {}).get('frac_of_achievable'), 'oracle', d['dedup'].get('oracle_check', {}).get('store_size_mismatches'))
for k, v in (d.get('configs') or {}).items(): print(k, v.get('value'), v.get('error'))"
done
