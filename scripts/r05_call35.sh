#!/bin/bash
# Round 5, call 35: the default bench line with no flags (20 timed steps, 2 warmup, sub-lines and CPU leg), timed end to end
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
s=$(date +%s)
timeout -k 10 600 python -u bench.py > gpurun_out/r05_bench_default20.json.log 2>&1 || { tail -20 gpurun_out/r05_bench_default20.json.log; exit 1; }
echo "wall $(( $(date +%s) - s )) s"
tail -1 gpurun_out/r05_bench_default20.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d['roofline']
print('bench', d['value'], 'steps', d['steps'], 'warmup', d['warmup'], 'period', r.get('batch_period_ms'), 'frac', r.get('frac'), ' '.join('%s=%s' % (k, v.get('value')) for k, v in (d.get('configs') or {}).items()))"
