#!/bin/bash
# A/B of env-selected kernel variants on the bench workload: ab.sh "ENV=.. ENV2=.." "ENV=.." ...
# Prints the stage table of each variant (first 64 blocks of the config-2 corpus, 3 steps).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
ARGS=${BENCH_ARGS:-"--blocks 128 --steps 3 --warmup 1 --no-cpu"}
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/ab_$i.log 2>&1 || { echo "variant $v failed"; tail -20 gpurun_out/ab_$i.log; exit 1; }
  echo "== $v"
  tail -1 gpurun_out/ab_$i.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('value', d['value'], 'ms/step', d['ms_per_step'])
print('  '.join('%s=%.2f' % (k.split('(')[0], v['ms_per_step']) for k, v in d['stages'].items()))"
done
