#!/bin/bash
# A/B of env-selected variants: full default bench (config 2, no CPU leg, no alone pass) run in
# the order given (repeat a variant to alternate), then one read/write-request PMC pass per
# distinct variant over a 96-block bench.  Usage: r03_ab.sh "ENV=a" "ENV=b" "ENV=a" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
TAG=${TAG:-ab}
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu --no-alone"}
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/${TAG}_$i.log 2>&1 || { echo "variant $v failed"; tail -20 gpurun_out/${TAG}_$i.log; exit 1; }
  echo "== $v"
  tail -1 gpurun_out/${TAG}_$i.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('value', d['value'], 'ms/step', d['ms_per_step'], 'period', d['roofline']['batch_period_ms'], d['roofline']['chains_ms_per_batch'])
print('  '.join('%s=%.3f' % (k.split('(')[0], v['avg_launch_ms']) for k, v in d['stages'].items()))"
done
[ -n "$NO_PMC" ] && exit 0
export TMPDIR=/tmp
j=0
declare -A seen
for v in "$@"; do
  [ -n "${seen[$v]}" ] && continue
  seen[$v]=1
  j=$((j+1))
  OUT=$R/gpurun_out/pmc_${TAG}_$j; mkdir -p $OUT
  echo "$v" > $OUT/variant.txt
  (cd /tmp && env $v timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/p1 -o run -- python3 $R/bench.py --blocks 96 --steps 1 --warmup 0 --no-cpu --no-alone > $OUT/p1.log 2>&1) || { echo "pmc $v failed"; tail -5 $OUT/p1.log; exit 1; }
  echo "== pmc $v"; python3 scripts/pmc_table.py $OUT | grep -E "kernel|sha_|lane_walk|place|gmax|idx_"
done
