#!/bin/bash
# Round 3 iteration check: GPU parity tests (selected files, or the whole suite with ALL=1), then
# the default bench line and one request-count PMC pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
TAG=${TAG:-chk}
FILES=${FILES:-"tests/test_bench_shape.py tests/test_gpu_parity.py tests/test_config2_shape.py"}
[ -n "$ALL" ] && FILES=tests
timeout -k 10 1100 python -u -m pytest -x -q --timeout 600 --timeout-method thread $FILES -m gpu > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---no-cpu --no-alone} > gpurun_out/${TAG}_bench.json.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.json.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('value', d['value'], 'ms/step', d['ms_per_step'], 'period', d['roofline']['batch_period_ms'], d['roofline']['chains_ms_per_batch'])
print('  '.join('%s=%.3f' % (k.split('(')[0], v['avg_launch_ms']) for k, v in d['stages'].items()))"
[ -n "$NO_PMC" ] && exit 0
export TMPDIR=/tmp
OUT=$R/gpurun_out/pmc_${TAG}; mkdir -p $OUT
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/p1 -o run -- python3 $R/bench.py --blocks 96 --steps 1 --warmup 0 --no-cpu --no-alone > $OUT/p1.log 2>&1) || { echo "pmc failed"; tail -5 $OUT/p1.log; exit 1; }
python3 scripts/pmc_table.py $OUT | grep -vE "rocclr|corpus|clear"
