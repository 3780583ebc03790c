#!/bin/bash
# Round 6, call 2: the advisor fixes' tests (reset_async refusal/restore, gx reads), the JNI shim, the
# primed bench-shape test, then the default bench line with the whole-corpus storeSize check.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
V=${V:-c2}
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_reset_async.py tests/test_jni.py tests/test_node.py "tests/test_bench_shape.py::test_bench_primed_depth4_reset_async_generations" \
  > gpurun_out/r06_tests_$V.log 2>&1 || { tail -40 gpurun_out/r06_tests_$V.log; exit 1; }
tail -1 gpurun_out/r06_tests_$V.log
timeout -k 10 900 python -u bench.py > gpurun_out/r06_bench_$V.json.log 2>&1 || { tail -20 gpurun_out/r06_bench_$V.json.log; exit 1; }
tail -1 gpurun_out/r06_bench_$V.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d['roofline']
print('bench', d['value'], 'period', r.get('batch_period_ms'), 'frac', r.get('frac'), 'sha.valu', r['sha'].get('valu'))
print('oracle_check', d['dedup'].get('oracle_check'))
for k, v in (d.get('configs') or {}).items(): print(k, v.get('value'), (v.get('dedup') or {}).get('oracle_check'), v.get('error'))"
