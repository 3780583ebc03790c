#!/bin/bash
# Round 5, first call: the new GPU tests (dirty slack, the JNI binding executed, packet driver at the
# bench shape), smoke, then the default bench line (config 2 + the config-4 / config-5 sub-lines).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-a}
timeout -k 10 900 python -u -m pytest tests/test_slack.py tests/test_jni.py tests/test_packet_driver.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_newtests_$V.log 2>&1 || { tail -60 gpurun_out/r05_newtests_$V.log; exit 1; }
tail -3 gpurun_out/r05_newtests_$V.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_$V.log 2>&1 || { tail -20 gpurun_out/r05_smoke_$V.log; exit 1; }
tail -1 gpurun_out/r05_smoke_$V.log
timeout -k 10 900 python -u bench.py > gpurun_out/r05_bench_$V.json.log 2>&1 || { tail -30 gpurun_out/r05_bench_$V.json.log; exit 1; }
tail -1 gpurun_out/r05_bench_$V.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d.get('roofline') or {}
print('c2', d['value'], 'period', r.get('batch_period_ms'), 'frac', r.get('frac'))
for k, v in (d.get('configs') or {}).items():
    print(k, v.get('value'), v.get('error', ''), (v.get('cpu_baseline') or {}).get('container_file_mismatches'), v.get('wall_s'))"
