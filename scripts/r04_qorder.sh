#!/bin/bash
# Round 4: the recipe stream R created after the LZ4 streams (hardware queues follow creation order):
# config 4 and config 2 twice each, config 5 whole blocks once.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
run() {
  local tag=$1; shift
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/r04_qorder_$tag.json.log 2>&1 || { echo "$tag failed"; tail -20 gpurun_out/r04_qorder_$tag.json.log; exit 1; }
  tail -1 gpurun_out/r04_qorder_$tag.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d.get('roofline') or {}
print('$tag', d['value'], 'period', r.get('batch_period_ms'), r.get('chains_ms_per_batch'))"
}
run c4a --workload config4 --no-cpu
run c2a --no-cpu
run c4b --workload config4 --no-cpu
run c2b --no-cpu
run c5w --workload config5 --steps 3
