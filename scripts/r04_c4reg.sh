#!/bin/bash
# Round 4: config 4 fell from 40.4 (closing run f) to 32.9-34.2 GB/s after the config-5 changes.
# A/B on one box: HEAD, the closing-run build (3d0fb1a, hdrf_amd/_build_f) and HEAD with the recipe
# copies back on stream C (hdrf_amd/_build_rc), alternated twice.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
i=0
for rep in 1 2; do
for v in "X=head" "HDRF_LIB_PATH=hdrf_amd/_build_f/libhdrf.so" "HDRF_LIB_PATH=hdrf_amd/_build_rc/libhdrf.so"; do
  i=$((i+1))
  env $v timeout -k 10 600 python -u bench.py --workload config4 --no-cpu > gpurun_out/r04_c4reg_$i.json.log 2>&1 || { echo "c4 $v failed"; tail -20 gpurun_out/r04_c4reg_$i.json.log; exit 1; }
  tail -1 gpurun_out/r04_c4reg_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d.get('roofline') or {}
print('c4 $v', d['value'], 'period', r.get('batch_period_ms'), r.get('chains_ms_per_batch'))"
done
done
