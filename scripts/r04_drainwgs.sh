#!/bin/bash
# Round 4: the CU drain's grid sized to the drained bytes (>= 4 workgroups, one per ~320 MiB; default)
# vs one workgroup per item (HDRF_XFER_WGS=0) and fixed 3 / 5: boundary tests, then config 5 whole
# blocks compressor 1 (alternated twice) and compressor 2 (default vs 0).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_boundary.py > gpurun_out/r04_drainwgs_tests.log 2>&1 || { tail -30 gpurun_out/r04_drainwgs_tests.log; exit 1; }
tail -1 gpurun_out/r04_drainwgs_tests.log
i=0
for rep in 1 2; do
for v in "X=rule" "HDRF_XFER_WGS=0" "HDRF_XFER_WGS=3" "HDRF_XFER_WGS=5"; do
  i=$((i+1))
  env $v timeout -k 10 400 python -u bench.py --workload config5 --steps 3 > gpurun_out/r04_drainwgs_$i.json.log 2>&1 || { echo "whole $v failed"; tail -20 gpurun_out/r04_drainwgs_$i.json.log; exit 1; }
  tail -1 gpurun_out/r04_drainwgs_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); print('whole c1 $v', d['value'], d['roofline'].get('batch_period_ms'))"
done
done
for v in "X=rule" "HDRF_XFER_WGS=0" "X=rule" "HDRF_XFER_WGS=0"; do
  i=$((i+1))
  env $v timeout -k 10 400 python -u bench.py --workload config5 --steps 3 --compressor 2 > gpurun_out/r04_drainwgs_$i.json.log 2>&1 || { echo "whole c2 $v failed"; tail -20 gpurun_out/r04_drainwgs_$i.json.log; exit 1; }
  tail -1 gpurun_out/r04_drainwgs_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); print('whole c2 $v', d['value'], d['roofline'].get('batch_period_ms'))"
done
