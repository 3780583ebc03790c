#!/bin/bash
# Round 4: cap the CU drain's write rate (HDRF_XFER_WGS workgroups looping over the drain items)
# so the next blocks' H2D copies keep more of the link: boundary tests with a capped grid, then
# config 5 whole blocks (compressor 1) with 0 (one workgroup per item) / 32 / 64 / 128 / 256.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
HDRF_XFER_WGS=32 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_boundary.py > gpurun_out/r04_xferab_tests.log 2>&1 || { tail -30 gpurun_out/r04_xferab_tests.log; exit 1; }
tail -1 gpurun_out/r04_xferab_tests.log
i=0
for rep in 1 2; do
for w in 0 32 64 128 256; do
  i=$((i+1))
  HDRF_XFER_WGS=$w timeout -k 10 400 python -u bench.py --workload config5 --steps 3 > gpurun_out/r04_xferab_$i.json.log 2>&1 || { echo "whole wgs=$w failed"; tail -20 gpurun_out/r04_xferab_$i.json.log; exit 1; }
  tail -1 gpurun_out/r04_xferab_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); print('whole wgs=$w', d['value'], d['roofline'].get('batch_period_ms'))"
done
done
