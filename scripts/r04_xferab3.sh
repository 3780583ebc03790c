#!/bin/bash
# Round 4: the CU drain capped to a few workgroups (HDRF_XFER_WGS 2 / 4 / 6 vs 0): a drain at about
# the rate the batch period needs (~27 GB/s) instead of ~50 GB/s, so the H2D copies keep more of the link.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
i=0
for w in 0 4 6 2 0 4 6 2; do
  i=$((i+1))
  HDRF_XFER_WGS=$w timeout -k 10 400 python -u bench.py --workload config5 --steps 3 > gpurun_out/r04_xferab3_$i.json.log 2>&1 || { echo "whole wgs=$w failed"; tail -20 gpurun_out/r04_xferab3_$i.json.log; exit 1; }
  tail -1 gpurun_out/r04_xferab3_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); print('whole wgs=$w', d['value'], d['roofline'].get('batch_period_ms'), d['pcie'].get('d2h_GB_s_drain'))"
done
