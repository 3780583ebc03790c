#!/bin/bash
# Round 4: config-5 whole-block timeline after the stream-C fix (kernel + memory-copy trace), then
# the CU drain capped harder (HDRF_XFER_WGS 8 / 16 vs 0 / 32).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/c5trace2 -o run -- python3 $R/bench.py --workload config5 --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/c5trace2.log 2>&1) || { tail -20 gpurun_out/c5trace2.log; exit 1; }
tail -1 gpurun_out/c5trace2.log | cut -c1-120
i=0
for w in 0 16 8 32 0 16 8 32; do
  i=$((i+1))
  HDRF_XFER_WGS=$w timeout -k 10 400 python -u bench.py --workload config5 --steps 3 > gpurun_out/r04_xferab2_$i.json.log 2>&1 || { echo "whole wgs=$w failed"; tail -20 gpurun_out/r04_xferab2_$i.json.log; exit 1; }
  tail -1 gpurun_out/r04_xferab2_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); print('whole wgs=$w', d['value'], d['roofline'].get('batch_period_ms'))"
done
