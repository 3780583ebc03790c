#!/bin/bash
# Round 3: receive staging chunk size (HDRF_RX_CHUNK_MB: 4 default, 16, 1) for 64 KiB packets from 4
# native receiver threads; packet-path tests under 16.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
HDRF_RX_CHUNK_MB=16 timeout -k 10 400 python -u -m pytest tests/test_boundary.py tests/test_packet_driver.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c35_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c35_tests.log; exit 1; }
tail -1 gpurun_out/c35_tests.log
i=0
for v in 16 4 1 16 4 1; do
  i=$((i+1))
  HDRF_RX_CHUNK_MB=$v timeout -k 10 400 python -u bench.py --workload config5 --packet-kib 64 --packet-threads 4 --packet-driver cpp --steps 2 --warmup 1 --no-cpu > gpurun_out/c35_$i.json.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/c35_$i.json.log; exit 1; }
  grep '^{"metric"' gpurun_out/c35_$i.json.log | tail -1 | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== pk64 chunk $v MiB', d['value'], d['packet_driver']['best_GB_s'])"
done
