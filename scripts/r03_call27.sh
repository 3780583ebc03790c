#!/bin/bash
# Round 3: 16 receive buffers.  Packet-path GPU tests, then config 5 64 KiB packets from 4 and 8
# native receiver threads (two runs each).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_boundary.py tests/test_packet_driver.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c27_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c27_tests.log; exit 1; }
tail -1 gpurun_out/c27_tests.log
i=0
for t in 8 4 8 4; do
  i=$((i+1))
  timeout -k 10 400 python -u bench.py --workload config5 --packet-kib 64 --packet-threads $t --packet-driver cpp --steps 2 --warmup 1 --no-cpu > gpurun_out/c27_$i.json.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/c27_$i.json.log; exit 1; }
  tail -1 gpurun_out/c27_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c5 pk64 threads $t', d['value'], d['packet_driver']['best_GB_s'], d['driver_wall_s'])"
done
