#!/bin/bash
# Round 3: full GPU suite on the LZ4-trim build, then config 4 with the LZ4 pass at raised wave
# priority (HDRF_SETPRIO=64) against the default; the 95-VGPR LZ4 pass alone (HDRF_VCAP=1) at 16 and
# 17 waves per CU (LDS allows 17 with the 9 KiB table, 101 VGPRs only 16).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c25_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c25_tests.log; exit 1; }
tail -1 gpurun_out/c25_tests.log
i=0
for v in "HDRF_SETPRIO=64" "HDRF_SETPRIO=0" "HDRF_VCAP=1 HDRF_LZ4_WAVES=17" "HDRF_SETPRIO=64" "HDRF_SETPRIO=0" "HDRF_VCAP=1 HDRF_LZ4_WAVES=17" "HDRF_VCAP=1"; do
  i=$((i+1))
  env $v timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/c25_$i.json.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/c25_$i.json.log; exit 1; }
  tail -1 gpurun_out/c25_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c4 $v', d['value'], d['roofline']['chains_ms_per_batch'], d['roofline']['batch_period_ms'])"
done
# config 5, 64 KiB packets from 4 native receiver threads: completer thread (default) vs the serial
# driver loop (HDRF_DRIVER_SERIAL=1)
for v in "HDRF_DRIVER_X=0" "HDRF_DRIVER_SERIAL=1" "HDRF_DRIVER_X=0"; do
  i=$((i+1))
  env $v timeout -k 10 400 python -u bench.py --workload config5 --packet-kib 64 --packet-threads 4 --packet-driver cpp --steps 2 --warmup 1 --no-cpu > gpurun_out/c25_$i.json.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/c25_$i.json.log; exit 1; }
  tail -1 gpurun_out/c25_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c5 pk64 $v', d['value'], d['packet_driver']['best_GB_s'])"
done
