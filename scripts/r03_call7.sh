#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_boundary.py tests/test_packet_driver.py -m gpu > gpurun_out/c7_tests.log 2>&1 || { tail -30 gpurun_out/c7_tests.log; exit 1; }
tail -1 gpurun_out/c7_tests.log
for v in "" "HDRF_DRAIN_KERNEL=0" "NODRAIN"; do
  if [ "$v" = "NODRAIN" ]; then A="--no-drain"; E=""; else A=""; E="$v"; fi
  env $E timeout -k 10 600 python -u bench.py --workload config5 --steps 2 --warmup 1 --no-cpu $A > gpurun_out/r03_c5_$v.json.log 2>&1 || { tail -20 gpurun_out/r03_c5_$v.json.log; exit 1; }
  tail -1 gpurun_out/r03_c5_$v.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); p=d['pcie']; print('config5 [$v]', d['value'], p['h2d_GB_s_raw_copy'], p['value_over_raw_copy'], p['d2h_GB_s_drain'], p['drained_container_bytes_per_step'])"
done
for v in "" "HDRF_DRIVER_NODRAIN=1"; do
  env $v timeout -k 10 900 python -u bench.py --workload config5 --packet-driver cpp --packet-kib 64 --steps 2 > gpurun_out/r03_c5_pk64_$v.json.log 2>&1 || { tail -20 gpurun_out/r03_c5_pk64_$v.json.log; exit 1; }
  tail -1 gpurun_out/r03_c5_pk64_$v.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('packets64 [$v]', d['value'], d['packet_driver'])"
done
