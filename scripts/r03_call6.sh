#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload config5 --steps 2 --warmup 1 --no-cpu > gpurun_out/r03_c5_v1.json.log 2>&1 || { tail -20 gpurun_out/r03_c5_v1.json.log; exit 1; }
tail -1 gpurun_out/r03_c5_v1.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('config5', d['value'], d['pcie'])"
timeout -k 10 900 python -u bench.py --workload config5 --packet-driver cpp --packet-kib 64 --steps 2 > gpurun_out/r03_c5_pk64_v1.json.log 2>&1 || { tail -20 gpurun_out/r03_c5_pk64_v1.json.log; exit 1; }
tail -1 gpurun_out/r03_c5_pk64_v1.json.log | cut -c1-900
