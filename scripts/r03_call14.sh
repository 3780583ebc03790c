#!/bin/bash
# Round 3: SHA lane count vs its line re-fetches.  A lane's window shares a 64-B sector with the
# next iteration's; whether that sector is still in L2 depends on how many lanes stream at once.
# Bench A/B then one read/write-request PMC pass per variant.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=wpc bash scripts/r03_ab.sh HDRF_SHA_WPC=8 HDRF_SHA_WPC=4 HDRF_SHA_WPC=6 HDRF_SHA_WPC=4 HDRF_SHA_WPC=8 "HDRF_SHA_RING=1 HDRF_SHA_WPC=4"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_config2_shape.py -m gpu > gpurun_out/c14_tests.log 2>&1 || { tail -30 gpurun_out/c14_tests.log; exit 1; }
tail -1 gpurun_out/c14_tests.log
timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/r03_c4_v2.json.log 2>&1 || { tail -20 gpurun_out/r03_c4_v2.json.log; exit 1; }
tail -1 gpurun_out/r03_c4_v2.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('config4', d['value'], d['roofline']['chains_ms_per_batch']); print({k:v['avg_launch_ms'] for k,v in d['stages'].items()})"
