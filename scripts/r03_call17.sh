#!/bin/bash
# Round 3: sha_dual (two interleaved chains per lane, 4 waves per CU): parity under HDRF_SHA_DUAL=1
# (SHA-1 and SHA-224 suites, bench shape), then A/B on config 2 (+ with sha_line-free default).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
HDRF_SHA_DUAL=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_config2_shape.py tests/test_bench_shape.py -m gpu > gpurun_out/c17_tests.log 2>&1 || { tail -30 gpurun_out/c17_tests.log; exit 1; }
tail -1 gpurun_out/c17_tests.log
TAG=dual bash scripts/r03_ab.sh HDRF_SHA_DUAL=1 HDRF_SHA_DUAL=0 HDRF_SHA_DUAL=1 HDRF_SHA_DUAL=0 "HDRF_SHA_DUAL=1 HDRF_SHA_WPC=6" "HDRF_SHA_DUAL=1 HDRF_SHA_WPC=5" "HDRF_SHA_DUAL=1 HDRF_SETPRIO=8"
HDRF_SHA_DUAL=1 timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/r03_c4_dual.json.log 2>&1 || { tail -20 gpurun_out/r03_c4_dual.json.log; exit 1; }
tail -1 gpurun_out/r03_c4_dual.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('config4 dual', d['value'], d['roofline']['chains_ms_per_batch']); print({k:v['avg_launch_ms'] for k,v in d['stages'].items()})"
