#!/bin/bash
# Round 3: sha_line (each 128-B line fetched once, window cut out of two register-held lines by a
# barrel shift): parity under HDRF_SHA_LINE=1, then A/B against sha_chunk with a request-count pass.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
HDRF_SHA_LINE=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_config2_shape.py tests/test_bench_shape.py -m gpu > gpurun_out/c15_tests.log 2>&1 || { tail -30 gpurun_out/c15_tests.log; exit 1; }
tail -1 gpurun_out/c15_tests.log
TAG=line bash scripts/r03_ab.sh HDRF_SHA_LINE=1 HDRF_SHA_LINE=0 HDRF_SHA_LINE=1 HDRF_SHA_LINE=0 "HDRF_SHA_LINE=1 HDRF_SHA_WPC=6" "HDRF_SHA_LINE=1 HDRF_SHA_WPC=12"
HDRF_LIB_PATH=$(pwd)/hdrf_amd/_build_dbg/libhdrf.so timeout -k 10 300 python -u scripts/c4_fallback_dbg.py > gpurun_out/c4_fallback_dbg.log 2>&1 || { tail -20 gpurun_out/c4_fallback_dbg.log; exit 1; }
grep -c "give-up" gpurun_out/c4_fallback_dbg.log; grep -c "fallback:" gpurun_out/c4_fallback_dbg.log; grep -E "fallback:|stages" gpurun_out/c4_fallback_dbg.log | head -20; grep "give-up" gpurun_out/c4_fallback_dbg.log | head -10
timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/r03_c4_v3.json.log 2>&1 || { tail -20 gpurun_out/r03_c4_v3.json.log; exit 1; }
tail -1 gpurun_out/r03_c4_v3.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('config4', d['value'], d['roofline']['chains_ms_per_batch']); print({k:v['avg_launch_ms'] for k,v in d['stages'].items()})"
HDRF_SETPRIO=7 timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/r03_c4_v3p.json.log 2>&1 || { tail -20 gpurun_out/r03_c4_v3p.json.log; exit 1; }
tail -1 gpurun_out/r03_c4_v3p.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('config4 prio7', d['value'], d['roofline']['chains_ms_per_batch']); print({k:v['avg_launch_ms'] for k,v in d['stages'].items()})"
NO_PMC=1 TAG=prio bash scripts/r03_ab.sh HDRF_SETPRIO=0 HDRF_SETPRIO=3 HDRF_SETPRIO=7 HDRF_SETPRIO=15 HDRF_SETPRIO=3
