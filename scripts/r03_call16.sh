#!/bin/bash
# Round 3: windowed stitch path (no irregular-boundary cap) + per-workgroup jump ranges: parity
# (chunking-heavy suites, node loopback), config 4; then issue-priority A/B (granule pass, place,
# walk) on config 2.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_config2_shape.py tests/test_bench_shape.py tests/test_node.py tests/test_boundary.py -m gpu > gpurun_out/c16_tests.log 2>&1 || { tail -30 gpurun_out/c16_tests.log; exit 1; }
tail -1 gpurun_out/c16_tests.log
timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/r03_c4_v4.json.log 2>&1 || { tail -20 gpurun_out/r03_c4_v4.json.log; exit 1; }
tail -1 gpurun_out/r03_c4_v4.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('config4', d['value'], d['roofline']['chains_ms_per_batch']); print({k:v['avg_launch_ms'] for k,v in d['stages'].items()})"
NO_PMC=1 TAG=prio2 bash scripts/r03_ab.sh HDRF_SETPRIO=0 HDRF_SETPRIO=16 HDRF_SETPRIO=48 HDRF_SETPRIO=0 HDRF_SETPRIO=17 HDRF_SETPRIO=49 HDRF_SETPRIO=32
