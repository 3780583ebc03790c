#!/bin/bash
# Round-3 closing run at HEAD defaults: GPU suite, kernel trace + FETCH/WRITE/VALU traffic of the
# default bench, the default line (with its CPU baseline), config 4 (with CPU baseline) + its kernel
# trace, config 5 (whole blocks, durable drains) and the native 64 KiB packet driver.
# PART=1 (suite + config 2) / PART=2 (configs 4, 5) / unset: both.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-c1}
if [ "${PART:-1}" = 1 ] || [ -z "$PART" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03_tests_$V.log 2>&1 || { tail -30 gpurun_out/r03_tests_$V.log; exit 1; }
tail -1 gpurun_out/r03_tests_$V.log
TAG=r03_prof_$V BENCH="--steps 2 --warmup 1 --no-cpu --no-alone" bash scripts/r02_prof.sh > gpurun_out/r03_prof_$V.txt 2>&1 || { tail -20 gpurun_out/r03_prof_$V.txt; exit 1; }
head -12 gpurun_out/r03_prof_$V.txt | cut -c1-160
TAG=r03_$V EXTRA_GROUPS="SQ_INSTS_VALU" bash scripts/r02_traffic.sh > gpurun_out/r03_traffic_$V.txt 2>&1 || { tail -20 gpurun_out/r03_traffic_$V.txt; exit 1; }
cp gpurun_out/r03_${V}_traffic.json profiles/r03_v${V}_traffic.json   # sorts after r03_v2 (bench takes the newest name)
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_$V.json.log 2>&1 || { tail -20 gpurun_out/r03_bench_$V.json.log; exit 1; }
tail -1 gpurun_out/r03_bench_$V.json.log | cut -c1-300
fi
if [ "${PART:-2}" = 2 ] || [ -z "$PART" ]; then
timeout -k 10 900 python -u bench.py --workload config4 --steps 2 --warmup 1 --cpu-sample-blocks 16 > gpurun_out/r03_c4_$V.json.log 2>&1 || { tail -20 gpurun_out/r03_c4_$V.json.log; exit 1; }
tail -1 gpurun_out/r03_c4_$V.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('config4', d['value'], d['roofline']['chains_ms_per_batch'], d['cpu_baseline']['container_file_mismatches'])"
TAG=r03_c4prof_$V BENCH="--workload config4 --steps 1 --warmup 1 --no-cpu" bash scripts/r02_prof.sh > gpurun_out/r03_c4prof_$V.txt 2>&1 || { tail -20 gpurun_out/r03_c4prof_$V.txt; exit 1; }
head -8 gpurun_out/r03_c4prof_$V.txt | cut -c1-160
timeout -k 10 600 python -u bench.py --workload config5 --steps 2 --warmup 1 --no-cpu > gpurun_out/r03_c5_$V.json.log 2>&1 || { tail -20 gpurun_out/r03_c5_$V.json.log; exit 1; }
tail -1 gpurun_out/r03_c5_$V.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('config5', d['value'], d['pcie'])"
timeout -k 10 900 python -u bench.py --workload config5 --packet-driver cpp --packet-kib 64 --steps 2 > gpurun_out/r03_c5pk64_$V.json.log 2>&1 || { tail -20 gpurun_out/r03_c5pk64_$V.json.log; exit 1; }
tail -1 gpurun_out/r03_c5pk64_$V.json.log | cut -c1-600
fi
