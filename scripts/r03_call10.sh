#!/bin/bash
# Round 3 (re-entry) baseline at HEAD: full GPU suite, kernel trace + FETCH/WRITE/VALU traffic of
# the default bench, the default bench line (with CPU baseline), then a SHA ring A/B.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-v1}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03_tests_$V.log 2>&1 || { tail -30 gpurun_out/r03_tests_$V.log; exit 1; }
tail -1 gpurun_out/r03_tests_$V.log
TAG=r03_prof_$V BENCH="--steps 2 --warmup 1 --no-cpu --no-alone" bash scripts/r02_prof.sh > gpurun_out/r03_prof_$V.txt 2>&1 || { tail -20 gpurun_out/r03_prof_$V.txt; exit 1; }
head -12 gpurun_out/r03_prof_$V.txt | cut -c1-160
TAG=r03_$V EXTRA_GROUPS="SQ_INSTS_VALU" bash scripts/r02_traffic.sh > gpurun_out/r03_traffic_$V.txt 2>&1 || { tail -20 gpurun_out/r03_traffic_$V.txt; exit 1; }
cp gpurun_out/r03_${V}_traffic.json profiles/r03_${V}_traffic.json
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_$V.json.log 2>&1 || { tail -20 gpurun_out/r03_bench_$V.json.log; exit 1; }
tail -1 gpurun_out/r03_bench_$V.json.log | cut -c1-300
NO_PMC=1 TAG=ring bash scripts/r03_ab.sh HDRF_SHA_RING=1 HDRF_SHA_RING=0 HDRF_SHA_RING=1 HDRF_SHA_RING=0
