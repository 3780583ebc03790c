#!/bin/bash
# Round-2 closing run, part 1: full GPU suite, kernel trace + PMC traffic of the default bench,
# the default bench line (with CPU baseline) carrying those counters.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-v3}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_tests_$V.log 2>&1 || { tail -30 gpurun_out/final_tests_$V.log; exit 1; }
tail -1 gpurun_out/final_tests_$V.log
TAG=prof_$V BENCH="--steps 2 --warmup 1 --no-cpu --no-alone" bash scripts/r02_prof.sh > gpurun_out/prof_$V.txt 2>&1 || { tail -20 gpurun_out/prof_$V.txt; exit 1; }
head -6 gpurun_out/prof_$V.txt | cut -c1-160
TAG=r02_$V EXTRA_GROUPS="SQ_INSTS_VALU" bash scripts/r02_traffic.sh > gpurun_out/traffic_$V.txt 2>&1 || { tail -20 gpurun_out/traffic_$V.txt; exit 1; }
cp gpurun_out/r02_${V}_traffic.json profiles/r02_${V}_traffic.json
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$V.json.log 2>&1 || { tail -20 gpurun_out/bench_$V.json.log; exit 1; }
tail -1 gpurun_out/bench_$V.json.log | cut -c1-200
