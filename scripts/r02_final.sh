#!/bin/bash
# Round-2 closing measurements: full GPU suite, default bench (config 2) with CPU baseline, rocprof
# kernel stats, PMC traffic + SHA VALU, bench again carrying the counters, config 4 and 5 lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
V=${V:-v2}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
  tail -2 gpurun_out/final_tests.log
fi
TAG=prof_$V BENCH="--steps 2 --warmup 1 --no-cpu" bash scripts/r02_prof.sh > gpurun_out/prof_$V.txt 2>&1 || { tail -20 gpurun_out/prof_$V.txt; exit 1; }
head -8 gpurun_out/prof_$V.txt
TAG=r02_$V EXTRA_GROUPS="SQ_INSTS_VALU" bash scripts/r02_traffic.sh > gpurun_out/traffic_$V.txt 2>&1 || { tail -20 gpurun_out/traffic_$V.txt; exit 1; }
cp gpurun_out/r02_${V}_traffic.json profiles/r02_${V}_traffic.json
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$V.json.log 2>&1 || { tail -20 gpurun_out/bench_$V.json.log; exit 1; }
tail -1 gpurun_out/bench_$V.json.log | cut -c1-300
timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_c4_$V.json.log 2>&1 || { tail -20 gpurun_out/bench_c4_$V.json.log; exit 1; }
tail -1 gpurun_out/bench_c4_$V.json.log | cut -c1-200
timeout -k 10 600 python -u bench.py --workload config5 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_c5_$V.json.log 2>&1 || { tail -20 gpurun_out/bench_c5_$V.json.log; exit 1; }
tail -1 gpurun_out/bench_c5_$V.json.log | cut -c1-200
