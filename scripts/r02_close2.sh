#!/bin/bash
# Round-2 closing run, part 2: config 4 (line + kernel trace) and config 5 lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-v3}
timeout -k 10 400 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_c4_$V.json.log 2>&1 || { tail -20 gpurun_out/bench_c4_$V.json.log; exit 1; }
tail -1 gpurun_out/bench_c4_$V.json.log | cut -c1-200
TAG=c4prof_$V BENCH="--workload config4 --steps 1 --warmup 1 --no-cpu" bash scripts/r02_prof.sh > gpurun_out/c4prof_$V.txt 2>&1 || { tail -20 gpurun_out/c4prof_$V.txt; exit 1; }
head -8 gpurun_out/c4prof_$V.txt | cut -c1-160
timeout -k 10 400 python -u bench.py --workload config5 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_c5_$V.json.log 2>&1 || { tail -20 gpurun_out/bench_c5_$V.json.log; exit 1; }
tail -1 gpurun_out/bench_c5_$V.json.log | cut -c1-200
