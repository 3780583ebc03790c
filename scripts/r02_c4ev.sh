#!/bin/bash
# GPU suite, then config-4 evidence: bench line, rocprof kernel stats, one SQ counter pass.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
mkdir -p gpurun_out
V=${V:-v3}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$V.log 2>&1 || { tail -30 gpurun_out/tests_$V.log; exit 1; }
tail -2 gpurun_out/tests_$V.log
timeout -k 10 300 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_c4_$V.json.log 2>&1 || { tail -20 gpurun_out/bench_c4_$V.json.log; exit 1; }
tail -1 gpurun_out/bench_c4_$V.json.log | cut -c1-200
TAG=c4prof_$V BENCH="--workload config4 --steps 1 --warmup 1 --no-cpu" bash scripts/r02_prof.sh > gpurun_out/c4prof_$V.txt 2>&1 || { tail -20 gpurun_out/c4prof_$V.txt; exit 1; }
head -12 gpurun_out/c4prof_$V.txt
TAG=c4_$V bash scripts/r02_pmc_c4.sh > gpurun_out/c4pmc_$V.txt 2>&1 || { tail -20 gpurun_out/c4pmc_$V.txt; exit 1; }
grep lz4 gpurun_out/c4pmc_$V.txt | cut -c1-300
