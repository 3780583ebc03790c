#!/bin/bash
# Round 4: GPU suite at HEAD (packet driver full-state parity, submit_slots), config-2 evidence
# (kernel trace + FETCH/WRITE/VALU traffic), then the default bench line reading it.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-c3}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_tests_$V.log 2>&1 || { tail -40 gpurun_out/r04_tests_$V.log; exit 1; }
tail -1 gpurun_out/r04_tests_$V.log
TAG=r04_prof_$V BENCH="--steps 2 --warmup 1 --no-cpu --no-alone" bash scripts/r02_prof.sh > gpurun_out/r04_prof_$V.txt 2>&1 || { tail -20 gpurun_out/r04_prof_$V.txt; exit 1; }
head -14 gpurun_out/r04_prof_$V.txt | cut -c1-160
TAG=r04_$V EXTRA_GROUPS="SQ_INSTS_VALU" bash scripts/r02_traffic.sh > gpurun_out/r04_traffic_$V.txt 2>&1 || { tail -20 gpurun_out/r04_traffic_$V.txt; exit 1; }
mkdir -p profiles && cp gpurun_out/r04_${V}_traffic.json profiles/r04_${V}_traffic.json
timeout -k 10 600 python -u bench.py > gpurun_out/r04_bench_$V.json.log 2>&1 || { tail -20 gpurun_out/r04_bench_$V.json.log; exit 1; }
tail -1 gpurun_out/r04_bench_$V.json.log | cut -c1-400
