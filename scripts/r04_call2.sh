#!/bin/bash
# Round 4: index epochs (reset = epoch bump, no 8.6 GB clear) — GPU suite, then the default bench.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-c2}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_tests_$V.log 2>&1 || { tail -40 gpurun_out/r04_tests_$V.log; exit 1; }
tail -1 gpurun_out/r04_tests_$V.log
timeout -k 10 600 python -u bench.py --no-cpu > gpurun_out/r04_bench_$V.json.log 2>&1 || { tail -20 gpurun_out/r04_bench_$V.json.log; exit 1; }
tail -1 gpurun_out/r04_bench_$V.json.log | cut -c1-300
timeout -k 10 600 python -u bench.py --no-cpu > gpurun_out/r04_bench_${V}b.json.log 2>&1 || { tail -20 gpurun_out/r04_bench_${V}b.json.log; exit 1; }
tail -1 gpurun_out/r04_bench_${V}b.json.log | cut -c1-300
