#!/bin/bash
# Re-entry check: GPU suite on the current tree, then config-4 and default bench lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-v3}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$V.log 2>&1 || { tail -30 gpurun_out/tests_$V.log; exit 1; }
tail -2 gpurun_out/tests_$V.log
timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/bench_c4_$V.json.log 2>&1 || { tail -20 gpurun_out/bench_c4_$V.json.log; exit 1; }
tail -1 gpurun_out/bench_c4_$V.json.log | cut -c1-300
