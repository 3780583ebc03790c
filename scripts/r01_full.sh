#!/bin/bash
# Full GPU check: parity suite, smoke, default bench (config 2), config 4 bench.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/pytest_gpu.log | head -30; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
timeout -k 10 600 python -u bench.py --workload config4 > gpurun_out/bench_c4.log 2>&1 || { echo "bench c4 failed"; tail -30 gpurun_out/bench_c4.log; exit 1; }
tail -1 gpurun_out/bench_c4.log | cut -c1-400
echo ALLDONE
