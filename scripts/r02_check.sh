#!/bin/bash
# Round-2 GPU check: chunking parity first (fast fail), then a short bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
T=${TESTS:-tests/test_gpu_parity.py tests/test_config2_shape.py}
timeout -k 10 900 python -u -m pytest $T -x -v --timeout 150 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?
tail -25 gpurun_out/t.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python -u bench.py $BENCH > gpurun_out/b.log 2>&1 || { tail -30 gpurun_out/b.log; exit 1; }
  tail -1 gpurun_out/b.log | cut -c1-1500
fi
