#!/bin/bash
# Round 3, first GPU call: new parity tests (bench batch shape, 64-block batches, packet receive
# cancel/race, lzop fixture), the Infinity-Cache probe, one default bench line with the widened
# chunk-by-chunk CPU check.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 120 ./tools/_build/mall_probe > gpurun_out/mall_probe.txt 2>&1 || { tail -20 gpurun_out/mall_probe.txt; exit 1; }
cat gpurun_out/mall_probe.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_bench_shape.py tests/test_boundary.py tests/test_lzop.py -m gpu > gpurun_out/r03_tests1.log 2>&1 || { tail -40 gpurun_out/r03_tests1.log; exit 1; }
grep -E "passed|failed" gpurun_out/r03_tests1.log | tail -3
timeout -k 10 600 python -u bench.py > gpurun_out/r03_bench_v0.json.log 2>&1 || { tail -20 gpurun_out/r03_bench_v0.json.log; exit 1; }
tail -1 gpurun_out/r03_bench_v0.json.log | cut -c1-400
