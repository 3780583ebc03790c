#!/bin/bash
# LZ4 off stream B: parity of the compressor-2 tests, then config-4 bench at depth 2 and 3.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-ov1}
timeout -k 10 600 python -u -m pytest tests/test_config2_shape.py tests/test_lz4.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lz4 or config4 or compression or corpus" > gpurun_out/tests_$V.log 2>&1 || { tail -30 gpurun_out/tests_$V.log; exit 1; }
tail -2 gpurun_out/tests_$V.log
for d in ${DEPTHS:-2 3}; do
timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu --depth $d > gpurun_out/bench_c4_${V}_d$d.json.log 2>&1 || { tail -20 gpurun_out/bench_c4_${V}_d$d.json.log; exit 1; }
tail -1 gpurun_out/bench_c4_${V}_d$d.json.log | cut -c1-200
done
