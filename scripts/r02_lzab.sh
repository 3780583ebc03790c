#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lz4.py tests/test_gpu_parity.py tests/test_config2_shape.py tests/test_boundary.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lz4 or config4 or compression or corpus or stream or durable or drain" > gpurun_out/tests_lzab.log 2>&1 || { tail -30 gpurun_out/tests_lzab.log; exit 1; }
tail -1 gpurun_out/tests_lzab.log
VARIANTS=${VARIANTS:-scripts/ab_lzw.txt} bash scripts/r02_ab.sh
