#!/bin/bash
# LZ4 change check: byte parity (all LZ4 GPU tests), phase profile, aggregate scaling
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_lz4.py tests/test_gpu_parity.py tests/test_config2_shape.py -m gpu -x -q --timeout 300 --timeout-method thread -k "lz4 or config4 or compression or corpus or stream" > gpurun_out/tests_lzw.log 2>&1 || { tail -30 gpurun_out/tests_lzw.log; exit 1; }
tail -2 gpurun_out/tests_lzw.log
bash scripts/r02_lzp.sh || exit 1
LZS_MIB=64,2048 bash scripts/r02_lzs.sh
