#!/bin/bash
# LZOP (compressor 3) GPU parity + the other stream codecs sharing the planner
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 170 python -u -m pytest tests/test_lzop.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/tests_lzop.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|Timeout" gpurun_out/tests_lzop.log | tail -20
[ $rc -ne 0 ] && { tail -40 gpurun_out/tests_lzop.log; exit $rc; }
timeout -k 10 400 python -u -m pytest tests/test_lz4.py tests/test_snappy.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_lzop2.log 2>&1; rc=$?
tail -2 gpurun_out/tests_lzop2.log
exit $rc
