#!/bin/bash
# Round 5 call 3: sha_line parity (the SHA tests with HDRF_SHA_LINE=1), its A/B under the primed
# steps, and FETCH/WRITE passes of both SHA variants (one counter per rocprofv3 run).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
HDRF_SHA_LINE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_shape.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_line_tests.log 2>&1 || { tail -40 gpurun_out/r05_line_tests.log; exit 1; }
tail -1 gpurun_out/r05_line_tests.log
TAG=r05_line bash scripts/abrun.sh scripts/ab_r05_line.txt || exit 1
ARGS="--steps 1 --warmup 0 --no-cpu --no-alone --no-sub" TAG=r05_c2 bash scripts/r02_traffic.sh > gpurun_out/r05_c2_traffic.log 2>&1 || { tail -20 gpurun_out/r05_c2_traffic.log; exit 1; }
HDRF_SHA_LINE=1 ARGS="--steps 1 --warmup 0 --no-cpu --no-alone --no-sub" TAG=r05_c2line bash scripts/r02_traffic.sh > gpurun_out/r05_c2line_traffic.log 2>&1 || { tail -20 gpurun_out/r05_c2line_traffic.log; exit 1; }
python3 - <<'PY'
import json
for t in ("r05_c2", "r05_c2line"):
    d = json.load(open("gpurun_out/%s_traffic.json" % t))
    tot = sum(v["hbm_bytes_per_launch"] for k, v in d.items() if k != "_config")
    print(t, {k: round(v["hbm_bytes_per_launch"] / 1e9, 3) for k, v in d.items() if k != "_config" and v["hbm_bytes_per_launch"] > 5e7}, "sum %.2f GB" % (tot / 1e9))
PY
