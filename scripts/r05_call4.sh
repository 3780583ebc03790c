#!/bin/bash
# Round 5 call 4: the whole GPU suite with the sole-chunk index path (default), the index-related
# tests with it off, its A/B, and FETCH/WRITE passes at the new default.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_tests_c.log 2>&1 || { tail -60 gpurun_out/r05_tests_c.log; exit 1; }
tail -1 gpurun_out/r05_tests_c.log
HDRF_SOLE=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_tests_nosole.log 2>&1 || { tail -40 gpurun_out/r05_tests_nosole.log; exit 1; }
tail -1 gpurun_out/r05_tests_nosole.log
TAG=r05_sole bash scripts/abrun.sh scripts/ab_r05_sole.txt || exit 1
ARGS="--steps 1 --warmup 0 --no-cpu --no-alone --no-sub" TAG=r05_c2sole bash scripts/r02_traffic.sh > gpurun_out/r05_c2sole_traffic.log 2>&1 || { tail -20 gpurun_out/r05_c2sole_traffic.log; exit 1; }
python3 - <<'PY'
import json
for t in ("r05_c2sole",):
    d = json.load(open("gpurun_out/%s_traffic.json" % t))
    skip = ("_config", "corpus_kernel", "idx_clear_kernel")
    tot = sum(v["hbm_bytes_per_launch"] for k, v in d.items() if k not in skip)
    print(t, {k: round(v["hbm_bytes_per_launch"] / 1e9, 3) for k, v in d.items() if k not in skip and v["hbm_bytes_per_launch"] > 5e7}, "sum %.2f GB" % (tot / 1e9))
PY
