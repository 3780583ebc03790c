#!/bin/bash
# Round 3 last check on the committed tree: the full GPU suite, then the receive-chunk A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/final3_tests.log 2>&1 || { tail -30 gpurun_out/final3_tests.log; exit 1; }
tail -1 gpurun_out/final3_tests.log
bash scripts/r03_call35.sh
