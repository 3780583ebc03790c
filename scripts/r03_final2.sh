#!/bin/bash
# Round 3 final check after removing the losing SHA / LZ4 variants: smoke(), the full GPU suite,
# the default bench line, config 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
bash scripts/r03_final.sh || exit 1
timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/final_c4.json.log 2>&1 || { tail -20 gpurun_out/final_c4.json.log; exit 1; }
tail -1 gpurun_out/final_c4.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('config4', d['value'], d['roofline']['chains_ms_per_batch'], d['roofline']['batch_period_ms'])"
