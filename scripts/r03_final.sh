#!/bin/bash
# Round 3 final check on the committed defaults: smoke(), the full GPU suite, the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/final_bench.json.log 2>&1 || { tail -20 gpurun_out/final_bench.json.log; exit 1; }
tail -1 gpurun_out/final_bench.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d['roofline']
print('config2', d['value'], r['kernel'], r['achieved'], r['frac'], r['traffic'], r['traffic_source'], r['critical_path'], r['chains_ms_per_batch'], r['batch_period_ms'])"
