#!/bin/bash
# Round 3: kernel traces of four default config-2 runs (the batch period shows two modes, ~4.13 and
# ~4.27 ms): which kernels co-run in each mode.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c33_$i -o run -- python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-alone > gpurun_out/c33_$i.log 2>&1 || { tail -20 gpurun_out/c33_$i.log; exit 1; }
  tail -1 gpurun_out/c33_$i.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== run $i', d['value'], d['roofline']['chains_ms_per_batch'], d['roofline']['batch_period_ms'])"
done
