#!/bin/bash
# Round 3: the config-2 line falls into two modes per process (~1005 / ~1037 GB/s) with the same
# kernel interleaving, every kernel ~4 % slower in the slow mode.  Does the corpus address decide?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
i=0
for p in 0 0 2 2 6 6 64 64 0 2; do
  i=$((i+1))
  HDRF_BENCH_PAD_MB=$p timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-alone > gpurun_out/c34_$i.json.log 2> gpurun_out/c34_$i.err || { echo "bench failed"; tail -20 gpurun_out/c34_$i.err; exit 1; }
  a=$(grep "corpus at" gpurun_out/c34_$i.err)
  tail -1 gpurun_out/c34_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== pad $p', d['value'], d['roofline']['batch_period_ms'], '$a')"
done
