#!/bin/bash
# Round 5: config 5 whole blocks with primed steps (hdrf_reset_async on durable-container contexts).
# Parity first (reset_async + durable drain tests), then primed vs --no-prime, c2 and c1, alternating.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_reset_async.py tests/test_boundary.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_c5prime_tests.log 2>&1 || { tail -40 gpurun_out/r05_c5prime_tests.log; exit 1; }
tail -1 gpurun_out/r05_c5prime_tests.log
for rep in 1 2; do
  for cmp in 2 1; do
    for v in prime noprime; do
      X=""; [ $v = noprime ] && X="--no-prime"
      f=gpurun_out/r05_c5prime_${v}_c${cmp}_$rep.json.log
      timeout -k 10 600 python -u bench.py --workload config5 --compressor $cmp --steps 3 --warmup 1 --no-cpu $X > $f 2>&1 || { tail -20 $f; exit 1; }
      tail -1 $f | python3 -c "
import json,sys
d=json.load(sys.stdin); p=d.get('pcie') or {}
print('$v c$cmp rep $rep', d['value'], 'ms/step', d['ms_per_step'], 'v/bidir', p.get('value_over_bidirectional_raw'), 'primed', d['config'].get('steps_back_to_back'))"
    done
  done
done
