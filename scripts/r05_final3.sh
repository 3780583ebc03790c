#!/bin/bash
# Round 5 final check on the committed tree: GPU suite, smoke, the default bench line as the driver runs it
# (no flags: N=1, default steps), and the 2-rank same-device rehearsal of the node-global path (gloo, one
# GPU; not a measurement: its per-rank chains and front period are reported)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-final_c}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_tests_$V.log 2>&1 || { tail -40 gpurun_out/r05_tests_$V.log; exit 1; }
tail -1 gpurun_out/r05_tests_$V.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_$V.log 2>&1 || { tail -20 gpurun_out/r05_smoke_$V.log; exit 1; }
tail -1 gpurun_out/r05_smoke_$V.log
timeout -k 10 600 python -u bench.py > gpurun_out/r05_bench_$V.json.log 2>&1 || { tail -20 gpurun_out/r05_bench_$V.json.log; exit 1; }
tail -1 gpurun_out/r05_bench_$V.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d['roofline']
print('bench', d['value'], 'period', r.get('batch_period_ms'), 'frac', r.get('frac'), ' '.join('%s=%s' % (k, v.get('value')) for k, v in (d.get('configs') or {}).items()))"
HDRF_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 2 --steps 2 --warmup 1 --blocks 64 --no-cpu > gpurun_out/r05_g2_$V.log 2>&1 || { tail -30 gpurun_out/r05_g2_$V.log; exit 1; }
grep "^{" gpurun_out/r05_g2_$V.log | tail -1 | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d['roofline']
print('g2 rehearsal', d['value'], 'front_period_ms', r.get('front_period_ms'), 'chains', r.get('chains_ms_per_batch'))"
