#!/bin/bash
# Round 3: register caps (HDRF_VCAP=1: LZ4 byU32 pass at 96 VGPRs, SHA at 128) so one SHA wave fits
# on a SIMD beside four LZ4 waves.  LZ4 + SHA parity under the caps, then config 4 and config 2 A/B.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
HDRF_VCAP=1 timeout -k 10 300 python -u -m pytest tests/test_lz4.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c23_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c23_tests.log; exit 1; }
tail -2 gpurun_out/c23_tests.log
i=0
for v in "HDRF_VCAP=0" "HDRF_VCAP=1" "HDRF_VCAP=0" "HDRF_VCAP=1"; do
  i=$((i+1))
  env $v timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/c23_$i.json.log 2>&1 || { echo "variant $v failed"; tail -20 gpurun_out/c23_$i.json.log; exit 1; }
  tail -1 gpurun_out/c23_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c4 $v', d['value'], d['roofline']['chains_ms_per_batch'], d['roofline']['batch_period_ms'])
print('  '.join('%s=%.1f' % (k.split('(')[0], v['avg_launch_ms']) for k, v in d['stages'].items()))"
done
for v in "HDRF_VCAP=1" "HDRF_VCAP=0" "HDRF_VCAP=1"; do
  i=$((i+1))
  env $v timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/c23_$i.json.log 2>&1 || { echo "variant $v failed"; tail -20 gpurun_out/c23_$i.json.log; exit 1; }
  tail -1 gpurun_out/c23_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c2 $v', d['value'], d['roofline']['chains_ms_per_batch'])"
done
