#!/bin/bash
# Round 5 closing run on the committed tree: GPU suite, smoke, the default line (config 2 primed at
# depth 4, with the CPU leg and the config-4 / config-5 sub-results), config 4 with its CPU leg
# (container-file check), config 5 whole blocks (c1, c2) and 64 KiB mirrored packets (c1, c2).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-final}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_tests_$V.log 2>&1 || { tail -40 gpurun_out/r05_tests_$V.log; exit 1; }
tail -1 gpurun_out/r05_tests_$V.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_$V.log 2>&1 || { tail -20 gpurun_out/r05_smoke_$V.log; exit 1; }
tail -1 gpurun_out/r05_smoke_$V.log
run() {
  local tag=$1; shift
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/r05_${tag}_$V.json.log 2>&1 || { echo "$tag failed"; tail -20 gpurun_out/r05_${tag}_$V.json.log; exit 1; }
  tail -1 gpurun_out/r05_${tag}_$V.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); p=d.get('pcie') or {}; r=d.get('roofline') or {}
subs=' '.join('%s=%s' % (k, v.get('value')) for k, v in (d.get('configs') or {}).items())
print('$tag', d['value'], 'period', r.get('batch_period_ms'), 'frac', r.get('frac'), 'pd', (d.get('packet_driver') or {}).get('best_GB_s'), 'v/bidir', p.get('value_over_bidirectional_raw'), subs)"
}
run bench --steps 20 --warmup 2
run c4 --workload config4
run c5_whole_c1 --workload config5 --steps 3
run c5_whole_c2 --workload config5 --steps 3 --compressor 2
run c5_pk64_c1_ring --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1
run c5_pk64_c2_ring --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 2
