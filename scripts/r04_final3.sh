#!/bin/bash
# Round 4 final check on the committed tree after the config-5 changes (copy stream with copies only,
# drain pacing, non-temporal staging copy): GPU suite, smoke, the default line (config 2 with the CPU
# leg), config 4, config 5 whole blocks (c1, c2) and 64 KiB mirrored packets (c1, c2; twice each).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-i}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_tests_$V.log 2>&1 || { tail -40 gpurun_out/r04_tests_$V.log; exit 1; }
tail -1 gpurun_out/r04_tests_$V.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke_$V.log 2>&1 || { tail -20 gpurun_out/r04_smoke_$V.log; exit 1; }
tail -1 gpurun_out/r04_smoke_$V.log
run() {
  local tag=$1; shift
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/r04_${tag}_$V.json.log 2>&1 || { echo "$tag failed"; tail -20 gpurun_out/r04_${tag}_$V.json.log; exit 1; }
  tail -1 gpurun_out/r04_${tag}_$V.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); p=d.get('pcie') or {}; r=d.get('roofline') or {}
print('$tag', d['value'], 'period', r.get('batch_period_ms'), 'frac', r.get('frac'), 'pd', (d.get('packet_driver') or {}).get('best_GB_s'), 'v/bidir', p.get('value_over_bidirectional_raw'))"
}
run bench
run c4 --workload config4
run c5_whole_c1 --workload config5 --steps 3
run c5_whole_c2 --workload config5 --steps 3 --compressor 2
run c5_pk64_c1_ring --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1
run c5_pk64_c2_ring --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 2
run c5_pk64_c1_ring_2 --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1
run c5_pk64_c2_ring_2 --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 2
