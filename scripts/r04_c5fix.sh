#!/bin/bash
# Round 4: stream C carries only H2D copies (no slack-fill kernels between the block copies, recipe
# copies on their own stream R): host-path / packet-path / boundary GPU tests, then config 5 (whole
# blocks c1 / c2, 64 KiB mirrored packets c1 x2, c2) and config 2.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-g}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_boundary.py tests/test_gpu_parity.py tests/test_packet_driver.py > gpurun_out/r04_c5fix_tests_$V.log 2>&1 || { tail -30 gpurun_out/r04_c5fix_tests_$V.log; exit 1; }
tail -1 gpurun_out/r04_c5fix_tests_$V.log
run() {
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r04_${tag}_$V.json.log 2>&1 || { echo "$tag failed"; tail -20 gpurun_out/r04_${tag}_$V.json.log; exit 1; }
  tail -1 gpurun_out/r04_${tag}_$V.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); p=d.get('pcie') or {}; r=d.get('roofline') or {}
print('$tag', d['value'], 'period', r.get('batch_period_ms'), 'pd', (d.get('packet_driver') or {}).get('best_GB_s'), 'bidir', p.get('bidirectional_GB_s_raw_copy'), 'frac', p.get('value_over_bidirectional_raw'))"
}
run c5_whole_c1 --workload config5 --steps 3
run c5_whole_c2 --workload config5 --steps 3 --compressor 2
run c5_pk64_c1_ring --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1
run c5_pk64_c2_ring --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 2
run c5_pk64_c1_ring_2 --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1
run c2 --steps 5 --no-cpu
