#!/bin/bash
# Round 4: packet driver with continuous receivers (no lockstep rounds) — parity, then config-5 lines.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-d}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_packet_driver.py tests/test_boundary.py > gpurun_out/r04_c5d_tests_$V.log 2>&1 || { tail -30 gpurun_out/r04_c5d_tests_$V.log; exit 1; }
tail -1 gpurun_out/r04_c5d_tests_$V.log
run() {   # name, env, args...
  local n=$1; local e=$2; shift 2
  env $e timeout -k 10 400 python -u bench.py --workload config5 --steps 3 "$@" > gpurun_out/r04_c5_${n}_$V.json.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/r04_c5_${n}_$V.json.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d.get('pcie',{}); q=d.get('packet_driver',{}); print(sys.argv[2], d['value'], 'ms/step', d['ms_per_step'], 'link', p.get('link_GB_s'), 'drain', p.get('d2h_GB_s_drain'), 'v/bidir', p.get('value_over_bidirectional_raw'), 'batches', q.get('batches_per_step'), 'mirror_ok', q.get('mirror_ok'))" gpurun_out/r04_c5_${n}_$V.json.log $n
}
run pk64_c1_ring X=1 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1
run pk64_c1_ring_r2 X=1 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1
run pk64_c1_ring_r3 X=1 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1
run pk64_c1_ring_t8 X=1 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1 --packet-threads 8
run pk64_c1_ring_batch X=1 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1 --packet-batch
run pk64_c1_ring_batch_t8 X=1 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1 --packet-batch --packet-threads 8
run pk64_c2_ring X=1 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 2
run pk64_c2_ring_batch_t8 X=1 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 2 --packet-batch --packet-threads 8
run pk64_c1_socket X=1 --packet-driver cpp --packet-kib 64 --mirror socket --compressor 1
run pk64_c1_none X=1 --packet-driver cpp --packet-kib 64 --mirror none --compressor 1
