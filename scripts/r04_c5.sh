#!/bin/bash
# Round 4: config-5 lines (streaming DataNode write path): native packet driver with block mirroring,
# compressor 1 and 2, per-block and batched submits; whole blocks c1/c2; then the config-4 line.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-a}
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py --workload config5 --steps 3 "$@" > gpurun_out/r04_c5_${n}_$V.json.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/r04_c5_${n}_$V.json.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d.get('pcie',{}); print(sys.argv[2], d['value'], 'mirror', d.get('mirror'), 'bidir', p.get('bidirectional_GB_s_raw_copy'), 'h2d', p.get('h2d_GB_s_raw_copy'), 'v/bidir', p.get('value_over_bidirectional_raw'), 'drain', p.get('d2h_GB_s_drain'))" gpurun_out/r04_c5_${n}_$V.json.log $n
}
run pk64_c1_ring --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1
run pk64_c1_ring_r2 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1
run pk64_c1_ring_r3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1
run pk64_c1_ring_batch --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1 --packet-batch
run pk64_c2_ring --packet-driver cpp --packet-kib 64 --mirror ring --compressor 2
run pk64_c2_ring_batch --packet-driver cpp --packet-kib 64 --mirror ring --compressor 2 --packet-batch
run pk64_c2mixed_ring_batch --packet-driver cpp --packet-kib 64 --mirror ring --compressor 2 --packet-batch --mixed
run pk64_c1_none --packet-driver cpp --packet-kib 64 --mirror none --compressor 1
run pk64_c1_socket --packet-driver cpp --packet-kib 64 --mirror socket --compressor 1
run whole_c1 --compressor 1
run whole_c2 --compressor 2
timeout -k 10 600 python -u bench.py --workload config4 > gpurun_out/r04_c4_$V.json.log 2>&1 || { tail -20 gpurun_out/r04_c4_$V.json.log; exit 1; }
tail -1 gpurun_out/r04_c4_$V.json.log | cut -c1-300
