#!/bin/bash
# Round 4: config-5 exploration — whole-block batch size / step length / drain engine, packet
# receiver thread count.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-b}
run() {   # name, env, args...
  local n=$1; local e=$2; shift 2
  env $e timeout -k 10 400 python -u bench.py --workload config5 --steps 3 "$@" > gpurun_out/r04_c5_${n}_$V.json.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/r04_c5_${n}_$V.json.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d.get('pcie',{}); print(sys.argv[2], d['value'], 'ms/step', d['ms_per_step'], 'link', p.get('link_GB_s'), 'drain', p.get('d2h_GB_s_drain'), 'drained', p.get('drained_container_bytes_per_step'))" gpurun_out/r04_c5_${n}_$V.json.log $n
}
run whole_c1 X=1 --compressor 1
run whole_c1_b16 X=1 --compressor 1 --batch 16
run whole_c1_b8 X=1 --compressor 1 --batch 8
run whole_c1_ce HDRF_DRAIN_KERNEL=0 --compressor 1
run whole_c1_256 X=1 --compressor 1 --blocks 256
run whole_c1_b8r X=1 --compressor 1 --batch 8
run whole_c1r X=1 --compressor 1
run pk64_c1_ring_t8 X=1 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1 --packet-threads 8
run pk64_c1_ring_t16 X=1 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1 --packet-threads 16
run pk64_c1_none_t8 X=1 --packet-driver cpp --packet-kib 64 --mirror none --compressor 1 --packet-threads 8
run pk64_c1_ring_t4 X=1 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1 --packet-threads 4
