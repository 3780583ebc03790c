#!/bin/bash
# Round 4: packet path A/B, alternated: HW queues 4 / 8 with per-receive-buffer H2D streams.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-f}
run() {   # name, env, args...
  local n=$1; local e=$2; shift 2
  env $e timeout -k 10 400 python -u bench.py --workload config5 --steps 3 "$@" > gpurun_out/r04_c5_${n}_$V.json.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/r04_c5_${n}_$V.json.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d.get('pcie',{}); q=d.get('packet_driver',{}); print(sys.argv[2], d['value'], 'ms/step', d['ms_per_step'], 'link', p.get('link_GB_s'), 'drain', p.get('d2h_GB_s_drain'), 'v/bidir', p.get('value_over_bidirectional_raw'), 'batches', q.get('batches_per_step'), 'mirror_ok', q.get('mirror_ok'))" gpurun_out/r04_c5_${n}_$V.json.log $n
}
P="--packet-driver cpp --packet-kib 64 --mirror ring --compressor 1"
for r in 1 2 3; do
  run q4_rxs_$r "GPU_MAX_HW_QUEUES=4 HDRF_RX_STREAMS=1" $P
  run q8_rxs_$r "GPU_MAX_HW_QUEUES=8 HDRF_RX_STREAMS=1" $P
  run q4_$r GPU_MAX_HW_QUEUES=4 $P
  run q6_rxs_$r "GPU_MAX_HW_QUEUES=6 HDRF_RX_STREAMS=1" $P
done
