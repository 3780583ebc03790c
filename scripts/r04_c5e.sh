#!/bin/bash
# Round 4: packet path — hardware queues for the driver's streams (GPU_MAX_HW_QUEUES, HIP default 4
# vs the in-process lines' 8) and per-receive-buffer H2D streams (HDRF_RX_STREAMS=1).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-e}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_packet_driver.py tests/test_boundary.py > gpurun_out/r04_c5e_tests_$V.log 2>&1 || { tail -30 gpurun_out/r04_c5e_tests_$V.log; exit 1; }
HDRF_RX_STREAMS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_packet_driver.py tests/test_boundary.py -k "packet" > gpurun_out/r04_c5e_tests2_$V.log 2>&1 || { tail -30 gpurun_out/r04_c5e_tests2_$V.log; exit 1; }
tail -1 gpurun_out/r04_c5e_tests_$V.log; tail -1 gpurun_out/r04_c5e_tests2_$V.log
run() {   # name, env, args...
  local n=$1; local e=$2; shift 2
  env $e timeout -k 10 400 python -u bench.py --workload config5 --steps 3 "$@" > gpurun_out/r04_c5_${n}_$V.json.log 2>&1 || { echo "FAIL $n"; tail -5 gpurun_out/r04_c5_${n}_$V.json.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); p=d.get('pcie',{}); q=d.get('packet_driver',{}); print(sys.argv[2], d['value'], 'ms/step', d['ms_per_step'], 'link', p.get('link_GB_s'), 'drain', p.get('d2h_GB_s_drain'), 'v/bidir', p.get('value_over_bidirectional_raw'), 'batches', q.get('batches_per_step'), 'mirror_ok', q.get('mirror_ok'))" gpurun_out/r04_c5_${n}_$V.json.log $n
}
P="--packet-driver cpp --packet-kib 64 --mirror ring --compressor 1"
run q4 GPU_MAX_HW_QUEUES=4 $P
run q8 GPU_MAX_HW_QUEUES=8 $P
run q8_rxs "GPU_MAX_HW_QUEUES=8 HDRF_RX_STREAMS=1" $P
run q16_rxs "GPU_MAX_HW_QUEUES=16 HDRF_RX_STREAMS=1" $P
run q4b GPU_MAX_HW_QUEUES=4 $P
run q8b GPU_MAX_HW_QUEUES=8 $P
run q8_rxsb "GPU_MAX_HW_QUEUES=8 HDRF_RX_STREAMS=1" $P
run q16_rxsb "GPU_MAX_HW_QUEUES=16 HDRF_RX_STREAMS=1" $P
run q8_batch GPU_MAX_HW_QUEUES=8 $P --packet-batch
run q8_c2 GPU_MAX_HW_QUEUES=8 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 2
