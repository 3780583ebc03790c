#!/bin/bash
# Round 4, after the stream-C fix: the packet path's staging copies (4 MiB copies ran at ~36 GB/s
# in the trace vs 56 for 128 MiB): staging chunk 4 vs 16 MiB, shared stream C vs a stream per
# receive buffer, alternated twice (64 KiB mirrored packets, compressor 1).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
i=0
for rep in 1 2; do
for v in "X=def" "HDRF_RX_CHUNK_MB=16" "HDRF_RX_STREAMS=1" "HDRF_RX_CHUNK_MB=16 HDRF_RX_STREAMS=1" "HDRF_RX_CHUNK_MB=8"; do
  i=$((i+1))
  env $v timeout -k 10 400 python -u bench.py --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring > gpurun_out/r04_rxab_$i.json.log 2>&1 || { echo "pk $v failed"; tail -20 gpurun_out/r04_rxab_$i.json.log; exit 1; }
  tail -1 gpurun_out/r04_rxab_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); print('pk64 $v', d['value'], d['packet_driver']['best_GB_s'])"
done
done
