#!/bin/bash
# Round 4: staging chunk 8 MiB vs 4 MiB (default), 64 KiB mirrored packets, compressor 1 three more
# alternated pairs, compressor 2 two pairs.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
i=0
for c in 1 1 1 2 2; do
for v in "X=def" "HDRF_RX_CHUNK_MB=8"; do
  i=$((i+1))
  env $v timeout -k 10 400 python -u bench.py --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor $c > gpurun_out/r04_rxchunk3_$i.json.log 2>&1 || { echo "pk $v failed"; tail -20 gpurun_out/r04_rxchunk3_$i.json.log; exit 1; }
  tail -1 gpurun_out/r04_rxchunk3_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); print('pk64 c$c $v', d['value'], d['packet_driver']['best_GB_s'])"
done
done
