#!/bin/bash
# Round 4, with the non-temporal staging copy: staging chunk 4 (default) vs 8 vs 2 MiB, 64 KiB mirrored
# packets, compressor 1, alternated twice.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
i=0
for rep in 1 2; do
for v in "X=def" "HDRF_RX_CHUNK_MB=8" "HDRF_RX_CHUNK_MB=2"; do
  i=$((i+1))
  env $v timeout -k 10 400 python -u bench.py --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring > gpurun_out/r04_rxchunk2_$i.json.log 2>&1 || { echo "pk $v failed"; tail -20 gpurun_out/r04_rxchunk2_$i.json.log; exit 1; }
  tail -1 gpurun_out/r04_rxchunk2_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); print('pk64 $v', d['value'], d['packet_driver']['best_GB_s'])"
done
done
