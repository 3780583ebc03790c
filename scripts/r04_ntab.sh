#!/bin/bash
# Round 4: non-temporal stores for the packet staging copy (HDRF_RX_NT, default on) — packet-path
# GPU tests, then 64 KiB mirrored packets alternated with HDRF_RX_NT=0, three pairs.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_boundary.py tests/test_packet_driver.py > gpurun_out/r04_ntab_tests.log 2>&1 || { tail -30 gpurun_out/r04_ntab_tests.log; exit 1; }
tail -1 gpurun_out/r04_ntab_tests.log
i=0
for rep in 1 2 3; do
for v in "X=nt" "HDRF_RX_NT=0"; do
  i=$((i+1))
  env $v timeout -k 10 400 python -u bench.py --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring > gpurun_out/r04_ntab_$i.json.log 2>&1 || { echo "pk $v failed"; tail -20 gpurun_out/r04_ntab_$i.json.log; exit 1; }
  tail -1 gpurun_out/r04_ntab_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); print('pk64 $v', d['value'], d['packet_driver']['best_GB_s'])"
done
done
bash scripts/r04_xferab.sh
