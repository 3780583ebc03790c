#!/bin/bash
# Round 3: what sets config 5 — drain by the CUs (default) vs the copy engine (HDRF_DRAIN_KERNEL=0)
# vs no drain (ring arena), whole blocks and 64 KiB packets.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
i=0
for v in "X=0" "HDRF_DRAIN_KERNEL=0" "NODRAIN" "X=0" "HDRF_DRAIN_KERNEL=0"; do
  i=$((i+1))
  if [ "$v" = "NODRAIN" ]; then A="--no-drain"; E="X=1"; else A=""; E="$v"; fi
  env $E timeout -k 10 400 python -u bench.py --workload config5 --steps 2 --warmup 1 --no-cpu $A > gpurun_out/c28_$i.json.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/c28_$i.json.log; exit 1; }
  tail -1 gpurun_out/c28_$i.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); p=d['pcie']; print('config5 [$v]', d['value'], p['h2d_GB_s_raw_copy'], p.get('d2h_GB_s_drain'), p.get('link_GB_s'))"
done
for v in "X=0" "HDRF_DRIVER_NODRAIN=1" "HDRF_DRAIN_KERNEL=0"; do
  i=$((i+1))
  env $v timeout -k 10 400 python -u bench.py --workload config5 --packet-driver cpp --packet-kib 64 --steps 2 --warmup 1 --no-cpu > gpurun_out/c28_$i.json.log 2>&1 || { echo "pk failed"; tail -20 gpurun_out/c28_$i.json.log; exit 1; }
  tail -1 gpurun_out/c28_$i.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('packets64 [$v]', d['value'], d['packet_driver']['best_GB_s'])"
done
