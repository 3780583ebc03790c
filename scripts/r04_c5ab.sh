#!/bin/bash
# Round 4: drain engine A/B after the stream-C fix (HDRF_DRAIN_KERNEL=0: copy engine, 1: CUs) for
# whole blocks and 64 KiB mirrored packets, alternated; then a kernel + memory-copy trace of the
# packet driver itself (2 steps).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
R=$(pwd)
i=0
for v in "X=def" "HDRF_DRAIN_KERNEL=0" "X=def" "HDRF_DRAIN_KERNEL=0"; do
  i=$((i+1))
  env $v timeout -k 10 400 python -u bench.py --workload config5 --steps 3 > gpurun_out/r04_c5ab_w$i.json.log 2>&1 || { echo "whole $v failed"; tail -20 gpurun_out/r04_c5ab_w$i.json.log; exit 1; }
  tail -1 gpurun_out/r04_c5ab_w$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); print('whole $v', d['value'], d['roofline'].get('batch_period_ms'))"
done
i=0
for v in "X=def" "HDRF_DRAIN_KERNEL=1" "X=def" "HDRF_DRAIN_KERNEL=1"; do
  i=$((i+1))
  env $v timeout -k 10 400 python -u bench.py --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring > gpurun_out/r04_c5ab_p$i.json.log 2>&1 || { echo "pk $v failed"; tail -20 gpurun_out/r04_c5ab_p$i.json.log; exit 1; }
  tail -1 gpurun_out/r04_c5ab_p$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); print('pk64 $v', d['value'], d['packet_driver']['best_GB_s'])"
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/pktrace -o run -- $R/tools/_build/packet_driver 128 128 64 4 2 --compressor 1 --mirror ring --arena-slots 512 > $R/gpurun_out/pktrace.log 2>&1) || { echo "trace failed"; tail -20 gpurun_out/pktrace.log; exit 1; }
tail -1 gpurun_out/pktrace.log | cut -c1-300
