#!/bin/bash
# packet receive path: parity tests, then config 5 with 4 MiB / 64 KiB packets at 1 and 4 receiver threads
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_boundary.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_rx.log 2>&1 || { tail -30 gpurun_out/tests_rx.log; exit 1; }
tail -1 gpurun_out/tests_rx.log
for cfg in "4096 1" "4096 4" "64 4" "64 8"; do set -- $cfg
timeout -k 10 300 python -u bench.py --workload config5 --steps 1 --warmup 1 --no-cpu --packet-kib $1 --packet-threads $2 > gpurun_out/bench_c5_rx_$1_$2.json.log 2>&1 || { tail -5 gpurun_out/bench_c5_rx_$1_$2.json.log; exit 1; }
echo "packets $1 KiB threads $2: $(tail -1 gpurun_out/bench_c5_rx_$1_$2.json.log | cut -c90-130)"
done
