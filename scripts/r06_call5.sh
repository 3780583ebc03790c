#!/bin/bash
# Round 6, call 5: the config5_packets sub-line alone (link probe before the checks), the two-rank
# same-device rehearsal of the primed N > 1 bench line (node-global hdrf_reset_async between steps),
# and the rehearsal test.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py --workload config5 --packet-driver cpp --packet-batch --compressor 2 --mirror ring --steps 3 > gpurun_out/r06_c5pk.json.log 2>&1 || { tail -20 gpurun_out/r06_c5pk.json.log; exit 1; }
tail -1 gpurun_out/r06_c5pk.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('c5 packets', d['value'], d['packet_driver'].get('best_GB_s'), d.get('mirror_ok'), d.get('oracle_check'), d['pcie'].get('link_frac_of_bidirectional_raw'), d['pcie'].get('bidirectional_passes_GB_s'))"
HDRF_BENCH_SAME_DEVICE=1 timeout -k 10 500 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 2 --steps 2 --warmup 1 --blocks 64 --no-cpu > gpurun_out/r06_g2_c5.log 2>&1 || { tail -30 gpurun_out/r06_g2_c5.log; exit 1; }
grep '^{' gpurun_out/r06_g2_c5.log | tail -1 | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d['roofline']
print('g2 rehearsal', d['value'], 'primed', d['config'].get('steps_back_to_back'), 'chains', r.get('chains_ms_per_batch'), 'period', r.get('batch_period_ms'))"
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_node.py::test_node_bench_rehearsal_two_ranks_one_device" > gpurun_out/r06_tests_c5.log 2>&1 || { tail -40 gpurun_out/r06_tests_c5.log; exit 1; }
tail -1 gpurun_out/r06_tests_c5.log
