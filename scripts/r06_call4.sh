#!/bin/bash
# Round 6, call 4: wave-aggregated record counters (gx_emit, place part 1): the node-global GPU tests,
# the packet-driver tests (untimed results step), the loopback bench-shape trace again, then the
# default bench line with the config5_packets sub-line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 880 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_node.py tests/test_packet_driver.py > gpurun_out/r06_tests_c4.log 2>&1 || { tail -40 gpurun_out/r06_tests_c4.log; exit 1; }
tail -1 gpurun_out/r06_tests_c4.log
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06_prof_lb2b -o run -- python3 $R/scripts/node_loopback.py --G 2 --batches 6 > $R/gpurun_out/r06_prof_lb2b.log 2>&1) || { echo "loopback trace failed"; tail -20 gpurun_out/r06_prof_lb2b.log; exit 1; }
grep '^{' gpurun_out/r06_prof_lb2b.log | cut -c1-1500
timeout -k 10 900 python -u bench.py > gpurun_out/r06_bench_c4.json.log 2>&1 || { tail -20 gpurun_out/r06_bench_c4.json.log; exit 1; }
tail -1 gpurun_out/r06_bench_c4.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d['roofline']
print('bench', d['value'], 'period', r.get('batch_period_ms'), 'frac', r.get('frac'))
for k, v in (d.get('configs') or {}).items(): print(k, v.get('value'), v.get('mirror_ok'), v.get('oracle_check') or (v.get('dedup') or {}).get('oracle_check'), (v.get('pcie') or {}).get('link_frac_of_bidirectional_raw'), v.get('error'))"
