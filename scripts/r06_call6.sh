#!/bin/bash
# Round 6, call 6: workgroup-reserved record counters (gx_emit x4 tiles, own_decide, x3want, place
# part 1): the node-global GPU tests, then the loopback bench-shape kernel trace again.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 880 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_node.py > gpurun_out/r06_tests_c6.log 2>&1 || { tail -40 gpurun_out/r06_tests_c6.log; exit 1; }
tail -1 gpurun_out/r06_tests_c6.log
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06_prof_lb2c -o run -- python3 $R/scripts/node_loopback.py --G 2 --batches 6 > $R/gpurun_out/r06_prof_lb2c.log 2>&1) || { echo "loopback trace failed"; tail -20 gpurun_out/r06_prof_lb2c.log; exit 1; }
grep '^{' gpurun_out/r06_prof_lb2c.log | cut -c1-400
timeout -k 10 300 python3 scripts/node_loopback.py --G 2 --batches 8 > gpurun_out/r06_lb2c_noprof.log 2>&1 || { tail -20 gpurun_out/r06_lb2c_noprof.log; exit 1; }
grep '^{' gpurun_out/r06_lb2c_noprof.log | cut -c1-300
