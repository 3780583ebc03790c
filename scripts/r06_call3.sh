#!/bin/bash
# Round 6, call 3: node-global ranks measurable on one GPU (verdict r5 item 5).  The loopback G = 2
# bench-shape parity test, then kernel traces of (a) the loopback at the bench's batch shape (one
# process, two contexts, no gloo) and (b) the N = 1 pipeline, for the per-rank kernel time per batch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 880 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_node.py::test_node_loopback_bench_shape_two_ranks" > gpurun_out/r06_tests_c3.log 2>&1 || { tail -40 gpurun_out/r06_tests_c3.log; exit 1; }
tail -1 gpurun_out/r06_tests_c3.log
grep -o '{"G".*' gpurun_out/r06_tests_c3.log | head -1 | cut -c1-600
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06_prof_lb2 -o run -- python3 $R/scripts/node_loopback.py --G 2 --batches 6 > $R/gpurun_out/r06_prof_lb2.log 2>&1) || { echo "loopback trace failed"; tail -20 gpurun_out/r06_prof_lb2.log; exit 1; }
tail -1 gpurun_out/r06_prof_lb2.log | cut -c1-1500
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06_prof_c2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-sub --no-cpu --no-alone > $R/gpurun_out/r06_prof_c2.log 2>&1) || { echo "c2 trace failed"; tail -20 gpurun_out/r06_prof_c2.log; exit 1; }
tail -1 gpurun_out/r06_prof_c2.log | cut -c1-300
echo traces ok
