#!/bin/bash
# Default bench + rocprofv3 kernel-trace/stats of the same workload (profiles/ summaries).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --alone --read-blocks 16 --no-cpu --steps 3 > gpurun_out/bench_alone.log 2>&1 || { echo "bench --alone failed"; tail -30 gpurun_out/bench_alone.log; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_kt -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_kt.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_kt.log; exit 1; }
echo ALLDONE
