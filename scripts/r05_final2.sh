#!/bin/bash
# Round 5 closing profiles: rocprofv3 kernel-trace summaries of the config-2 and config-4 pipelines
# (timed region only: no sub-results, no CPU leg, no alone pass), then the config-4 FETCH_SIZE /
# WRITE_SIZE passes (profiles/r05_c4_traffic.json, read by bench.py's config-4 line).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05_prof_c2 -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-sub --no-cpu --no-alone > $R/gpurun_out/r05_prof_c2.log 2>&1) || { echo "c2 trace failed"; tail -20 gpurun_out/r05_prof_c2.log; exit 1; }
tail -1 gpurun_out/r05_prof_c2.log
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05_prof_c4 -o run -- python3 $R/bench.py --workload config4 --steps 2 --warmup 1 --no-sub --no-cpu --no-alone > $R/gpurun_out/r05_prof_c4.log 2>&1) || { echo "c4 trace failed"; tail -20 gpurun_out/r05_prof_c4.log; exit 1; }
tail -1 gpurun_out/r05_prof_c4.log
TAG=r05_c4 WORKLOAD=config4 ARGS="--workload config4 --steps 1 --warmup 0 --no-cpu --no-alone --no-sub" bash scripts/r02_traffic.sh || exit 1
ls gpurun_out/r05_c4_traffic.json
