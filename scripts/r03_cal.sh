#!/bin/bash
# Round 3: which memory-side counters gfx950 exposes, and one pass of the request-size split
# (32 / 64 / 128-B read requests) over a short default-shape bench, to calibrate FETCH_SIZE for
# the non-streaming access patterns (walk, SHA lanes, tails, index, place).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r03_counters.txt 2>&1 || { tail -5 gpurun_out/r03_counters.txt; }
grep -oE "TCC_(EA0|BUBBLE|EA_|REQ|READ|WRITE|HIT|MISS)[A-Za-z0-9_]*" gpurun_out/r03_counters.txt | sort -u > gpurun_out/r03_tcc.txt
cat gpurun_out/r03_tcc.txt | tr '\n' ' '; echo
OUT=$R/gpurun_out/pmc_cal
mkdir -p $OUT
cd /tmp
ARGS="--blocks 96 --steps 1 --warmup 0 --no-cpu --no-alone"
i=0
for grp in "${@}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok: $grp"
done
