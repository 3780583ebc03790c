#!/bin/bash
# like run_counters.sh but with an env assignment applied to the profiled bench (arg 2)
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; ENVS=$2; shift 2
ARGS="--blocks 64 --steps 1 --warmup 1 --cpu-sample-blocks 0"
OUT=$R/gpurun_out/cnt_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export $ENVS
cd /tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
