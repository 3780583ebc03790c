#!/bin/bash
# Extra PMC passes (one counter group per pass) for kernel analysis; run from the repo root on the box.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
ARGS="--blocks 64 --steps 1 --warmup 1 --cpu-sample-blocks 0"
OUT=$R/gpurun_out/cnt_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
