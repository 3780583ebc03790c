#!/bin/bash
# Knob sweep on the default config-2 workload (one GPU): prints one "tag value ms" line per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sweep
mkdir -p $OUT
run() {
  tag=$1; shift
  env "$@" timeout -k 10 120 python3 $R/bench.py --no-cpu --steps 4 --warmup 1 $EXTRA > $OUT/$tag.log 2>&1 || { echo "$tag FAILED"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_step'])" | tee -a $OUT/summary.txt
}
EXTRA="" run base X=0
EXTRA="--depth 3" run depth3 X=0
EXTRA="" run place32k HDRF_PLACE_LDS=32768
EXTRA="" run place48k HDRF_PLACE_LDS=49152
EXTRA="" run place64k HDRF_PLACE_LDS=65536
EXTRA="" run walk6 HDRF_WALK_WAVES=6
EXTRA="" run walk10 HDRF_WALK_WAVES=10
EXTRA="" run sha3 HDRF_SHA_WAVES=3
EXTRA="" run sha5 HDRF_SHA_WAVES=5
EXTRA="" run prio0 HDRF_PRIO=0
EXTRA="--batch 32" run batch32 X=0
EXTRA="" run base2 X=0
