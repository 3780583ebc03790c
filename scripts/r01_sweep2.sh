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
EXTRA="--batch 32" run b32 X=0
EXTRA="--batch 32 --depth 3" run b32d3 X=0
EXTRA="--batch 32" run b32sha3 HDRF_SHA_WAVES=3
EXTRA="--batch 32" run b32p32k HDRF_PLACE_LDS=32768
EXTRA="--batch 16" run b16 X=0
EXTRA="--batch 16 --depth 3" run b16d3 X=0
EXTRA="--batch 32" run b32b X=0
EXTRA="" run base_b X=0
EXTRA="--batch 32" run b32c X=0
