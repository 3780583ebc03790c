#!/bin/bash
# Round 6, call 25: the whole-line maxima A/B again on another box, order swapped (scripts/ab_r06_walkline2.txt),
# then the walk's FETCH_SIZE on both builds (one counter per rocprofv3 run).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=r06_wm bash scripts/abrun.sh scripts/ab_r06_walkline2.txt || exit 1
export TMPDIR=/tmp
for v in a b; do
  if [ $v = b ]; then export HDRF_LIB_PATH=$R/hdrf_amd/_build_ab/libhdrf.so; fi
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r06_wlpmc_$v -o run -- \
    python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-alone --no-sub --no-corpus-check > $R/gpurun_out/r06_wlpmc_$v.log 2>&1) || { echo "pmc $v failed"; exit 1; }
done
unset HDRF_LIB_PATH
python3 - <<'PY'
import csv, glob
for v in 'ab':
    vals = {}
    for f in glob.glob('gpurun_out/r06_wlpmc_%s/*/run_counter_collection.csv' % v) + glob.glob('gpurun_out/r06_wlpmc_%s/run_counter_collection.csv' % v):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '').replace('hdrf::', '')
            vals.setdefault(k, []).append(float(r['Counter_Value']))
    for k in sorted(vals):
        if 'lane_walk' in k or 'gmax2' in k:
            print(v, k, 'FETCH_SIZE KiB x2 per launch', round(2 * sum(vals[k]) / len(vals[k])))
PY
