#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over the default bench (one counter per rocprofv3 run) ->
# profiles-ready traffic json (scripts/traffic.py applies the gfx950 FETCH_SIZE correction).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r02}
ARGS=${ARGS:-"--steps 1 --warmup 0 --no-cpu --no-alone"}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_GROUPS}; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
WL=${WORKLOAD:-config2}
python3 $R/scripts/traffic.py $OUT $R/gpurun_out/${TAG}_traffic.json "{\"blocks\": 512, \"block_mib\": 128, \"batch\": 32, \"n_gpus\": 1, \"hasher\": 0, \"workload\": \"$WL\"}"
