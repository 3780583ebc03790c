#!/bin/bash
# SQ counters per kernel for env-selected variants: pmc_ab.sh "ENV=.." "ENV=.." (serial bench, 64 blocks)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
ARGS=${BENCH_ARGS:-"--blocks 64 --steps 1 --warmup 1 --no-cpu --serial"}
CTRS=${CTRS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"}
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  OUT=$R/gpurun_out/pmcab_$i
  mkdir -p $OUT
  cd /tmp
  env $v timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d $OUT -o run -- python3 $R/bench.py $ARGS > $OUT/log 2>&1 || { echo "pmc $v failed"; tail -5 $OUT/log; exit 1; }
  cd $R
  echo "== $v"
  python3 scripts/cnt_report.py $OUT ${KFILTER:-spec_walk}
done
