#!/bin/bash
# rocprofv3 passes for one bench configuration (run on the GPU box from the repo root).
# Pass 1: kernel trace + stats. Passes 2-4: PMC counters, one group per pass (gfx950 TCC slots:
# FETCH_SIZE and WRITE_SIZE cannot share a pass), kernel trace only alongside.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
shift || true
ARGS=${@:-"--blocks 64 --steps 2 --warmup 1 --cpu-sample-blocks 0"}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $R/bench.py $ARGS > $OUT/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/bench.py $ARGS > $OUT/write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python3 $R/bench.py $ARGS > $OUT/sq.log 2>&1
echo done
