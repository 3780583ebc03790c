#!/bin/bash
# Round 4: the whole GPU suite + smoke on the current tree (LZ4 non-returning table updates, X3
# counts, drain tails, batched hand-over), then config 2 with and without the carried SHA window,
# alternated three times.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-A}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_tests_$V.log 2>&1 || { tail -40 gpurun_out/r04_tests_$V.log; exit 1; }
tail -1 gpurun_out/r04_tests_$V.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke_$V.log 2>&1 || { tail -20 gpurun_out/r04_smoke_$V.log; exit 1; }
tail -1 gpurun_out/r04_smoke_$V.log
NO_PMC=1 TAG=r04_carry_$V BENCH_ARGS="--steps 3 --warmup 1 --no-cpu --no-alone" bash scripts/r03_ab.sh \
  "HDRF_SHA_CARRY=0" "HDRF_SHA_CARRY=1" "HDRF_SHA_CARRY=0" "HDRF_SHA_CARRY=1" "HDRF_SHA_CARRY=0" "HDRF_SHA_CARRY=1"
