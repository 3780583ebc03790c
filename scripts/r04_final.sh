#!/bin/bash
# Round 4 closing run on the committed tree: GPU suite, config-2 kernel trace + FETCH/WRITE/VALU
# traffic, the default bench line (config 2, CPU leg); part 2 (r04_final2.sh): config 4, config 5, g2.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_tests_$V.log 2>&1 || { tail -40 gpurun_out/r04_tests_$V.log; exit 1; }
tail -1 gpurun_out/r04_tests_$V.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke_$V.log 2>&1 || { tail -20 gpurun_out/r04_smoke_$V.log; exit 1; }
tail -1 gpurun_out/r04_smoke_$V.log
TAG=r04_prof_$V BENCH="--steps 2 --warmup 1 --no-cpu --no-alone" bash scripts/r02_prof.sh > gpurun_out/r04_prof_$V.txt 2>&1 || { tail -20 gpurun_out/r04_prof_$V.txt; exit 1; }
head -14 gpurun_out/r04_prof_$V.txt | cut -c1-160
TAG=r04_$V EXTRA_GROUPS="SQ_INSTS_VALU" bash scripts/r02_traffic.sh > gpurun_out/r04_traffic_$V.txt 2>&1 || { tail -20 gpurun_out/r04_traffic_$V.txt; exit 1; }
mkdir -p profiles && cp gpurun_out/r04_${V}_traffic.json profiles/r04_${V}_traffic.json
timeout -k 10 600 python -u bench.py > gpurun_out/r04_bench_$V.json.log 2>&1 || { tail -20 gpurun_out/r04_bench_$V.json.log; exit 1; }
tail -1 gpurun_out/r04_bench_$V.json.log | cut -c1-300
