#!/bin/bash
# Round 6, call 8: sha_carry loads clamped at the chunk end — parity tests on the variant build, the
# config-2 A/B (scripts/ab_r06_shaclamp.txt), and the variant's FETCH_SIZE / WRITE_SIZE passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
HDRF_LIB_PATH=$R/hdrf_amd/_build_shaclamp/libhdrf.so timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_parity.py tests/test_slack.py "tests/test_bench_shape.py::test_bench_primed_depth4_reset_async_generations" > gpurun_out/r06_tests_c8.log 2>&1 || { tail -40 gpurun_out/r06_tests_c8.log; exit 1; }
tail -1 gpurun_out/r06_tests_c8.log
TAG=r06_shaclamp bash scripts/abrun.sh scripts/ab_r06_shaclamp.txt || exit 1
OUT=$R/gpurun_out/pmc_r06_shaclamp
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  (cd /tmp && HDRF_LIB_PATH=$R/hdrf_amd/_build_shaclamp/libhdrf.so timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-alone --no-sub > $OUT/p$i.log 2>&1) || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/traffic.py $OUT gpurun_out/r06_shaclamp_traffic_ab.json '{"blocks": 512, "block_mib": 128, "batch": 32, "n_gpus": 1, "hasher": 0, "workload": "config2", "variant": "HDRF_SHA_CLAMP=1"}' | grep -E "sha_carry|place|gmax2"
