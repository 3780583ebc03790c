#!/bin/bash
# Round 4: LZ4 table tags — byte parity (LZ4 / compressor-2 / stream-mode GPU tests), then config-4
# A/B against the previous build (HDRF_LIB_PATH=hdrf_amd/_build_prev/libhdrf.so), alternated.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
V=${V:-a}
[ -n "$NO_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_lz4.py tests/test_config2_shape.py tests/test_bench_shape.py tests/test_packet_driver.py tests/test_boundary.py \
  -k "lz4 or config4 or packet or durable or stream" > gpurun_out/r04_lz4_tests_$V.log 2>&1 || { tail -30 gpurun_out/r04_lz4_tests_$V.log; exit 1; }
[ -n "$NO_TESTS" ] || tail -1 gpurun_out/r04_lz4_tests_$V.log
i=0
for v in ${VARIANTS:-"X=new" "HDRF_LIB_PATH=hdrf_amd/_build_prev/libhdrf.so" "HDRF_LIB_PATH=hdrf_amd/_build_v1/libhdrf.so" "X=new" "HDRF_LIB_PATH=hdrf_amd/_build_prev/libhdrf.so" "HDRF_LIB_PATH=hdrf_amd/_build_v1/libhdrf.so"}; do
  i=$((i+1))
  env $v timeout -k 10 400 python -u bench.py --workload config4 --no-cpu --steps 3 > gpurun_out/r04_lz4ab_${V}_$i.log 2>&1 || { echo "variant $v failed"; tail -20 gpurun_out/r04_lz4ab_${V}_$i.log; exit 1; }
  tail -1 gpurun_out/r04_lz4ab_${V}_$i.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d['roofline']
print('$v', d['value'], 'period', r['batch_period_ms'], r['chains_ms_per_batch'], 'lz4', r.get('lz4',{}).get('avg_launch_ms'))"
done
