#!/bin/bash
# Round 3: LZ4 parse trims (one-clamp window loads, scalar hash words, extension stop logic only
# near matchlimit).  Parity, then per-kind LZ4 kernel times (lz4_scale, one wave per segment at
# 64 MiB, full chip at 2048 MiB) and config 4, each against the previous build (_build_base).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_lz4.py tests/test_snappy.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/c24_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c24_tests.log; exit 1; }
tail -1 gpurun_out/c24_tests.log
B=$R/hdrf_amd/_build_base/libhdrf.so
N=$R/hdrf_amd/_build/libhdrf.so
i=0
for lib in $B $N $B $N; do
  i=$((i+1))
  cd /tmp && export TMPDIR=/tmp
  HDRF_LIB_PATH=$lib LZS_MIB=64,2048 LZS_KINDS=1,2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/lzs24_$i -o run -- python3 $R/scripts/lz4_scale.py > $R/gpurun_out/lzs24_$i.log 2>&1 || { tail -20 $R/gpurun_out/lzs24_$i.log; exit 1; }
  cd $R
  f=$(find gpurun_out/lzs24_$i -name "*kernel_trace.csv" | head -1)
  python3 - $f $lib <<'PY'
import csv, sys
t = [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, 2) for r in csv.DictReader(open(sys.argv[1])) if "lz4_list" in r["Kernel_Name"]]
print(sys.argv[2].split('/')[-2], "lz4_list ms (text 64, 2048 MiB; binary 64, 2048 MiB; first of each pair is warm-up order):", t)
PY
done
for lib in $N $B $N $B; do
  i=$((i+1))
  HDRF_LIB_PATH=$lib timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/c24_$i.json.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/c24_$i.json.log; exit 1; }
  tail -1 gpurun_out/c24_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c4 $(basename $(dirname $lib))', d['value'], d['roofline']['chains_ms_per_batch'], d['roofline']['batch_period_ms'])"
done
