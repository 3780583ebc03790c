#!/bin/bash
# Round 3: the carried SHA window with the chain's last window trimmed to 132 B (default now) vs the
# 132-B window per iteration (HDRF_SHA_CARRY=0), and the place copy at four 16-B words per thread
# in flight (HDRF_PLACE_DEEP=1).  Full GPU suite on the default, parity of the store path under
# PLACE_DEEP, config 2 rounds of three, config 4 pair, SHA read requests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c30_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c30_tests.log; exit 1; }
tail -1 gpurun_out/c30_tests.log
HDRF_PLACE_DEEP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_shape.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c30_tests2.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c30_tests2.log; exit 1; }
tail -1 gpurun_out/c30_tests2.log
i=0
for v in "X=0" "HDRF_SHA_CARRY=0" "HDRF_PLACE_DEEP=1" "X=0" "HDRF_SHA_CARRY=0" "HDRF_PLACE_DEEP=1" "X=0" "HDRF_SHA_CARRY=0" "HDRF_PLACE_DEEP=1"; do
  i=$((i+1))
  env $v timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/c30_$i.json.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/c30_$i.json.log; exit 1; }
  tail -1 gpurun_out/c30_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c2 $v', d['value'], d['roofline']['chains_ms_per_batch'], d['roofline']['batch_period_ms'], 'sha', d['stages']['sha(sha_chunk_kernel)']['avg_launch_ms'], 'place', d['stages']['place(place_kernel)']['avg_launch_ms'])"
done
for v in "HDRF_PLACE_DEEP=1" "X=0"; do
  i=$((i+1))
  env $v timeout -k 10 600 python -u bench.py --workload config4 --steps 2 --warmup 1 --no-cpu > gpurun_out/c30_$i.json.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/c30_$i.json.log; exit 1; }
  tail -1 gpurun_out/c30_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c4 $v', d['value'], d['roofline']['chains_ms_per_batch'], d['roofline']['batch_period_ms'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum --output-format csv -d $R/gpurun_out/c30_pmc -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-alone > $R/gpurun_out/c30_pmc.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/c30_pmc.log; exit 1; }
python3 - $R/gpurun_out/c30_pmc <<'PY'
import collections, csv, glob, sys
v = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
        v[k].append(float(r["Counter_Value"]))
for k in sorted(v):
    if "sha" in k:
        print("%-26s TCC_EA0_RDREQ per launch %.4e" % (k, sum(v[k]) / len(v[k])))
PY
