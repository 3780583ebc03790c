#!/bin/bash
# Round 3: idx_decide settles the designated chunk of entries without repeats (idx_finalize then
# only clears them: stores, no entry fetch); HDRF_DECIDE_DESIG=0 restores the c2 finalize.  Full GPU
# suite, the same under =0, config 2 A/B (four pairs), finalize read requests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c32_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c32_tests.log; exit 1; }
tail -1 gpurun_out/c32_tests.log
HDRF_DECIDE_DESIG=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_shape.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c32_tests0.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c32_tests0.log; exit 1; }
tail -1 gpurun_out/c32_tests0.log
i=0
for v in "HDRF_DECIDE_DESIG=0" "X=0" "HDRF_DECIDE_DESIG=0" "X=0" "HDRF_DECIDE_DESIG=0" "X=0" "HDRF_DECIDE_DESIG=0" "X=0"; do
  i=$((i+1))
  env $v timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/c32_$i.json.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/c32_$i.json.log; exit 1; }
  tail -1 gpurun_out/c32_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c2 $v', d['value'], d['roofline']['chains_ms_per_batch'], d['roofline']['batch_period_ms'])"
done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  HDRF_DECIDE_DESIG=$v timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/c32_pmc$v -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-alone > $R/gpurun_out/c32_pmc$v.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/c32_pmc$v.log; exit 1; }
  python3 - $R/gpurun_out/c32_pmc$v $v <<'PY'
import collections, csv, glob, sys
v = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
        v[k].append(float(r["Counter_Value"]))
for k in sorted(v):
    if "idx_" in k:
        print("decide_desig=%s %-24s FETCH_SIZE KiB per launch %.4e" % (sys.argv[2], k, sum(v[k]) / len(v[k])))
PY
done
