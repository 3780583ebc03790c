#!/bin/bash
# Round 3: sha_carry (HDRF_SHA_CARRY=1: 4-block windows, the second pair carried in registers).
# Parity under it, config 2 A/B (three pairs), then L2->memory read requests of the SHA kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
HDRF_SHA_CARRY=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c29_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/c29_tests.log; exit 1; }
tail -1 gpurun_out/c29_tests.log
i=0
for v in "HDRF_SHA_CARRY=1" "HDRF_SHA_CARRY=0" "HDRF_SHA_CARRY=1" "HDRF_SHA_CARRY=0" "HDRF_SHA_CARRY=1" "HDRF_SHA_CARRY=0"; do
  i=$((i+1))
  env $v timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/c29_$i.json.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/c29_$i.json.log; exit 1; }
  tail -1 gpurun_out/c29_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c2 $v', d['value'], d['roofline']['chains_ms_per_batch'], d['roofline']['batch_period_ms'], 'sha', d['stages']['sha(sha_chunk_kernel)']['avg_launch_ms'])"
done
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  HDRF_SHA_CARRY=$v timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum --output-format csv -d $R/gpurun_out/c29_pmc$v -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-alone > $R/gpurun_out/c29_pmc$v.log 2>&1 || { echo "pmc failed"; tail -5 $R/gpurun_out/c29_pmc$v.log; exit 1; }
  python3 - $R/gpurun_out/c29_pmc$v $v <<'PY'
import collections, csv, glob, sys
v = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
        v[k].append(float(r["Counter_Value"]))
for k in sorted(v):
    if "sha" in k:
        print("carry=%s %-26s TCC_EA0_RDREQ per launch %.4e" % (sys.argv[2], k, sum(v[k]) / len(v[k])))
PY
done
