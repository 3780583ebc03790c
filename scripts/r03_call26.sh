#!/bin/bash
# Round 3: config-4 FETCH/WRITE traffic passes (-> profiles/r03_c4_traffic.json, the LZ4 line's
# `traffic`), the config-2 line with the split chains, and config 5 64 KiB packets: completer
# thread vs serial driver loop, three pairs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=r03_c4 WORKLOAD=config4 ARGS="--workload config4 --steps 1 --warmup 0 --no-cpu --no-alone" bash scripts/r02_traffic.sh > gpurun_out/c26_traffic.txt 2>&1 || { tail -20 gpurun_out/c26_traffic.txt; exit 1; }
grep -E "lz4|sha_chunk|place" gpurun_out/c26_traffic.txt
cd $R
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/c26_c2.json.log 2>&1 || { tail -20 gpurun_out/c26_c2.json.log; exit 1; }
tail -1 gpurun_out/c26_c2.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c2', d['value'], d['roofline']['critical_path'], d['roofline']['chains_ms_per_batch'], d['roofline']['batch_period_ms'])"
i=0
for v in "HDRF_DRIVER_SERIAL=1" "HDRF_DRIVER_X=0" "HDRF_DRIVER_SERIAL=1" "HDRF_DRIVER_X=0" "HDRF_DRIVER_SERIAL=1" "HDRF_DRIVER_X=0"; do
  i=$((i+1))
  env $v timeout -k 10 400 python -u bench.py --workload config5 --packet-kib 64 --packet-threads 4 --packet-driver cpp --steps 2 --warmup 1 --no-cpu > gpurun_out/c26_$i.json.log 2>&1 || { echo "c5 failed"; tail -20 gpurun_out/c26_$i.json.log; exit 1; }
  tail -1 gpurun_out/c26_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin)
print('== c5 pk64 $v', d['value'], d['packet_driver']['best_GB_s'], d['driver_wall_s'])"
done
# L2 hit rate of the LZ4 pass (and its neighbours) on config 4
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/gpurun_out/c26_tcc -o run -- python3 $R/bench.py --workload config4 --steps 1 --warmup 0 --no-cpu --no-alone > $R/gpurun_out/c26_tcc.log 2>&1 || { echo "tcc pass failed"; tail -5 $R/gpurun_out/c26_tcc.log; exit 1; }
cd $R
python3 - gpurun_out/c26_tcc <<'PY'
import collections, csv, glob, sys
v = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
        v[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for k in sorted({k for k, _ in v}):
    h = sum(v.get((k, "TCC_HIT_sum"), [0])); m = sum(v.get((k, "TCC_MISS_sum"), [0]))
    if h + m > 1e6:
        print("%-28s TCC hit %.3e miss %.3e hit rate %.3f" % (k[:28], h, m, h / (h + m)))
PY
