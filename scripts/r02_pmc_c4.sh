#!/bin/bash
# One SQ counter pass over the config-4 bench (instruction mix, waves, busy cycles) -> per-kernel means.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_${TAG:-c4}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- python3 $R/bench.py ${ARGS:---workload config4 --steps 1 --warmup 0 --no-cpu} > $OUT/p1.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/p1.log; exit 1; }
python3 - $OUT <<'PY'
import collections, csv, glob, sys
v = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
        v[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
ks = sorted({k for k, _ in v})
for k in ks:
    d = {c: sum(x) / len(x) for (kk, c), x in v.items() if kk == k}
    if d.get("SQ_WAVES", 0) < 1000: continue
    print(k, {c: "%.4g" % d[c] for c in sorted(d)})
PY
