#!/bin/bash
# Kernel-trace summary of a short default bench (per-kernel average durations).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-prof}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o run -- python3 -u bench.py ${BENCH:---steps 2 --warmup 1 --no-cpu} > gpurun_out/$TAG.log 2>&1 || { tail -20 gpurun_out/$TAG.log; exit 1; }
tail -1 gpurun_out/$TAG.log | cut -c1-400
f=$(find gpurun_out/$TAG -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print("%-60s %6s calls  avg %9.1f us  total %8.2f ms" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
