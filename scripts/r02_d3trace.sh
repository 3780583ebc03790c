# kernel-trace timeline of the config-2 pipeline at depth 2 and 3 (gaps per stream)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for d in 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/d3t_$d -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --depth $d > $R/gpurun_out/d3t_$d.log 2>&1 || { tail -20 $R/gpurun_out/d3t_$d.log; exit 1; }
done
cd $R
for d in 2 3; do
f=$(find gpurun_out/d3t_$d -name "*kernel_trace.csv" | head -1)
python3 - $f $d <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows = [r for r in rows if "corpus" not in r["Kernel_Name"] and "idx_clear" not in r["Kernel_Name"]]
t0 = min(int(r["Start_Timestamp"]) for r in rows); t1 = max(int(r["End_Timestamp"]) for r in rows)
# take the last 45% of the trace (timed steps)
cut = t0 + (t1 - t0) * 0.55
rows = [r for r in rows if int(r["Start_Timestamp"]) >= cut]
span = (t1 - cut) / 1e6
busy = collections.defaultdict(float)
bykern = collections.defaultdict(float)
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    busy[r.get("Queue_Id", r.get("Stream_Id", "?"))] += d
    bykern[r["Kernel_Name"].split("(")[0][-28:]] += d
# union of busy time (any kernel running)
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
u, cs, ce = 0, iv[0][0], iv[0][1]
for s, e in iv[1:]:
    if s > ce: u += ce - cs; cs, ce = s, e
    else: ce = max(ce, e)
u += ce - cs
print("depth", sys.argv[2], "span %.1f ms, any-kernel busy %.1f ms (%.0f%%)" % (span, u / 1e6, 100 * u / 1e6 / span))
print("  per queue busy ms:", {k: round(v, 1) for k, v in busy.items()})
print("  top kernels ms:", {k: round(v, 1) for k, v in sorted(bykern.items(), key=lambda x: -x[1])[:8]})
PY
done
