# per-kind LZ4 kernel durations (rocprofv3 kernel trace of scripts/lz4_kinds.py)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/lzk -o run -- python3 $R/scripts/lz4_kinds.py > $R/gpurun_out/lzk.log 2>&1 || { tail -20 $R/gpurun_out/lzk.log; exit 1; }
cd $R
cat gpurun_out/lzk.log | grep MiB
f=$(find gpurun_out/lzk -name "*kernel_trace.csv" | head -1)
python3 - $f <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "lz4" in n:
        print(n[:48], round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, 3), "ms")
PY
