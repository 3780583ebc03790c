# LZ4 aggregate throughput vs pieces in flight (rocprofv3 kernel trace of scripts/lz4_scale.py)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/lzs -o run -- python3 $R/scripts/lz4_scale.py > $R/gpurun_out/lzs.log 2>&1 || { tail -20 $R/gpurun_out/lzs.log; exit 1; }
cd $R
grep MiB gpurun_out/lzs.log
f=$(find gpurun_out/lzs -name "*kernel_trace.csv" | head -1)
python3 - $f <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "lz4_list" in n:
        print(n[:40], round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, 3), "ms")
PY
