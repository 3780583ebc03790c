# inflate phases: kernel stats of scripts/inflate_speed.py (16 and 64 MiB files)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/infl -o run -- python3 $R/scripts/inflate_speed.py 16777216 67108864 > $R/gpurun_out/infl.log 2>&1 || { tail -20 $R/gpurun_out/infl.log; exit 1; }
cd $R
grep MiB gpurun_out/infl.log
f=$(find gpurun_out/infl -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 $f | cut -c1-150 | head -12
