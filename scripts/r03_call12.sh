#!/bin/bash
# Round 3: config 4 (compression stage) evidence: the line WITH its CPU baseline (oracle incl. lz4 r123
# containers, container-file parity over the sample), a kernel trace, and SQ counters of the
# persistent LZ4 pass (waves, busy cycles, LDS instructions and bank conflicts, waits).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
V=${V:-v1}
timeout -k 10 900 python -u bench.py --workload config4 --steps 2 --warmup 1 --cpu-sample-blocks 16 > gpurun_out/r03_c4_$V.json.log 2>&1 || { tail -20 gpurun_out/r03_c4_$V.json.log; exit 1; }
tail -1 gpurun_out/r03_c4_$V.json.log | python3 -c "import json,sys; d=json.load(sys.stdin); print('config4', d['value'], d['cpu_baseline'])"
TAG=r03_c4prof_$V BENCH="--workload config4 --steps 1 --warmup 1 --no-cpu" bash scripts/r02_prof.sh > gpurun_out/r03_c4prof_$V.txt 2>&1 || { tail -20 gpurun_out/r03_c4prof_$V.txt; exit 1; }
head -12 gpurun_out/r03_c4prof_$V.txt | cut -c1-160
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out/pmc_r03_c4_$V; mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --workload config4 --blocks 64 --steps 1 --warmup 0 --no-cpu > $OUT/p$i.log 2>&1) || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_table.py $OUT | grep -E "kernel|lz4|sha|place|gmax"
