#!/bin/bash
# Round 6, call 33: config-2 traffic at the round's final HEAD (whole-line walk fetch, cooperative copies, single-wave small kernels) with an SQ_INSTS_VALU pass (roofline.sha.valu for
# sha_carry_kernel<5>): profiles/r06_final_traffic.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
TAG=r06_final
ARGS="--steps 1 --warmup 0 --no-cpu --no-alone --no-sub"
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py $ARGS > $OUT/p$i.log 2>&1) || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/traffic.py $OUT gpurun_out/${TAG}_traffic.json '{"blocks": 512, "block_mib": 128, "batch": 32, "n_gpus": 1, "hasher": 0, "workload": "config2"}' > /dev/null || exit 1
grep -A3 '"sha_carry_kernel<5>"' gpurun_out/${TAG}_traffic.json | head -5
