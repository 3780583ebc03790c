#!/bin/bash
# Round 6: where the LZ4 pass's fabric traffic comes from (config 4, one step, no CPU leg): L2 requests,
# hits, memory-side read requests (all / 32-B) and write requests per lz4_seg_kernel launch.  One
# counter group per rocprofv3 run, each under its own kill timer.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
OUT=$R/gpurun_out/r06_lz4tcc
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_REQ_sum TCC_HIT_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --workload config4 --steps 1 --warmup 0 --no-cpu --no-alone --no-sub > $OUT/p$i.log 2>&1) || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i done"
done
python3 - $OUT > gpurun_out/r06_lz4tcc.txt <<'PY'
import collections, csv, glob, sys
out = sys.argv[1]
v = collections.defaultdict(list)
for f in glob.glob(f"{out}/p*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
        v[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
ks = sorted({k for k, _ in v})
cs = sorted({c for _, c in v})
print("# per-launch means (config 4, 32 x 128 MiB mixed-entropy batches, compressor 2)")
for k in ks:
    if not any(s in k for s in ("lz4", "sha_carry", "place", "gmax2")):
        continue
    print(f"{k:28s} " + " ".join(f"{c.replace('_sum', '')} {sum(v[(k, c)]) / len(v[(k, c)]):.4g}" for c in cs if v.get((k, c))))
PY
cat gpurun_out/r06_lz4tcc.txt
