#!/bin/bash
# Round 5: where the index kernels' fabric traffic comes from (config 2, one step, no CPU leg): write
# requests, 64-B writes and atomics past the L2 (TCC_EA0_*), and L2 atomics, per launch of the
# claim / apply / decide / finalize kernels.  One counter group per rocprofv3 run, each under its own kill timer.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
OUT=$R/gpurun_out/r05_idxpmc
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_REQ_sum TCC_HIT_sum"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-alone --no-sub > $OUT/p$i.log 2>&1) || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i done"
done
python3 - $OUT > gpurun_out/r05_idxpmc.txt <<'PY'
import collections, csv, glob, sys
out = sys.argv[1]
v = collections.defaultdict(list)
for f in glob.glob(f"{out}/p*/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
        v[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
ks = sorted({k for k, _ in v})
cs = sorted({c for _, c in v})
print("# per-launch means (config 2, 32 x 128 MiB batches, ~4.53 M chunks per batch)")
for k in ks:
    if not any(s in k for s in ("idx_", "place", "sha_carry", "gmax2", "lane_walk")):
        continue
    print(f"{k:28s} " + " ".join(f"{c.replace('_sum', '')} {sum(v[(k, c)]) / len(v[(k, c)]):.4g}" for c in cs if v.get((k, c))))
PY
cat gpurun_out/r05_idxpmc.txt
