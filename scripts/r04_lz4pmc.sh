#!/bin/bash
# Round 4: PMC record of the LZ4 table tags on config 4 (one step, no CPU leg): L2 hits/misses,
# FETCH_SIZE and wave-state counters per lz4_seg_kernel launch, HEAD vs the pre-tag build
# (HDRF_LIB_PATH=hdrf_amd/_build_notag/libhdrf.so, lz4.hip from 31ae9e2).  One counter group
# per rocprofv3 run (<= 4 TCC, <= 8 SQ), each under its own kill timer.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
OUT=$R/gpurun_out/r04_lz4pmc
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" \
           "SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for b in head notag; do
    if [ $b = notag ]; then E="HDRF_LIB_PATH=$R/hdrf_amd/_build_notag/libhdrf.so"; else E="X=head"; fi
    (cd /tmp && env $E timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/${b}_p$i -o run -- python3 $R/bench.py --workload config4 --steps 1 --warmup 0 --no-cpu --no-alone > $OUT/${b}_p$i.log 2>&1) || { echo "pmc pass $i $b ($grp) failed"; tail -5 $OUT/${b}_p$i.log; exit 1; }
    echo "pass $i $b done"
  done
done
python3 - $OUT > gpurun_out/r04_lz4pmc.txt <<'PY'
import collections, csv, glob, sys
out = sys.argv[1]
for b in ("notag", "head"):
    v = collections.defaultdict(list)
    for f in glob.glob(f"{out}/{b}_p*/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
            v[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    print(f"== build {b}: per-launch means (launches counted from the TCC pass)")
    for k in sorted({k for k, _ in v}):
        if not (k.startswith("lz4") or k.startswith("sha_chunk") or k.startswith("place")):
            continue
        m = {c: sum(x) / len(x) for (kk, c), x in v.items() if kk == k}
        n = len(v.get((k, "TCC_HIT_sum"), []))
        h, ms = m.get("TCC_HIT_sum", 0), m.get("TCC_MISS_sum", 0)
        line = f"{k[:26]:26s} launches {n:3d} TCC hit {h:.4g} miss {ms:.4g} rate {h / max(h + ms, 1):.3f}"
        line += f" FETCH_SIZE(x2, GB) {2 * m.get('FETCH_SIZE', 0) * 1024 / 1e9:.3f}"
        for c in ("SQ_INSTS_VMEM", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"):
            line += f" {c[3:]} {m.get(c, float('nan')):.4g}"
        if m.get("SQ_WAVE_CYCLES"):
            line += f" wait_frac {m.get('SQ_WAIT_ANY', 0) / m['SQ_WAVE_CYCLES']:.3f}"
        print(line)
PY
cat gpurun_out/r04_lz4pmc.txt
