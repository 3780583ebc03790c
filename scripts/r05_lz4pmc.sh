#!/bin/bash
# Round 5: PMC record of the LZ4 parse on config 4 (one step, no CPU leg), HEAD (and, when
# hdrf_amd/_build_prev exists, the lz4.hip before round 5's chain changes): wave-state and issue
# counters per lz4_seg_kernel launch, and VALU issue per SIMD-cycle = SQ_INSTS_VALU / (GRBM_GUI_ACTIVE
# / 8 XCDs x 1024 SIMDs).  One counter group per rocprofv3 run, each under its own kill timer.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
OUT=$R/gpurun_out/r05_lz4pmc
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for b in head $( [ -f $R/hdrf_amd/_build_prev/libhdrf.so ] && echo prev ); do
    if [ $b = prev ]; then E="HDRF_LIB_PATH=$R/hdrf_amd/_build_prev/libhdrf.so"; else E="X=head"; fi
    (cd /tmp && env $E timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/${b}_p$i -o run -- python3 $R/bench.py --workload config4 --steps 1 --warmup 0 --no-cpu --no-alone --no-sub > $OUT/${b}_p$i.log 2>&1) || { echo "pmc pass $i $b ($grp) failed"; tail -5 $OUT/${b}_p$i.log; exit 1; }
    echo "pass $i $b done"
  done
done
python3 - $OUT > gpurun_out/r05_lz4pmc.txt <<'PY'
import collections, csv, glob, sys
out = sys.argv[1]
for b in ("prev", "head"):
    v = collections.defaultdict(list)
    for f in glob.glob(f"{out}/{b}_p*/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
            v[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    print(f"== build {b}: per-launch means")
    for k in sorted({k for k, _ in v}):
        if not k.startswith("lz4_seg_kernel<false>"):
            continue
        m = {c: sum(x) / len(x) for (kk, c), x in v.items() if kk == k}
        n = len(v.get((k, "SQ_INSTS_VALU"), []))
        line = f"{k:22s} launches {n:3d}"
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES",
                  "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
            line += f" {c.replace('SQ_', '')} {m.get(c, float('nan')):.4g}"
        if m.get("GRBM_GUI_ACTIVE"):
            simd_cyc = m["GRBM_GUI_ACTIVE"] / 8 * 1024
            line += f" | VALU per SIMD-cycle {m['SQ_INSTS_VALU'] / simd_cyc:.4f}"
            line += f", SALU per SIMD-cycle {m.get('SQ_INSTS_SALU', 0) / simd_cyc:.4f}"
        if m.get("SQ_WAVE_CYCLES"):
            line += f", wait_frac {m.get('SQ_WAIT_ANY', 0) / m['SQ_WAVE_CYCLES']:.3f}"
        print(line)
PY
cat gpurun_out/r05_lz4pmc.txt
