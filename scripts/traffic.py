"""Per-launch HBM traffic from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (scripts/pmc.sh).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  MI355X_MICROARCH.md (HBM section): on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.  Usage:
    python scripts/traffic.py gpurun_out/pmc_TAG profiles/TAG_traffic.json ['{"blocks": 512, ...}']
"""
import collections
import csv
import glob
import json
import sys

vals = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
        if r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES"):
            vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {}
for (k, c), v in sorted(vals.items()):
    d = out.setdefault(k, {})
    d[c.lower() + ("_kib_raw" if c.endswith("SIZE") else "")] = round(sum(v) / len(v), 1)
for k, d in out.items():
    f = d.get("fetch_size_kib_raw", 0.0) * 1024 * 2      # gfx950 FETCH_SIZE correction (x2)
    w = d.get("write_size_kib_raw", 0.0) * 1024
    d["hbm_bytes_per_launch"] = int(f + w)
    d["note"] = "2*FETCH_SIZE + WRITE_SIZE (KiB->B), mean per dispatch"
# the workload the passes ran (bench.py attaches these figures only to the same workload)
out["_config"] = json.loads(sys.argv[3]) if len(sys.argv) > 3 else {
    "blocks": 512, "block_mib": 128, "batch": 64, "n_gpus": 1, "hasher": 0}
json.dump(out, open(sys.argv[2], "w"), indent=1, sort_keys=True)
print(json.dumps({k: v["hbm_bytes_per_launch"] for k, v in out.items() if k != "_config"}, indent=1))
