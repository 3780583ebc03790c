"""Summarise rocprofv3 counter CSVs: mean per dispatch per (kernel, counter)."""
import collections
import csv
import glob
import sys

d = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv") + glob.glob(sys.argv[1] + "/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
        if "rocclr" in k:
            continue
        d[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = sorted(set(k for k, _ in d))
ctrs = sorted(set(c for _, c in d))
filt = sys.argv[2].split(",") if len(sys.argv) > 2 else None
for k in kern:
    if filt and not any(x in k for x in filt):
        continue
    print(k)
    for c in ctrs:
        if (k, c) in d:
            v = d[(k, c)]
            print(f"   {c:28s} {sum(v)/len(v):14.4g}")
