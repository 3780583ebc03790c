"""Per-kernel mean counter values over rocprofv3 --pmc passes: python scripts/pmc_table.py DIR [DIR...]"""
import collections
import csv
import glob
import sys

vals = collections.defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
            vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = collections.defaultdict(dict)
for (k, c), v in vals.items():
    kern[k][c] = sum(v) / len(v)
cols = sorted({c for d in kern.values() for c in d})
print("%-28s" % "kernel" + "".join("%16s" % c[:15] for c in cols))
for k in sorted(kern):
    print("%-28s" % k[:28] + "".join("%16.4g" % kern[k].get(c, float("nan")) for c in cols))
