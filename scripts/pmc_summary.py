"""Mean PMC value per kernel and counter over the passes under a directory (rocprofv3 csv)."""
import collections
import csv
import glob
import sys

vals = collections.defaultdict(list)
dur = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
        vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for f in glob.glob(sys.argv[1] + "/*/*kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hdrf::", "")
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
kern = sorted({k for k, _ in vals}, key=lambda k: -sum(dur.get(k, [0])))
for k in kern[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    d = dur.get(k, [])
    print("%-32s n=%d avg_ms=%.4f" % (k[:32], len(d), sum(d) / max(len(d), 1)))
    for (kk, c), v in sorted(vals.items()):
        if kk == k:
            print("    %-24s %.4g" % (c, sum(v) / len(v)))
