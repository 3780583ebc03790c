#!/usr/bin/env python3
"""Copy/compute overlap from a rocprofv3 --kernel-trace --memory-copy-trace CSV pair: busy time of
host-to-device copies, of kernels, their union and intersection (interval arithmetic)."""
import csv
import glob
import sys


def intervals(path, filt=None):
    out = []
    for r in csv.DictReader(open(path)):
        if filt and not filt(r):
            continue
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return out


def merge(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def length(iv):
    return sum(b - a for a, b in iv)


def intersect(x, y):
    i = j = 0
    out = []
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if a < b:
            out.append([a, b])
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return out


d = sys.argv[1]
kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
mt = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)[0]
# the reduction window: from the first chunking kernel to the last kernel (excludes the corpus
# generation and the bench's own raw-copy rate measurement before it)
kraw = intervals(kt, lambda r: "corpus_kernel" not in r["Kernel_Name"])
w0 = min(a for a, _ in intervals(kt, lambda r: "gmax_kernel" in r["Kernel_Name"])) - 50_000_000   # 50 ms lead-in
w1 = max(b for _, b in kraw)
clip = lambda iv: [(max(a, w0), min(b, w1)) for a, b in iv if b > w0 and a < w1]
k = merge(clip(kraw))
c = merge(clip(intervals(mt, lambda r: "HOST_TO_DEVICE" in r.get("Direction", r.get("Operation", "HOST_TO_DEVICE")))))
t0, t1 = w0, w1
both = intersect(k, c)
print("window %.1f ms: H2D busy %.1f ms, kernels busy %.1f ms, both at once %.1f ms (%.0f %% of H2D time overlaps kernels)"
      % ((t1 - t0) / 1e6, length(c) / 1e6, length(k) / 1e6, length(both) / 1e6, 100.0 * length(both) / max(length(c), 1)))
