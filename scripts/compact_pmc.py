"""Reduce a rocprofv3 PMC pass directory to one row per (kernel, counter): the mean over its dispatches, written
back as run_counter_collection.csv with the columns scripts/summarize_profile.py reads (the per-dispatch file of a
training step is tens of MB; gpurun copies back at most 64 MiB).   usage: python3 scripts/compact_pmc.py <dir>"""
import collections
import csv
import glob
import os
import sys

for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    acc = collections.defaultdict(lambda: [0.0, 0])
    with open(f) as fh:
        for r in csv.DictReader(fh):
            a = acc[(r["Kernel_Name"], r["Counter_Name"])]
            a[0] += float(r["Counter_Value"])
            a[1] += 1
    os.remove(f)
    with open(os.path.join(sys.argv[1], "run_counter_collection.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value", "Dispatches"])
        for (k, c), (v, n) in sorted(acc.items()):
            w.writerow([k, c, v / n, n])
