"""Average PMC counters per dispatch for kernels matching a pattern: pmc_summary.py DIR_GLOB PATTERN"""
import csv
import glob
import sys
from collections import defaultdict

pat = sys.argv[2]
acc = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:28s} n={len(v):5d} avg={sum(v)/len(v):16.1f}")
