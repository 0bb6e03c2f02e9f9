"""Per-kernel PMC counter totals of a rocprofv3 --pmc run: pmc_kernels.py DIR [TOP]
(FETCH_SIZE / WRITE_SIZE are in KB; FETCH_SIZE is reported x2 on gfx950 as MI355X_MICROARCH.md's
HBM section prescribes -- the bytes column applies that correction.)"""
import csv
import glob
import re
import sys
from collections import defaultdict

acc = defaultdict(lambda: [0, 0.0])
ctrs = set()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        c = r["Counter_Name"]
        ctrs.add(c)
        a = acc[(name, c)]
        a[0] += 1
        a[1] += float(r["Counter_Value"])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
for c in sorted(ctrs):
    scale = 1024.0 * (2.0 if c == "FETCH_SIZE" else 1.0)
    rows = sorted(((k[0], v) for k, v in acc.items() if k[1] == c), key=lambda x: -x[1][1])[:top]
    print(f"== {c} (bytes = value x {scale:g})")
    for name, (n, tot) in rows:
        print(f"  {name:28s} dispatches {n:6d}  avg {tot * scale / n / 1e6:10.2f} MB  total {tot * scale / 1e9:8.3f} GB")
