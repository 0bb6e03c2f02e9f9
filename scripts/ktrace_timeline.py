"""Timeline of a slice of a rocprofv3 kernel_trace.csv: from the middle of the busiest run of
kernels (as ktrace_busy.py picks it), SPAN ms in buckets of BUCKET us; per bucket the busy fraction
and the kernels active (short names, count of overlapping instances).
    python3 scripts/ktrace_timeline.py TRACE.csv SPAN_MS BUCKET_US"""
import csv
import re
import sys
from collections import Counter

rows = list(csv.DictReader(open(sys.argv[1])))
span, bucket = float(sys.argv[2]) * 1e6, float(sys.argv[3]) * 1e3
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", r.get("Queue_Id", "?")))
            for r in rows)
segs, cur, hi = [], [], None
for x in iv:
    if hi is not None and x[0] > hi + 20e6:
        segs.append(cur)
        cur, hi = [], None
    cur.append(x)
    hi = x[1] if hi is None else max(hi, x[1])
segs.append(cur)
iv = max(segs, key=lambda sg: (sum('k_tr_a' in x[2] for x in sg), len(sg)))   # the most iterations
t0 = (iv[0][0] + max(e for _, e, _, _ in iv)) / 2
t1 = t0 + span


def short(n):
    m = re.search(r"(k_[A-Za-z0-9_]+)", n)
    return (m.group(1) if m else n[:20]).replace("k_", "")


sl = [x for x in iv if x[1] > t0 and x[0] < t1]
b = t0
while b < t1:
    e = b + bucket
    act = [x for x in sl if x[1] > b and x[0] < e]
    cov = 0
    for s_, e_, _, _ in act:
        cov += min(e_, e) - max(s_, b)
    c = Counter(short(x[2]) + "@" + str(x[3]) for x in act)
    print(f"{(b - t0)/1e3:8.0f}us busy-sum {cov/bucket:5.2f} | " + " ".join(f"{k}x{v}" for k, v in sorted(c.items())))
    b = e
