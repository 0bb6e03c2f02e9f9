"""GPU busy time from a rocprofv3 kernel_trace.csv: union of kernel intervals over the last
SPAN ms of the trace (SPAN 0: the run of kernels with no gap > 20 ms that holds the most
k_tr_a launches -- the timed steps), the sum of kernel durations (concurrency = sum / union), and the
kernels' share of the sum.   python3 scripts/ktrace_busy.py TRACE.csv SPAN_MS [TOP]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
span = float(sys.argv[2]) * 1e6
top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
if span > 0:
    t_end = max(e for _, e, _ in iv)
    iv = [x for x in iv if x[0] >= t_end - span]
else:
    segs, cur, hi = [], [], None
    for x in iv:
        if hi is not None and x[0] > hi + 20e6:
            segs.append(cur)
            cur = []
        cur.append(x)
        hi = x[1] if hi is None or not cur[:-1] else max(hi, x[1])
    segs.append(cur)
    iv = max(segs, key=lambda sg: (sum('k_tr_a' in x[2] for x in sg), len(sg)))   # the most iterations
t_end = max(e for _, e, _ in iv)
busy, cur_s, cur_e, tot = 0, None, None, 0
per = defaultdict(lambda: [0, 0])
for s, e, n in iv:
    tot += e - s
    per[n[:60]][0] += e - s
    per[n[:60]][1] += 1
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
wall = t_end - iv[0][0]
print(f"window {wall/1e6:.2f} ms: kernels {len(iv)}, busy (union) {busy/1e6:.2f} ms = {busy/wall:.2%}, "
      f"sum {tot/1e6:.2f} ms (concurrency {tot/max(busy,1):.2f})")
for n, (t, c) in sorted(per.items(), key=lambda x: -x[1][0])[:top]:
    print(f"  {n:60s} {c:7d} {t/1e6:9.2f} ms {t/tot:6.1%} avg {t/c/1e3:8.2f} us")
