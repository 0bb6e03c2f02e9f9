"""Kernel-by-kernel timeline of the last call in a rocprofv3 kernel_trace.csv (calls split at GPU
idle gaps > GAP us): start offset, duration and queue of each kernel, and the call's span.
    python3 scripts/call_timeline.py TRACE.csv [GAP_US]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
gap = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else 100e3
sid = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
calls, cur, hi = [], [], None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if hi is not None and s > hi + gap:
        calls.append(cur)
        cur, hi = [], None
    cur.append((s, e, r["Kernel_Name"], r[sid]))
    hi = e if hi is None else max(hi, e)
calls.append(cur)
c = [x for x in calls if any("k_tr_a" in k for _, _, k, _ in x)][-1]
t0 = c[0][0]
prev_end = t0
for s, e, k, q in c:
    m = re.search(r"(k_[A-Za-z0-9_]+|__amd_rocclr_[A-Za-z]+)", k)
    n = m.group(1) if m else k[:30]
    print(f"{(s - t0) / 1e3:8.1f} +{(e - s) / 1e3:7.1f} us  gap {(s - prev_end) / 1e3:6.1f}  q{q:>3}  {n}")
    prev_end = max(prev_end, e)
print(f"span {(max(e for _, e, _, _ in c) - t0) / 1e3:.1f} us, {len(c)} kernels")
