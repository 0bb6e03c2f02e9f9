"""One iteration's kernels from a rocprofv3 kernel_trace.csv: the launches around the middle
k_tr_a of the busiest run, start / duration relative to the first one shown (us), stream / queue.
    python3 scripts/ktrace_iter.py TRACE.csv [N_BEFORE] [N_AFTER]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 6
na = int(sys.argv[3]) if len(sys.argv) > 3 else 10
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
             r.get("Stream_Id", r.get("Queue_Id", "?"))) for r in rows)
tr = [i for i, x in enumerate(iv) if "k_tr_a" in x[2]]
mid = tr[len(tr) // 2]
sel = iv[max(0, mid - nb): mid + na]
t0 = sel[0][0]


def short(n):
    m = re.search(r"(k_[A-Za-z0-9_]+)", n)
    return m.group(1) if m else n[:30]


for s, e, n, q in sel:
    print(f"{(s - t0) / 1e3:9.1f} + {(e - s) / 1e3:8.1f} us  end {(e - t0) / 1e3:9.1f}  q {q:>3}  {short(n)}")
