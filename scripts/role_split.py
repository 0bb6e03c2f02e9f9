"""Dev tool: per-role k_iter durations from a rocprofv3 kernel trace of
`ROLE_AB=1 python3 scripts/prof_pagerank.py N T REPS` (masks 1,2,3,1,2,3 after the fp64/fp32 runs)."""
import csv
import sys

import numpy as np

path, reps = sys.argv[1], int(sys.argv[2])
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_iter<double>" in r["Kernel_Name"]]
calls = [d[i:i + 25] for i in range(0, len(d), 25)]
phases = [("fp64 both", calls[1:1 + reps])]
base = 1 + reps
for k, m in enumerate(("1", "2", "3", "1", "2", "3")):
    phases.append((f"mask {m}", calls[base + k * reps: base + (k + 1) * reps]))
for name, cs in phases:
    a = np.array([x for c in cs for x in c])
    print(f"{name:10s} launches {a.size:4d}  median {np.median(a):7.2f} us  min {a.min():7.2f}")
