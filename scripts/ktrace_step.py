"""Per-call critical path of mr_windows_batch from a rocprofv3 kernel_trace.csv: calls are split at
idle gaps of the GPU (> GAP us); per call, relative to its first kernel: when the auxiliary streams'
kernels (builds, spectra) end, when each PageRank group (25 k_tr_a launches on the PageRank
stream) starts and ends, and the call's length.
    python3 scripts/ktrace_step.py TRACE.csv [GAP_US]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
gap = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else 300e3
sid = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r[sid]) for r in rows)
pr_streams = {x[3] for x in iv if "k_tr_a" in x[2]}
calls, cur, hi = [], [], None
for x in iv:
    if hi is not None and x[0] > hi + gap:
        calls.append(cur)
        cur, hi = [], None
    cur.append(x)
    hi = x[1] if hi is None else max(hi, x[1])
calls.append(cur)
for c in calls:
    tra = [x for x in c if "k_tr_a" in x[2]]
    if len(tra) < 25:
        continue
    t0 = c[0][0]
    t_end = max(x[1] for x in c)
    aux = [x for x in c if x[3] not in pr_streams]
    spec = [x for x in aux if "spectrum" in x[2]]
    build = [x for x in aux if "spectrum" not in x[2]]
    groups = [tra[i:i + 25] for i in range(0, len(tra), 25)]
    busy, last = 0, t0
    for s, e, _, _ in c:
        if e > last:
            busy += e - max(s, last)
            last = e
    ms = lambda t: (t - t0) / 1e6
    print(f"call {ms(t_end):7.2f} ms  gpu busy {busy / (t_end - t0) * 100:4.1f} %  builds end {ms(max(x[1] for x in build)) if build else 0:7.2f}"
          f"  spectra {ms(min(x[0] for x in spec)) if spec else 0:6.2f}-{ms(max(x[1] for x in spec)) if spec else 0:6.2f}  groups: "
          + "  ".join(f"{ms(g[0][0]):6.2f}-{ms(g[-1][1]):6.2f}" for g in groups))
