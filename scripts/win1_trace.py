"""One C3 window per mr_windows_batch call, N times: host wall time per call, and (run under
rocprofv3 --kernel-trace) the kernel trace the analysis below splits per call.
    python3 scripts/win1_trace.py N                      # the calls (under rocprofv3 or alone)
    python3 scripts/win1_trace.py --analyze TRACE.csv    # per call: span, busy, gaps, kernels"""
import sys
import time


def run(n):
    sys.path.insert(0, ".")
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    ctx = _lib.default_context()
    _, nrm, ab = bench.make_window(71, 500, 20_000)
    s3, sok = bench.slo_from_gpu(ctx, nrm)
    d = DeviceSpans(ctx, ab)
    u0 = int(ab.tstart.min())
    one = [(d, u0, u0 + 5 * 60 * 10**9, s3, sok)]
    for _ in range(3):
        rank_windows(ctx, one)
    ctx.sync()
    lat = []
    for _ in range(n):
        ts = time.perf_counter()
        rank_windows(ctx, one)
        ctx.sync()
        lat.append((time.perf_counter() - ts) * 1e3)
    s = sorted(lat)
    print(f"W=1 host ms: median {s[len(s) // 2]:.3f} min {s[0]:.3f}", flush=True)
    d.close()


def analyze(path):
    import csv
    import re
    from collections import defaultdict

    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # calls: runs of kernels separated by > 300 us of idle (the host's fetch between calls)
    calls, cur, hi = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if hi is not None and s > hi + 300_000:
            calls.append(cur)
            cur, hi = [], None
        cur.append((s, e, r["Kernel_Name"]))
        hi = e if hi is None else max(hi, e)
    calls.append(cur)
    calls = [c for c in calls if any("k_tr_a" in k for _, _, k in c)][-10:]
    for c in calls:
        t0, t1 = c[0][0], max(e for _, e, _ in c)
        busy, last = 0, t0
        for s, e, _ in c:   # union of intervals
            if e > last:
                busy += e - max(s, last)
                last = e
        by = defaultdict(lambda: [0, 0])
        for s, e, k in c:
            m = re.search(r"(k_[A-Za-z0-9_]+)", k)
            n = m.group(1) if m else k[:24]
            by[n][0] += 1
            by[n][1] += e - s
        top = sorted(by.items(), key=lambda x: -x[1][1])[:8]
        print(f"call: span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, {len(c)} kernels; "
              + ", ".join(f"{n} {v[0]}x{v[1] / v[0] / 1e3:.1f}" for n, v in top))


if __name__ == "__main__":
    if sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run(int(sys.argv[1]))
