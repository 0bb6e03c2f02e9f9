"""Dev tool: mr_windows_batch calls of W windows (C3-shaped: 500 ops / 20k traces; OPS / TRACES
override), R times, for rocprofv3 kernel stats of the window chain with little overlap (e.g.
MR_WIN_STREAMS=1, W = one chunk).   python3 scripts/prof_batch.py W R [OPS TRACES]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from microrank_amd import _lib  # noqa: E402
from microrank_amd.online_rca import rank_windows  # noqa: E402
from microrank_amd.preprocess_data import DeviceSpans  # noqa: E402

W, R = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (8, 10)
OPS, TRACES = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (500, 20_000)
ctx = _lib.default_context()
wins = []
for s in range(min(W, 4)):
    _, normal, abnormal = bench.make_window(4242 + s, OPS, TRACES)
    a3, ok = bench.slo_from_gpu(ctx, normal)
    t0 = int(abnormal.tstart.min())
    wins.append((DeviceSpans(ctx, abnormal), t0, t0 + 5 * 60 * 10**9, a3, ok))
batch = [wins[i % len(wins)] for i in range(W)]
for i in range(R):
    t = time.perf_counter()
    rank_windows(ctx, batch)
    print(f"call {i}: {W} windows {(time.perf_counter()-t)*1e3:.2f} ms", flush=True)
