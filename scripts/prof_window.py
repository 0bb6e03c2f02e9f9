"""Dev tool: run the bench window a few times (for rocprofv3 kernel traces)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from microrank_amd import _lib  # noqa: E402
from microrank_amd.preprocess_data import DeviceSpans  # noqa: E402

ctx = _lib.default_context()
topo, normal, abnormal = bench.make_window(1234, 1000, 200_000)
a3, ok = bench.slo_from_gpu(ctx, normal)
t = time.perf_counter()
bench.slo_from_gpu(ctx, normal)
print(f"slo (upload + K4, {normal.n_spans} spans): {(time.perf_counter()-t)*1e3:.2f} ms", flush=True)
dev = DeviceSpans(ctx, abnormal)
t0 = int(abnormal.tstart.min())
t1 = t0 + 5 * 60 * 10**9
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    t = time.perf_counter()
    bench.run_window(ctx, dev, t0, t1, a3, ok, 0)
    print(f"window {i}: {(time.perf_counter()-t)*1e3:.2f} ms", flush=True)
