"""Dev tool: time K2 on a C2-shaped graph (oracle-built structure, uploaded once)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402

from gpu_util import c2_graph, host_graph_from_oracle  # noqa: E402
from microrank_amd import _lib  # noqa: E402
from microrank_amd.graph import DeviceGraph  # noqa: E402

n_ops = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
n_tr = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
t0 = time.time()
st, sg = c2_graph(n_ops, n_tr)
g = sg.as_graph()
print(f"graph N={g.N} T={g.T} nnz={g.sr_t.size} E={g.ss_c.size} built in {time.time()-t0:.1f}s", flush=True)
ctx = _lib.default_context()
dg = DeviceGraph.upload(ctx, host_graph_from_oracle(g))
for prec in ("fp64", "fp32"):
    dg.pagerank(True, precision=prec)
    ctx.sync()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        dg.pagerank(True, precision=prec)
        ctx.sync()
        ts.append(time.perf_counter() - t)
    t = float(np.median(ts))
    edges = 25 * (2 * g.sr_t.size + g.ss_c.size)
    print(f"{prec}: trace_pagerank median {t*1e3:.3f} ms  -> {edges/t/1e9:.2f} GTEPS (whole call incl. kinds)")
if os.environ.get("ROLE_AB"):
    for mask in ("1", "2", "3", "1", "2", "3"):
        os.environ["MR_ROLE_MASK"] = mask
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            dg.pagerank(True)
            ctx.sync()
            ts.append(time.perf_counter() - t)
        print(f"role mask {mask}: median {np.median(ts)*1e3:.3f} ms")
    os.environ.pop("MR_ROLE_MASK")
