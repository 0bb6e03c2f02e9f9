"""Dev tool: in-process A/B of K2 variants (env knobs) on a C2-shaped graph.
Variants: 'name=ENV=VAL,ENV=VAL' ...  Each variant runs `reps` timed calls, interleaved rounds."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402

from gpu_util import c2_graph, host_graph_from_oracle  # noqa: E402
from microrank_amd import _lib  # noqa: E402
from microrank_amd.graph import DeviceGraph  # noqa: E402

n_ops, n_tr, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
variants = []
for spec in sys.argv[4:]:
    name, _, kv = spec.partition("=")
    env = dict(x.split(":") for x in kv.split(",") if x)
    variants.append((name, env))
st, sg = c2_graph(n_ops, n_tr)
g = sg.as_graph()
ctx = _lib.default_context()
dg = DeviceGraph.upload(ctx, host_graph_from_oracle(g))
res = {n: [] for n, _ in variants}
for rnd in range(3):
    for name, env in variants:
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        dg.pagerank(True)
        ctx.sync()
        for _ in range(reps):
            t = time.perf_counter()
            dg.pagerank(True)
            ctx.sync()
            res[name].append(time.perf_counter() - t)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
for name, ts in res.items():
    print(f"{name:12s} median {np.median(ts)*1e3:.3f} ms  min {np.min(ts)*1e3:.3f} ms")
