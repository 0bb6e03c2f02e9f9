"""Dev tool: K2 at C4/C5 scale on one GPU -- k_iter launch time vs its algorithmic bytes.
usage: big_pagerank.py N_OPS N_TRACES [REPS]"""
import ctypes as C
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

from microrank_amd import _lib, synth  # noqa: E402
from microrank_amd.graph import DeviceGraph  # noqa: E402

n_ops, n_tr = int(sys.argv[1]), int(sys.argv[2])
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
t = time.time()
hg = synth.big_graph(n_ops, n_tr)
print(f"graph N={hg.N} T={hg.T} nnz={hg.sr_ops.size} E={hg.ss_par.size} generated in {time.time()-t:.1f}s", flush=True)
ctx = _lib.default_context()
t = time.time()
dg = DeviceGraph.upload(ctx, hg)
ctx.sync()
print(f"uploaded in {time.time()-t:.1f}s", flush=True)
lib = _lib.load()
masks = os.environ.get("ROLE_MASKS", "").split(",") if os.environ.get("ROLE_MASKS") else [None]
runs = [(p, m) for m in masks for p in (("fp64",) if m else ("fp64", "fp32"))]
for prec, mask in runs:
    if mask:
        os.environ["MR_ROLE_MASK"] = mask
    dg.pagerank(True, precision=prec)
    ctx.sync()
    lib.mr_ctx_profile(ctx.h, 1)
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        dg.pagerank(True, precision=prec)
        ctx.sync()
        ts.append(time.perf_counter() - t)
    n, ms, by = C.c_int64(), C.c_double(), C.c_double()
    lib.mr_ctx_prof_read(ctx.h, C.byref(n), C.byref(ms), C.byref(by))
    lib.mr_ctx_profile(ctx.h, 0)
    avg_us = ms.value / n.value * 1e3
    gbs = by.value / n.value / (avg_us * 1e-6) / 1e9
    edges = 25 * (2 * hg.sr_ops.size + hg.ss_par.size)
    os.environ.pop("MR_ROLE_MASK", None)
    print(f"{prec} mask={mask}: call {np.median(ts)*1e3:.2f} ms ({edges/np.median(ts)/1e9:.1f} GTEPS); k_iter {n.value} launches "
          f"avg {avg_us:.1f} us, {by.value/n.value/1e6:.1f} MB/launch -> {gbs:.0f} GB/s = {gbs/8000:.3f} of 8 TB/s",
          flush=True)
w, cov = dg.fetch()
print("weights finite:", bool(np.isfinite(w).all()), "max", float(w.max()))
