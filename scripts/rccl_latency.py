"""Dev tool (GPU box): latency of the library's RCCL all-reduce on one rank for the sharded
iteration's message sizes (the fused path's 2N+R u64 limbs: 160 KB at N = 10k)."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29517")

import ctypes as C  # noqa: E402

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from microrank_amd import _lib, shard  # noqa: E402

dist.init_process_group("gloo", rank=0, world_size=1)
ctx = _lib.default_context()
shard.use_rccl(ctx)
lib = _lib.load()
out = {}
for n in (1, 1024, 20_001, 200_001, 2_000_001):   # doubles: 8 B .. 16 MB
    buf = torch.zeros(n, dtype=torch.float64, device="cuda")
    p = C.cast(C.c_void_p(buf.data_ptr()), C.POINTER(C.c_double))
    for _ in range(20):
        ctx.check(lib.mr_comm_allreduce_f64(ctx.h, p, n, 0))
    ctx.sync()
    reps = 200
    t = time.perf_counter()
    for _ in range(reps):
        ctx.check(lib.mr_comm_allreduce_f64(ctx.h, p, n, 0))
    ctx.sync()
    out[f"{8 * n}B"] = round((time.perf_counter() - t) / reps * 1e6, 2)
print(json.dumps({"rccl_allreduce_us_1rank": out}))
dist.destroy_process_group()
