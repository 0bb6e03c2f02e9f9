"""Trace-sharded PageRank over several processes.

One process per GPU holds a shard of the traces (every span of a trace on one rank) over the
global node index space.  ``mr_pagerank_sharded`` (csrc/mr_pagerank.hip) exchanges, once per
graph, the per-op span counts / children counts / coverage, the call edges and the trace-kind
classes, and per iteration ONE all-reduce: the exact fixed-point P_sr r limbs (uint64 SUM) with
every rank's max r' in a one-hot slot, so every rank ends with the weights the whole graph would
give.  :func:`build_graph` builds a rank's graph from its span shard (K1 over the ranks: global
node order, cross-rank parent joins).

Collectives run over RCCL (:func:`use_rccl`, xGMI between GPUs) or, for ranks that share a GPU
or have no RCCL, over a host-staged callback on a ``torch.distributed`` process group
(:func:`use_host`; gloo in the tests).  torch is the control plane only.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import ptr

HOST_COLL = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int64, C.c_int, C.c_int)
_NP = {0: np.float64, 1: np.int32, 2: np.int64, 3: np.int64}   # uint64 reduced as int64: same bits
                                                                 # for sums mod 2^64 and for the
                                                                 # max of non-negative values


class _HostCollectives:
    """mr_host_coll_fn over a torch.distributed group; keeps the ctypes callback alive."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist, self.group = dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.fn = HOST_COLL(self._call)

    def _call(self, user, coll, buf, n, dtype, op):
        import torch

        try:
            dt = _NP[dtype]
            if coll == 0:
                a = np.ctypeslib.as_array((C.c_byte * (n * np.dtype(dt).itemsize)).from_address(buf)).view(dt)
                t = torch.from_numpy(a.copy())
                self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op else self.dist.ReduceOp.SUM, group=self.group)
                a[:] = t.numpy()
            else:
                a = np.ctypeslib.as_array(
                    (C.c_byte * (n * self.world * np.dtype(dt).itemsize)).from_address(buf)).view(dt)
                mine = torch.from_numpy(a[self.rank * n:(self.rank + 1) * n].copy())
                parts = [torch.empty_like(mine) for _ in range(self.world)]
                self.dist.all_gather(parts, mine, group=self.group)
                a[:] = torch.cat(parts).numpy()
            return 0
        except Exception:   # never raise through C
            return 1


def use_host(ctx: "_lib.Context", group=None):
    """Host-staged collectives over a torch.distributed group (any backend, e.g. gloo)."""
    hc = _HostCollectives(group)
    ctx.check(_lib.load().mr_comm_set_host(ctx.h, C.cast(hc.fn, C.c_void_p), None, hc.world, hc.rank),
              "mr_comm_set_host")
    ctx._host_coll = hc
    return hc


def use_rccl(ctx: "_lib.Context", group=None):
    """RCCL communicator for this context: rank 0's unique id travels over the torch group."""
    import torch
    import torch.distributed as dist

    lib = _lib.load()
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    uid = np.zeros(128, np.uint8)
    if rank == 0:
        ctx.check(lib.mr_comm_unique_id(ptr(uid, C.c_uint8)), "mr_comm_unique_id")
    t = torch.from_numpy(uid.copy())
    dist.broadcast(t, src=0, group=group)
    uid[:] = t.numpy()
    ctx.check(lib.mr_comm_init(ctx.h, world, rank, ptr(uid, C.c_uint8)), "mr_comm_init")


def use_peer(ctx: "_lib.Context", enable: bool = True):
    """The per-iteration all-reduce through IPC-mapped peer memory (mr_comm_peer_enable): one
    push of this rank's limbs into every rank's receive region, one local sum -- instead of the
    RCCL / host-staged all-reduce.  Needs a collective backend first (use_rccl / use_host) for the
    one-time exchange of the IPC handles."""
    ctx.check(_lib.load().mr_comm_peer_enable(ctx.h, int(bool(enable))), "mr_comm_peer_enable")


def peer_active(ctx: "_lib.Context") -> bool:
    """True while the peer path carries this context's all-reduces (its regions mapped on every
    rank); False before the first sharded call, or after the ranks fell back to RCCL / the host
    collective (a failed mapping, a peer timeout)."""
    a = C.c_int32()
    ctx.check(_lib.load().mr_comm_peer_active(ctx.h, C.byref(a)), "mr_comm_peer_active")
    return bool(a.value)


def sharded_pagerank(dg, anomaly: bool, d: float = 0.85, alpha: float = 0.01, iters: int = 25,
                     precision: str = "fp64"):
    """PageRank of the whole graph from this rank's shard ``dg`` (a DeviceGraph whose len_o /
    nchild are this rank's partial counts and whose call edges are its local ones).  Returns
    (weights, coverage) of the whole graph, identical on every rank."""
    lib = _lib.load()
    prec = _lib.MR_FP32 if precision == "fp32" else _lib.MR_FP64
    dg.ctx.check(lib.mr_pagerank_sharded(dg.ctx.h, dg.h, int(bool(anomaly)), d, alpha, iters, prec, 0),
                 "mr_pagerank_sharded")
    return dg.fetch()


def build_graph(dev_spans, trace_mask) -> "DeviceGraph":
    """K1 on this rank's span shard (mr_graph_build_sharded): ``dev_spans`` holds every span of
    this rank's traces with global codes and global row indices (SpanTable.shard);
    ``trace_mask`` selects the trace_list over the global trace codes.  The graph has the whole
    graph's node order (T10) and its cross-rank parent joins (T11); its len_o / nchild / edges are
    this rank's parts, which :func:`sharded_pagerank` combines."""
    from .graph import DeviceGraph

    lib = _lib.load()
    ctx = dev_spans.ctx
    mask = np.ascontiguousarray(trace_mask, dtype=np.uint8)
    h = _lib.P()
    ctx.check(lib.mr_graph_build_sharded(ctx.h, dev_spans.h, ptr(mask, C.c_uint8), C.byref(h)),
              "mr_graph_build_sharded")
    n, t, nnz, e = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int64()
    lib.mr_graph_info(h, C.byref(n), C.byref(t), C.byref(nnz), C.byref(e))
    node_podop = np.empty(n.value, np.int32)
    trace_code = np.empty(t.value, np.int32)
    ctx.check(lib.mr_graph_nodes(h, ptr(node_podop, C.c_int32), ptr(trace_code, C.c_int32)), "mr_graph_nodes")
    return DeviceGraph(ctx, h, node_podop, trace_code, n.value, t.value)
