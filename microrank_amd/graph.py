"""Host side of the PageRank graph: dicts <-> incidence arrays <-> device handle.

``trace_pagerank`` receives the four dicts of ``get_pagerank_graph``
(preprocess_data.py:146-171).  Two ways in:

* the dicts are :class:`GraphDicts` views produced by this package's
  ``get_pagerank_graph`` -- they carry the device graph built by K1, nothing is converted;
* any other mapping -- it is turned into index arrays here, with the same lookups (and
  the same ``ValueError`` on an unknown key) as the reference's dense matrix fill
  (pagerank.py:26-52), then uploaded.
"""
from __future__ import annotations

import ctypes as C
import sys
from collections.abc import Mapping
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from ._lib import GraphDesc, ptr


def _not_in_list(x) -> ValueError:
    return ValueError(f"{x!r} is not in list")


@dataclass
class HostGraph:
    nodes: list
    traces: list
    sr_off: np.ndarray      # int64 [T+1]
    sr_ops: np.ndarray      # int32
    rs_off: Optional[np.ndarray]
    rs_ops: Optional[np.ndarray]
    len_t: np.ndarray       # int32 [T]
    len_o: np.ndarray       # int32 [N]
    ss_off: np.ndarray      # int64 [N+1]
    ss_par: np.ndarray      # int32
    nchild: np.ndarray      # int32 [N]
    pr_trace: Optional[np.ndarray]   # int32, None = pr_trace is operation_trace
    pr_len: Optional[np.ndarray]

    @property
    def N(self):
        return len(self.nodes)

    @property
    def T(self):
        return len(self.traces)


def _csr(major: np.ndarray, minor: np.ndarray, n_major: int, n_minor: int):
    """Distinct (major, minor) pairs -> CSR with minors ascending."""
    if major.size == 0:
        return np.zeros(n_major + 1, np.int64), np.zeros(0, np.int32)
    key = np.unique(major.astype(np.int64) * max(n_minor, 1) + minor)
    maj = key // max(n_minor, 1)
    off = np.zeros(n_major + 1, np.int64)
    np.cumsum(np.bincount(maj, minlength=n_major), out=off[1:])
    return off, (key % max(n_minor, 1)).astype(np.int32)


def host_graph_from_dicts(operation_operation: Mapping, operation_trace: Mapping, trace_operation: Mapping,
                          pr_trace: Mapping) -> HostGraph:
    nodes = list(operation_operation.keys())
    traces = list(operation_trace.keys())
    ni = {k: i for i, k in enumerate(nodes)}
    ti = {k: i for i, k in enumerate(traces)}
    N, T = len(nodes), len(traces)

    def nget(x):
        try:
            return ni[x]
        except (KeyError, TypeError):
            raise _not_in_list(x) from None

    def tget(x):
        try:
            return ti[x]
        except (KeyError, TypeError):
            raise _not_in_list(x) from None

    # P_ss (pagerank.py:35-39): edge (child, parent), weight 1/len(children multiset of parent)
    nchild = np.zeros(N, np.int32)
    cs, ps = [], []
    for p, ch in operation_operation.items():
        pi = nget(p)
        nchild[pi] = len(ch)
        for c in ch:
            cs.append(nget(c))
            ps.append(pi)
    ss_off, ss_par = _csr(np.asarray(cs, np.int64), np.asarray(ps, np.int64), N, N)
    # P_sr (pagerank.py:42-45)
    len_t = np.fromiter((len(v) for v in operation_trace.values()), np.int32, count=T)
    flat = np.fromiter((nget(o) for v in operation_trace.values() for o in v), np.int64, count=int(len_t.sum()))
    sr_off, sr_ops = _csr(np.repeat(np.arange(T, dtype=np.int64), len_t), flat, T, N)
    # P_rs (pagerank.py:48-52)
    len_o = np.zeros(N, np.int32)
    rt, ro = [], []
    for o, trs in trace_operation.items():
        idx = [tget(t) for t in trs]   # trace looked up before the op, as at :52
        oi = nget(o)
        len_o[oi] = len(trs)
        rt.extend(idx)
        ro.extend([oi] * len(idx))
    rs_off, rs_ops = _csr(np.asarray(rt, np.int64), np.asarray(ro, np.int64), T, N)
    if rs_ops.size == sr_ops.size and np.array_equal(rs_off, sr_off) and np.array_equal(rs_ops, sr_ops):
        rs_off = rs_ops = None
    # pr_trace (pagerank.py:70-85)
    if pr_trace is operation_trace or (list(pr_trace.keys()) == traces and
                                       all(len(pr_trace[k]) == len_t[i] for i, k in enumerate(traces))):
        pr_t = pr_l = None
    else:
        pr_t = np.fromiter((tget(k) for k in pr_trace), np.int32, count=len(pr_trace))
        pr_l = np.fromiter((len(v) for v in pr_trace.values()), np.int32, count=len(pr_trace))
    return HostGraph(nodes, traces, sr_off, sr_ops, rs_off, rs_ops, len_t, len_o, ss_off, ss_par, nchild,
                     pr_t, pr_l)


class DeviceGraph:
    """An mr_graph handle (HBM-resident incidence lists) plus the host-side names."""

    def __init__(self, ctx: "_lib.Context", handle, nodes, traces, N: int, T: int):
        self.ctx = ctx
        self.h = handle
        self.nodes = nodes
        self.traces = traces
        self.N = N
        self.T = T

    @classmethod
    def upload(cls, ctx, hg: HostGraph) -> "DeviceGraph":
        lib = _lib.load()
        d = GraphDesc()
        d.n_nodes, d.n_traces = hg.N, hg.T
        keep = [np.ascontiguousarray(a) for a in (hg.sr_off, hg.sr_ops, hg.len_t, hg.len_o, hg.ss_off,
                                                  hg.ss_par, hg.nchild)]
        d.nnz_sr = int(hg.sr_ops.size)
        d.sr_off, d.sr_ops = ptr(keep[0], C.c_int64), ptr(keep[1], C.c_int32)
        d.len_t, d.len_o = ptr(keep[2], C.c_int32), ptr(keep[3], C.c_int32)
        d.n_edges = int(hg.ss_par.size)
        d.ss_off, d.ss_par, d.nchild = ptr(keep[4], C.c_int64), ptr(keep[5], C.c_int32), ptr(keep[6], C.c_int32)
        if hg.rs_off is not None:
            keep += [np.ascontiguousarray(hg.rs_off), np.ascontiguousarray(hg.rs_ops)]
            d.nnz_rs = int(hg.rs_ops.size)
            d.rs_off, d.rs_ops = ptr(keep[-2], C.c_int64), ptr(keep[-1], C.c_int32)
        if hg.pr_trace is not None:
            keep += [np.ascontiguousarray(hg.pr_trace), np.ascontiguousarray(hg.pr_len)]
            d.n_pr = int(hg.pr_trace.size)
            d.pr_trace, d.pr_len = ptr(keep[-2], C.c_int32), ptr(keep[-1], C.c_int32)
        else:
            d.n_pr = hg.T
        h = _lib.P()
        ctx.check(lib.mr_graph_upload(ctx.h, C.byref(d), C.byref(h)), "mr_graph_upload")
        return cls(ctx, h, hg.nodes, hg.traces, hg.N, hg.T)

    def pagerank(self, anomaly: bool, d: float = 0.85, alpha: float = 0.01, iters: int = 25,
                 precision: str = "fp64", exact_sums: bool = False, compress_kinds: bool = False,
                 phi: float = 0.5):
        """compress_kinds: iterate over one representative trace per kind (pagerank.py:54-66 --
        traces of a kind have identical r), the multiplicities carried; same weights.  phi: the
        anomaly preference's weight (pagerank.py:82-84)."""
        lib = _lib.load()
        prec = _lib.MR_FP32 if precision == "fp32" else _lib.MR_FP64
        flags = (_lib.MR_PR_EXACT_SUMS if exact_sums else 0) | (_lib.MR_PR_KIND_COMPRESS if compress_kinds else 0)
        if iters < 0:
            raise ValueError("iters must be >= 0")
        self.ctx.check(lib.mr_pagerank_ex(self.ctx.h, self.h, int(bool(anomaly)), float(d), float(alpha), int(iters),
                                          float(phi), prec, flags), "mr_pagerank_ex")

    def fetch(self, kinds: bool = False):
        lib = _lib.load()
        w = np.empty(self.N, np.float64)
        cov = np.empty(self.N, np.int32)
        kind = np.empty(self.T, np.float64) if kinds else None
        pref = np.empty(self.T, np.float32) if kinds else None
        self.ctx.check(lib.mr_graph_fetch(self.h, ptr(w, C.c_double), ptr(cov, C.c_int32),
                                          ptr(kind, C.c_double), ptr(pref, C.c_float)), "mr_graph_fetch")
        return (w, cov, kind, pref) if kinds else (w, cov)

    def info(self):
        n, t, nnz, e = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int64()
        _lib.load().mr_graph_info(self.h, C.byref(n), C.byref(t), C.byref(nnz), C.byref(e))
        return dict(N=n.value, T=t.value, nnz=nnz.value, E=e.value)

    def close(self):
        # a destroyed context has freed its handles already (mr_ctx_destroy)
        if getattr(self, "h", None) and getattr(getattr(self, "ctx", None), "h", None):
            _lib.load().mr_graph_free(self.h)
        self.h = None

    def __del__(self):  # pragma: no cover
        if sys.is_finalizing():   # the owning context may already be destroyed
            return
        try:
            self.close()
        except Exception:
            pass
