"""Drop-in for the reference module ``pagerank`` (pagerank.py).

``trace_pagerank(operation_operation, operation_trace, trace_operation, pr_trace, anomaly)``
returns ``(weight, trace_num_list)`` exactly like pagerank.py:15-112: two dicts in node
order, weights as ``np.float64``, coverage counts as ``int``.  The work runs on the GPU
(K2 in microrank_amd/csrc/mr_pagerank.hip); nothing is computed on the host except the
dict <-> index conversion for mappings that did not come from this package's
``get_pagerank_graph``.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .graph import DeviceGraph, host_graph_from_dicts

D, ALPHA, ITERATIONS = 0.85, 0.01, 25   # pagerank.py:116-117
PHI = 0.5                               # pagerank.py:82-84 (the anomaly preference's two 0.5s)


def _device_graph(operation_operation, operation_trace, trace_operation, pr_trace, ctx):
    from .preprocess_data import GraphDicts

    if isinstance(operation_operation, GraphDicts) and operation_operation.owner is not None:
        own = operation_operation.owner
        if (operation_trace is own.operation_trace and trace_operation is own.trace_operation and
                pr_trace is own.pr_trace):
            return own.device_graph(), False
    hg = host_graph_from_dicts(operation_operation, operation_trace, trace_operation, pr_trace)
    if hg.N == 0 or hg.T == 0:
        raise ValueError("zero-size array to reduction operation maximum which has no identity")
    return DeviceGraph.upload(ctx, hg), True


def trace_pagerank(operation_operation, operation_trace, trace_operation, pr_trace, anomaly, *,
                   d: float = D, alpha: float = ALPHA, iters: int = ITERATIONS, phi: float = PHI,
                   precision: str = "fp64", ctx=None, compress_kinds: bool = False):
    """pagerank.trace_pagerank on MI355X (pagerank.py:15-112).  The reference hard-codes d, alpha
    (pageRank's defaults, :116), the 25 iterations (:117) and phi (:82-84); they are keywords here
    with the reference's values as defaults.  compress_kinds: rank one representative per trace
    kind with its multiplicity (same weights within fp64 rounding)."""
    ctx = ctx or _lib.default_context()
    g, owned = _device_graph(operation_operation, operation_trace, trace_operation, pr_trace, ctx)
    try:
        g.pagerank(bool(anomaly), d, alpha, iters, precision, compress_kinds=compress_kinds, phi=phi)
        w, cov = g.fetch()
    finally:
        if owned:
            g.close()
    nodes = g.nodes
    weight = {}
    trace_num_list = {}
    for i, op in enumerate(nodes):
        trace_num_list[op] = int(cov[i])
    for i, op in enumerate(nodes):
        weight[op] = np.float64(w[i])
    return weight, trace_num_list

