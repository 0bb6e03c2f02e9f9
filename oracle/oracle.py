"""ORACLE -- TEST INFRASTRUCTURE ONLY.

CPU restatement of MicroRank's ranking path (reference @ /root/reference), used by
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg as the
CHECKER.  The product (``microrank_amd``) never imports, links or executes anything
under ``oracle/``.

Pinning: every function here is checked against golden vectors captured by running
the reference itself in the dev container (``tests/golden/make_golden.py``; fixtures
``tests/golden/*.json``) -- see ``tests/test_oracle_golden.py``.

Each function cites the reference lines it restates.  Semantics decoded in
SURVEY.md §8.1 (T1..T17).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

D_DEFAULT = 0.85      # pagerank.py:116
ALPHA_DEFAULT = 0.01  # pagerank.py:116
ITERS_DEFAULT = 25    # pagerank.py:117


def _index_error(x) -> ValueError:
    return ValueError(f"{x!r} is not in list")  # what list.index raises (pagerank.py:39,45,52)


@dataclass
class Graph:
    """Index form of the four graph dicts (pagerank.py:16-52 without the dense matrices).

    Node order = operation_operation key order; trace order = operation_trace key order.
    ``sr`` is the incidence P_sr (op o in operation_trace[t]), ``rs`` is P_rs
    (t in trace_operation[o]).  They coincide for graphs built by get_pagerank_graph.
    """
    nodes: list
    traces: list
    sr_t: np.ndarray            # int64 trace index per distinct (o,t) pair, sorted by (t,o)
    sr_o: np.ndarray            # int64 op index, same pairs
    rs_t: np.ndarray
    rs_o: np.ndarray
    len_t: np.ndarray           # int64 len(operation_trace[t])      -> P_sr value fp32(1/len_t)
    len_o: np.ndarray           # int64 len(trace_operation[o]) (0 if op not a key) -> P_rs value
    ss_c: np.ndarray            # int64 child index per distinct (child,parent) pair
    ss_p: np.ndarray            # int64 parent index
    nchild: np.ndarray          # int64 len(operation_operation[p])  -> P_ss value fp32(1/nchild)
    pr_idx: np.ndarray          # int64 trace index per pr_trace key, in pr_trace order
    pr_len: np.ndarray          # int64 len(pr_trace[key])

    @property
    def N(self) -> int:
        return len(self.nodes)

    @property
    def T(self) -> int:
        return len(self.traces)


def graph_from_dicts(operation_operation, operation_trace, trace_operation, pr_trace) -> Graph:
    """pagerank.py:16-52 -- same lookups, same ValueError on an unknown key."""
    nodes = list(operation_operation.keys())
    traces = list(operation_trace.keys())
    ni = {k: i for i, k in enumerate(nodes)}
    ti = {k: i for i, k in enumerate(traces)}

    def nget(x):
        try:
            return ni[x]
        except (KeyError, TypeError):
            raise _index_error(x) from None

    def tget(x):
        try:
            return ti[x]
        except (KeyError, TypeError):
            raise _index_error(x) from None

    N, T = len(nodes), len(traces)
    # :35-39 P_ss[child][parent] = 1/len(children)
    ss = set()
    nchild = np.zeros(N, dtype=np.int64)
    for p, ch in operation_operation.items():
        pi = nget(p)
        nchild[pi] = len(ch)
        for c in ch:
            ss.add((nget(c), pi))
    # :42-45 P_sr[op][trace] = 1/len(ops of trace)
    sr = set()
    len_t = np.zeros(T, dtype=np.int64)
    for t, ops in operation_trace.items():
        tix = tget(t)
        len_t[tix] = len(ops)
        for o in ops:
            sr.add((tix, nget(o)))
    # :48-52 P_rs[trace][op] = 1/len(traces of op)
    rs = set()
    len_o = np.zeros(N, dtype=np.int64)
    for o, trs in trace_operation.items():
        oi = nget(o)
        len_o[oi] = len(trs)
        for t in trs:
            rs.add((tget(t), oi))
    pr_idx = np.array([tget(t) for t in pr_trace], dtype=np.int64)
    pr_len = np.array([len(v) for v in pr_trace.values()], dtype=np.int64)

    def arr(pairs, k):
        a = np.array(sorted(pairs), dtype=np.int64).reshape(-1, 2)
        return a[:, 0], a[:, 1]

    sr_t, sr_o = arr(sr, 2)
    rs_t, rs_o = arr(rs, 2)
    ss_arr = np.array(sorted(ss), dtype=np.int64).reshape(-1, 2)
    return Graph(nodes, traces, sr_t, sr_o, rs_t, rs_o, len_t, len_o, ss_arr[:, 0], ss_arr[:, 1],
                 nchild, pr_idx, pr_len)


def trace_kinds(g: Graph) -> np.ndarray:
    """pagerank.py:54-66: kind[t] = number of traces whose P_sr column equals t's column.
    Column t is fp32(1/len_t) on the op set of t (T6) -> key (op set, fp32 bits)."""
    w = (1.0 / np.maximum(g.len_t, 1)).astype(np.float32)
    keys = {}
    order = np.lexsort((g.sr_o, g.sr_t))
    sets = [[] for _ in range(g.T)]
    for t, o in zip(g.sr_t[order], g.sr_o[order]):
        sets[t].append(int(o))
    kid = np.empty(g.T, dtype=np.int64)
    for t in range(g.T):
        key = (tuple(sets[t]), w[t].view(np.uint32).item() if sets[t] else 0)
        kid[t] = keys.setdefault(key, len(keys))
    counts = np.bincount(kid, minlength=len(keys))
    return counts[kid].astype(np.float64)


def preference(g: Graph, kind: np.ndarray, anomaly: bool, phi: float = 0.5) -> np.ndarray:
    """pagerank.py:68-85 -- sequential fp64 sums in pr_trace order (T7), stored as fp32.  phi: the
    two 0.5 weights of the anomaly form (:82-84), a keyword of the build's surface."""
    pr = np.zeros(g.T, dtype=np.float32)
    if not anomaly:
        s = 0.0
        for t in g.pr_idx:
            s += 1.0 / kind[t]
        for t in g.pr_idx:
            pr[t] = 1.0 / kind[t] / s
    else:
        ks = 0.0
        ns = 0.0
        for t, ln in zip(g.pr_idx, g.pr_len):
            ks += 1.0 / kind[t]
            ns += 1.0 / ln  # ZeroDivisionError for an empty list, as in the reference
        for t, ln in zip(g.pr_idx, g.pr_len):
            pr[t] = 1.0 / (kind[t] / ks * phi + 1.0 / ln) / ns * phi
    return pr


def _amax(x):
    if x.size == 0:
        raise ValueError("zero-size array to reduction operation maximum which has no identity")
    return np.max(x)


def power_iteration(g: Graph, v: np.ndarray, d: float = D_DEFAULT, alpha: float = ALPHA_DEFAULT,
                    iters: int = ITERS_DEFAULT, precision: str = "fp64") -> np.ndarray:
    """pagerank.py:116-130 (Jacobi update T8, max normalisation T3, fp32 (1-d)*v term T4).

    ``precision='fp32'`` keeps the vectors in float32 (the build's fp32 mode, 1e-4 target)."""
    N, T = g.N, g.T
    ft = np.float64 if precision == "fp64" else np.float32
    w_sr = (1.0 / np.maximum(g.len_t, 1)).astype(np.float32).astype(ft)[g.sr_t]
    w_rs = (1.0 / np.maximum(g.len_o, 1)).astype(np.float32).astype(ft)[g.rs_o]
    w_ss = (1.0 / np.maximum(g.nchild, 1)).astype(np.float32).astype(ft)[g.ss_p]
    s = (np.ones(N) / float(N + T)).astype(ft)
    r = (np.ones(T) / float(N + T)).astype(ft)
    c = ((1.0 - d) * v.astype(np.float32)).astype(ft)   # float32 product (NEP 50), then upcast
    d_, a_ = ft(d), ft(alpha)
    for _ in range(iters):
        sr = np.bincount(g.sr_o, weights=w_sr * r[g.sr_t], minlength=N).astype(ft)
        ss = np.bincount(g.ss_c, weights=w_ss * s[g.ss_p], minlength=N).astype(ft)
        rs = np.bincount(g.rs_t, weights=w_rs * s[g.rs_o], minlength=T).astype(ft)
        s_new = d_ * (sr + a_ * ss)
        r_new = d_ * rs + c
        s = s_new / _amax(s_new)
        r = r_new / _amax(r_new)
    return (s / _amax(s)).astype(np.float64)


def weights(g: Graph, s: np.ndarray):
    """pagerank.py:93-112: weight = s * sum(s) / N with a sequential node-order sum (T9);
    trace_num_list = distinct traces containing the op (nonzeros of the P_sr row)."""
    total = 0
    for i in range(g.N):
        total += s[i]
    cov = np.bincount(g.sr_o, minlength=g.N)
    weight = {}
    num = {}
    for i, op in enumerate(g.nodes):
        num[op] = int(cov[i])
    for i, op in enumerate(g.nodes):
        weight[op] = np.float64(s[i] * total / g.N)
    return weight, num


def trace_pagerank(operation_operation, operation_trace, trace_operation, pr_trace, anomaly,
                   precision: str = "fp64", d: float = D_DEFAULT, alpha: float = ALPHA_DEFAULT,
                   iters: int = ITERS_DEFAULT, phi: float = 0.5):
    """pagerank.trace_pagerank (pagerank.py:15-112); d / alpha / iters / phi default to the
    reference's hard-coded values (:116-117, :82-84)."""
    g = graph_from_dicts(operation_operation, operation_trace, trace_operation, pr_trace)
    kind = trace_kinds(g)
    v = preference(g, kind, anomaly, phi)
    s = power_iteration(g, v, d, alpha, iters, precision=precision)
    return weights(g, s)


# ----------------------------------------------------------------------------- spans -> graph
@dataclass
class SpanGraph:
    """get_pagerank_graph restated on int codes (preprocess_data.py:146-171)."""
    node_podop: np.ndarray      # podop code per node, node order (T10)
    trace_codes: np.ndarray     # sorted trace codes present
    sr_t: np.ndarray            # distinct (trace idx, node idx) pairs sorted by (t, o)
    sr_o: np.ndarray
    len_t: np.ndarray           # spans per trace
    len_o: np.ndarray           # spans per node
    ss_c: np.ndarray            # distinct (child node, parent node), sorted (c, p)
    ss_p: np.ndarray
    nchild: np.ndarray          # children-multiset size per node (0 for never-parents)
    n_parents: int              # nodes [0, n_parents) are the sorted parent ops
    rows: np.ndarray = field(default=None)   # filtered row indices (row order)
    node_of_row: np.ndarray = field(default=None)
    tidx_of_row: np.ndarray = field(default=None)

    def as_graph(self) -> Graph:
        return Graph(list(self.node_podop), list(self.trace_codes), self.sr_t, self.sr_o, self.sr_t,
                     self.sr_o, self.len_t, self.len_o, self.ss_c, self.ss_p, self.nchild,
                     np.arange(len(self.trace_codes), dtype=np.int64), self.len_t.copy())


def span_graph(trace: np.ndarray, podop: np.ndarray, span: np.ndarray, parent: np.ndarray,
               selected: np.ndarray) -> SpanGraph:
    """``selected``: bool per trace code (the trace_list membership, preprocess_data.py:148).

    * preprocess_data.py:157-158 merge ParentSpanId == spanID over the filtered spans, traceID
      ignored (T11): duplicated spanIDs fan out, orphans give no edge.
    * :159 groupby(parent op) sorts parents by name; :160-163 never-parent ops follow in
      first-appearance row order (T10).
    * :165-169 trace keys sorted; list entries one per span.
    """
    rows = np.flatnonzero(selected[trace])
    op = podop[rows].astype(np.int64)
    sp = span[rows]
    par = parent[rows]
    # multimap spanID -> filtered rows
    order = np.argsort(sp, kind="stable")
    sp_sorted = sp[order]
    lo = np.searchsorted(sp_sorted, par, side="left")
    hi = np.searchsorted(sp_sorted, par, side="right")
    has = (par >= 0) & (hi > lo)
    cnt = np.where(has, hi - lo, 0)
    child_rows = np.repeat(np.arange(rows.size), cnt)
    starts = np.repeat(lo, cnt)
    local = np.arange(child_rows.size) - np.repeat(np.cumsum(cnt) - cnt, cnt)
    parent_rows = order[starts + local]
    e_child_op = op[child_rows]
    e_parent_op = op[parent_rows]
    parent_ops = np.unique(e_parent_op)            # sorted by code == sorted by name
    # node order
    uniq_ops, first = np.unique(op, return_index=True)
    is_par = np.isin(uniq_ops, parent_ops)
    rest = uniq_ops[~is_par][np.argsort(first[~is_par], kind="stable")]
    node_podop = np.concatenate([parent_ops, rest])
    node_of_code = {int(c): i for i, c in enumerate(node_podop)}
    remap = np.vectorize(lambda c: node_of_code[int(c)], otypes=[np.int64]) if op.size else None
    node = remap(op) if op.size else np.zeros(0, np.int64)
    N = node_podop.size
    nchild = np.bincount(remap(e_parent_op), minlength=N) if e_parent_op.size else np.zeros(N, np.int64)
    if e_child_op.size:
        pairs = np.unique(np.stack([remap(e_child_op), remap(e_parent_op)], 1), axis=0)
    else:
        pairs = np.zeros((0, 2), np.int64)
    trace_codes, tidx = np.unique(trace[rows], return_inverse=True)
    tidx = tidx.astype(np.int64)
    len_t = np.bincount(tidx, minlength=trace_codes.size)
    len_o = np.bincount(node, minlength=N)
    pair_sr = np.unique(np.stack([tidx, node], 1), axis=0) if rows.size else np.zeros((0, 2), np.int64)
    return SpanGraph(node_podop.astype(np.int64), trace_codes.astype(np.int64), pair_sr[:, 0], pair_sr[:, 1],
                     len_t.astype(np.int64), len_o.astype(np.int64), pairs[:, 0], pairs[:, 1],
                     nchild.astype(np.int64), int(parent_ops.size), rows, node, tidx)


def span_graph_dicts(sg: SpanGraph, span: np.ndarray, parent: np.ndarray, podop_names, trace_names):
    """The four dicts of preprocess_data.py:158-171 from a SpanGraph: list entries one per span
    in row order; children in merge order (child row order, then matching parent rows)."""
    nodes = [podop_names[c] for c in sg.node_podop]
    tn = [trace_names[c] for c in sg.trace_codes]
    rows = sg.rows
    ot = {t: [] for t in tn}
    for ti, ni in zip(sg.tidx_of_row, sg.node_of_row):
        ot[tn[ti]].append(nodes[ni])
    to = {n: [] for n in sorted(nodes)}
    for ti, ni in zip(sg.tidx_of_row, sg.node_of_row):
        to[nodes[ni]].append(tn[ti])
    oo = {n: [] for n in nodes}
    sp = span[rows]
    order = np.argsort(sp, kind="stable")
    srt = sp[order]
    par = parent[rows]
    lo = np.searchsorted(srt, par, "left")
    hi = np.searchsorted(srt, par, "right")
    for i in range(rows.size):
        if par[i] < 0:
            continue
        for j in order[lo[i]:hi[i]]:
            oo[nodes[sg.node_of_row[j]]].append(nodes[sg.node_of_row[i]])
    return oo, ot, to, dict(ot)


# ----------------------------------------------------------------------------- spectrum
SPECTRUM_METHODS = ("dstar2", "ochiai", "jaccard", "sorensendice", "m1", "m2", "goodman",
                    "tarantula", "russellrao", "hamann", "dice", "simplematcing", "rogers")


def spectrum(anomaly_result, normal_result, anomaly_list_len, normal_list_len, top_max,
             normal_num_list, anomaly_num_list, spectrum_method):
    """online_rca.py:33-152 -- returns (top_list, score_list, printed_lines)."""
    sp = {}
    for node in anomaly_result:                       # online_rca.py:45-58
        a = anomaly_result[node]
        e = {"ef": a * anomaly_num_list[node], "nf": a * (anomaly_list_len - anomaly_num_list[node])}
        if node in normal_result:
            n = normal_result[node]
            e["ep"] = n * normal_num_list[node]
            e["np"] = n * (normal_list_len - normal_num_list[node])
        else:
            e["ep"] = 0.0000001
            e["np"] = 0.0000001
        sp[node] = e
    for node in normal_result:                        # online_rca.py:60-69
        if node not in sp:
            n = normal_result[node]
            sp[node] = {"ep": (1 + n) * normal_num_list[node], "np": normal_list_len - normal_num_list[node],
                        "ef": 0.0000001, "nf": 0.0000001}
    res = {}
    m = spectrum_method
    for node, e in sp.items():                        # online_rca.py:75-142
        ef, nf, ep, np_ = e["ef"], e["nf"], e["ep"], e["np"]
        if m == "dstar2":
            res[node] = ef * ef / (ep + nf)
        elif m == "ochiai":
            res[node] = ef / math.sqrt((ep + ef) * (ef + nf))
        elif m == "jaccard":
            res[node] = ef / (ef + ep + nf)
        elif m == "sorensendice":
            res[node] = 2 * ef / (2 * ef + ep + nf)
        elif m == "m1":
            res[node] = (ef + np_) / (ep + nf)
        elif m == "m2":
            res[node] = ef / (2 * ep + 2 * nf + ef + np_)
        elif m == "goodman":
            res[node] = (2 * ef - nf - ep) / (2 * ef + nf + ep)
        elif m == "tarantula":
            res[node] = ef / (ef + nf) / (ef / (ef + nf) + ep / (ep + np_))
        elif m == "russellrao":
            res[node] = ef / (ef + nf + ep + np_)
        elif m == "hamann":
            res[node] = (ef + np_ - ep - nf) / (ef + nf + ep + np_)
        elif m == "dice":
            res[node] = 2 * ef / (ef + nf + ep)
        elif m == "simplematcing":
            res[node] = (ef + np_) / (ef + np_ + nf + ep)
        elif m == "rogers":
            res[node] = (ef + np_) / (ef + np_ + 2 * nf + 2 * ep)
    top, score, lines = [], [], []
    for i, (k, v) in enumerate(sorted(res.items(), key=lambda x: x[1], reverse=True)):  # :147-150, stable
        if i < top_max + 6:
            top.append(k)
            score.append(v)
            lines.append("%-50s: %.8f" % (k, v))
    return top, score, lines


# ----------------------------------------------------------------------------- SLO / detector
def numpy_pairwise_sum(x: np.ndarray) -> float:
    """numpy's pairwise float64 summation (numpy/_core/src/umath/loops_utils.h.src,
    PW_BLOCKSIZE 128, 8 accumulators) -- the order np.std's umr_sum uses on a contiguous
    float64 array."""
    n = x.size
    if n < 8:
        r = 0.0 if n == 0 else x[0] - 0.0
        r = 0.0
        for i in range(n):
            r += x[i]
        return r
    if n <= 128:
        acc = [x[j] for j in range(8)]
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                acc[j] += x[i + j]
            i += 8
        r = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]))
        while i < n:
            r += x[i]
            i += 1
        return r
    n2 = n // 2
    n2 -= n2 % 8
    return numpy_pairwise_sum(x[:n2]) + numpy_pairwise_sum(x[n2:])


NPY_BUFSIZE = 8192   # numpy's default ufunc buffer (numpy/_core/include/numpy/ndarraytypes.h)


def numpy_reduce_sum(x: np.ndarray) -> float:
    """np.add.reduce of a 1-D float64 array as numpy runs it: the reduction loop is handed the
    array in NPY_BUFSIZE-element pieces, each piece summed pairwise (numpy_pairwise_sum) into the
    running accumulator (DOUBLE_add's ``io1 += pairwise_sum(...)``).  For n <= 8192 this is the
    plain pairwise sum; np.var / np.std use it for the squared deviations (pinned by
    tests/golden/slo_large.json, produced by the reference's get_operation_slo)."""
    acc = 0.0
    for i in range(0, x.size, NPY_BUFSIZE):
        acc += numpy_pairwise_sum(x[i:i + NPY_BUFSIZE])
    return acc


def np_round4(x: float) -> float:
    """round(np.float64, 4) == rint(x*1e4)/1e4 (T13)."""
    return float(np.rint(x * 10000.0) / 10000.0)


def operation_slo(svcop: np.ndarray, duration: np.ndarray, svcop_names, operation_list) -> dict:
    """preprocess_data.get_operation_slo (preprocess_data.py:50-78): per service-op [round(mean/1000,4),
    round(std/1000,4)], population std, keys in sorted name order filtered by operation_list."""
    keep = set(operation_list)
    out = {}
    order = np.argsort(svcop, kind="stable")          # groupby keeps row order inside a group
    codes = svcop[order]
    bounds = np.flatnonzero(np.diff(codes)) + 1
    for seg in np.split(order, bounds):
        if seg.size == 0:
            continue
        name = svcop_names[svcop[seg[0]]]
        if name not in keep:
            continue
        d = duration[seg].astype(np.int64)
        mean = float(d.sum()) / d.size
        dev = d.astype(np.float64) - mean
        var = numpy_reduce_sum(dev * dev) / d.size
        out[name] = [np.float64(np_round4(mean / 1000.0)), np.float64(np_round4(math.sqrt(var) / 1000.0))]
    return dict(sorted(out.items()))


def detect(trace: np.ndarray, svcop: np.ndarray, duration: np.ndarray, tstart, tend, t0: int, t1: int,
           slo_mean_plus3std: Dict[int, float]):
    """anormaly_detector.system_anomaly_detect (anormaly_detector.py:44-84) + get_operation_duration_data
    (preprocess_data.py:97-122):
    window on trace-level times (inclusive, T15); per trace real = max duration / 1000,
    expect = sum over ops in sorted name order of count * (mean + 3 std) (T14); traces with
    max duration <= 0 dropped.  Returns (flag, abnormal codes, normal codes) in sorted order,
    or None for an empty window."""
    m = (tstart >= t0) & (tend <= t1)
    if not m.any():
        return None
    tr, op, du = trace[m], svcop[m], duration[m]
    codes = np.unique(tr)
    ab, no = [], []
    key = tr.astype(np.int64) * (int(op.max()) + 1) + op
    uk, cnt = np.unique(key, return_counts=True)
    per_trace_ops = {}
    nops = int(op.max()) + 1
    for k, c in zip(uk, cnt):
        per_trace_ops.setdefault(int(k // nops), []).append((int(k % nops), int(c)))
    mx = {}
    for t, d in zip(tr, du):
        mx[int(t)] = max(mx.get(int(t), d), d)
    for t in codes:
        t = int(t)
        if not mx[t] > 0:
            continue
        real = float(mx[t]) / 1000.0
        exp = 0.0
        for o, c in per_trace_ops[t]:
            if o in slo_mean_plus3std:
                exp += c * slo_mean_plus3std[o]
        (ab if real > exp else no).append(t)
    return bool(ab), ab, no


def driver_sweep(trace, svcop, duration, tstart, tend, slo_mean_plus3std: Dict[int, float], *,
                 step_normal: int = 5 * 60 * 10**9, step_abnormal: int = 4 * 60 * 10**9):
    """The window chain of online_rca.online_anomaly_detect_RCA (online_rca.py:161-216): windows
    [t, t + 5 min] from min(startTime) while t < max(endTime); a window whose detector flags an
    anomaly with both lists non-empty is ranked and the next starts 9 minutes later, otherwise 5
    (:170-178, :215-216).  Returns [(t0, flag, abnormal codes, normal codes, ranked)] and True
    when the chain ended in an empty window (the detector's False: the driver's TypeError, T2)."""
    t, end = int(tstart.min()), int(tend.max())
    out = []
    while t < end:
        r = detect(trace, svcop, duration, tstart, tend, t, t + step_normal, slo_mean_plus3std)
        if r is None:
            return out, True
        flag, ab, no = r
        ranked = bool(flag and ab and no)
        out.append((t, flag, ab, no, ranked))
        t += step_normal + (step_abnormal if ranked else 0)
    return out, False


# ----------------------------------------------------------------------------- trace sharding
def sharded_pagerank(g: Graph, comm, anomaly: bool, d: float = D_DEFAULT, alpha: float = ALPHA_DEFAULT,
                     iters: int = ITERS_DEFAULT):
    """The multi-GPU decomposition restated on CPU: ``g`` holds THIS rank's
    traces (every span of a trace on one rank) over the GLOBAL node index space.  ``comm`` offers
    sum(np.ndarray) / max(float) / gather(obj) across ranks.  Per iteration one SUM of the N-length
    partial P_sr.r vector and one MAX of r'; everything else (len_o, nchild, coverage, kind classes,
    preference sums) is reduced once.  Returns (s, coverage) identical on every rank."""
    N = g.N
    len_o = comm.sum(g.len_o.astype(np.float64)).astype(np.int64)
    nchild = comm.sum(g.nchild.astype(np.float64)).astype(np.int64)
    cov = comm.sum(np.bincount(g.sr_o, minlength=N).astype(np.float64)).astype(np.int64)
    edges = set()
    for part in comm.gather(list(zip(g.ss_c.tolist(), g.ss_p.tolist()))):
        edges.update(map(tuple, part))
    ss = np.array(sorted(edges), dtype=np.int64).reshape(-1, 2)
    # kinds: global class sizes of the (op set, fp32(1/len)) keys
    w32 = (1.0 / np.maximum(g.len_t, 1)).astype(np.float32)
    sets = [[] for _ in range(g.T)]
    for t, o in zip(g.sr_t, g.sr_o):
        sets[t].append(int(o))
    keys = [(tuple(sorted(sets[t])), w32[t].view(np.uint32).item() if sets[t] else 0) for t in range(g.T)]
    counts = {}
    for part in comm.gather(keys):
        for k in part:
            counts[k] = counts.get(k, 0) + 1
    kind = np.array([counts[k] for k in keys], dtype=np.float64)
    # preference sums: global
    if not anomaly:
        S = comm.sum(np.array([np.sum(1.0 / kind)]))[0]
        v = (1.0 / kind / S).astype(np.float32)
    else:
        KS, NS = comm.sum(np.array([np.sum(1.0 / kind), np.sum(1.0 / g.len_t)]))
        v = (1.0 / (kind / KS * 0.5 + 1.0 / g.len_t) / NS * 0.5).astype(np.float32)
    T_global = int(comm.sum(np.array([float(g.T)]))[0])
    w_sr = (1.0 / np.maximum(g.len_t, 1)).astype(np.float32).astype(np.float64)[g.sr_t]
    w_rs = (1.0 / np.maximum(len_o, 1)).astype(np.float32).astype(np.float64)[g.sr_o]
    w_ss = (1.0 / np.maximum(nchild, 1)).astype(np.float32).astype(np.float64)[ss[:, 1]]
    s = np.ones(N) / float(N + T_global)
    r = np.ones(g.T) / float(N + T_global)
    c = ((1.0 - d) * v).astype(np.float64)
    for _ in range(iters):
        part = np.bincount(g.sr_o, weights=w_sr * r[g.sr_t], minlength=N)
        sr = comm.sum(part)
        ssv = np.bincount(ss[:, 0], weights=w_ss * s[ss[:, 1]], minlength=N)
        rs = np.bincount(g.sr_t, weights=w_rs * s[g.sr_o], minlength=g.T)
        s_new = d * (sr + alpha * ssv)
        r_new = d * rs + c
        mr = comm.max(float(np.max(r_new)) if r_new.size else -np.inf)
        s = s_new / np.max(s_new)
        r = r_new / mr
    return s / np.max(s), cov
