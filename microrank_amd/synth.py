"""Deterministic synthetic span generator.

A Train-Ticket-like call tree whose root service is ``ts-ui-dashboard`` (REST op
names ending in an id segment, to exercise the ``rsplit('/')`` naming rule of
preprocess_data.py:28-30).  Every trace is a random walk down the tree from the
root: each child is visited with probability ``min(p_max, branch/fanout)`` and a
visited child is called a second time with probability ``p_repeat`` (span
multiplicity, T5).  A span's duration is its own work plus its children's, so the
root span carries the trace latency.  One faulty operation gets ``+fault_ms`` in a
fraction of traces, which is what the 3-sigma detector (anormaly_detector.py:56-73)
flags.

Generation is vectorised level by level over all traces, so the 200k-trace C2
window and the 10M-trace C4 graph are generated in numpy without Python per-span
loops.  Output is an int-coded :class:`SpanTable`; :func:`to_dataframe` materialises
the reference's string schema for parity runs at small sizes.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import os

import numpy as np

from .spans import UI_SERVICE, SpanTable

NS_PER_MIN = 60 * 1_000_000_000


@dataclass
class Topology:
    n_ops: int
    parent: np.ndarray          # int32 [n_ops], -1 for the root
    depth: np.ndarray           # int32 [n_ops]
    child_off: np.ndarray       # int64 [n_ops+1]  CSR of the op tree
    child_ids: np.ndarray       # int32
    service: np.ndarray         # int32 [n_ops]   service index (0 = ts-ui-dashboard)
    base_ms: np.ndarray         # float64 [n_ops] mean self time
    op_names: list              # raw operationName stem per op
    svc_names: list
    pods_per_service: int


def make_topology(n_ops: int, seed: int = 0, *, zipf_s: float = 0.0, max_depth: int = 8,
                  pods_per_service: int = 1) -> Topology:
    """Random recursive call tree.  ``zipf_s>0`` gives power-law fan-out (C4/C5)."""
    rng = np.random.default_rng([seed, 0x70])
    parent = np.full(n_ops, -1, dtype=np.int32)
    depth = np.zeros(n_ops, dtype=np.int32)
    ok = np.zeros(n_ops, dtype=bool)
    ok[0] = True
    for i in range(1, n_ops):
        cand = np.flatnonzero(ok[:i])
        if zipf_s > 0:
            w = (cand + 1.0) ** (-zipf_s)
            j = cand[np.searchsorted(np.cumsum(w), rng.random() * w.sum(), side="right").clip(0, len(cand) - 1)]
        else:
            j = cand[rng.integers(0, len(cand))]
        parent[i] = j
        depth[i] = depth[j] + 1
        ok[i] = depth[i] < max_depth
    order = np.argsort(parent[1:], kind="stable") + 1
    counts = np.bincount(parent[1:], minlength=n_ops)
    child_off = np.zeros(n_ops + 1, dtype=np.int64)
    np.cumsum(counts, out=child_off[1:])
    child_ids = order.astype(np.int32)
    # two operations per service; service 0 is the UI gateway
    service = (np.arange(n_ops) // 2).astype(np.int32)
    n_svc = int(service.max()) + 1
    svc_names = [UI_SERVICE] + [f"ts-svc{s:05d}-service" for s in range(1, n_svc)]
    op_names = []
    for i in range(n_ops):
        if service[i] == 0:
            op_names.append(f"GET /api/v1/gateway/ep{i}")
        else:
            op_names.append(f"{['GET', 'POST'][i & 1]} /api/v1/svc{service[i]}/op{i}")
    base = rng.uniform(5.0, 50.0, size=n_ops)
    return Topology(n_ops, parent, depth, child_off, child_ids, service, base, op_names, svc_names,
                    pods_per_service)


def _walk(topo: Topology, n_traces: int, rng, branch: float, p_max: float, p_repeat: float):
    """Level-synchronous random walk.  Returns (trace, op, parent_span, level) per span;
    ``parent_span`` indexes the concatenated output (-1 for roots)."""
    fan = np.diff(topo.child_off)
    p_visit = np.minimum(p_max, branch / np.maximum(fan, 1)).astype(np.float64)
    f_tr = np.arange(n_traces, dtype=np.int64)
    f_op = np.zeros(n_traces, dtype=np.int32)
    f_id = np.arange(n_traces, dtype=np.int64)
    tr, op, par, lvl = [f_tr], [f_op], [np.full(n_traces, -1, dtype=np.int64)], [np.zeros(n_traces, np.int8)]
    count, level = n_traces, 0
    while f_op.size:
        level += 1
        nch = fan[f_op]
        rep = np.repeat(np.arange(f_op.size), nch)
        if rep.size == 0:
            break
        local = np.arange(rep.size) - np.repeat(np.cumsum(nch) - nch, nch)
        c_op = topo.child_ids[topo.child_off[f_op][rep] + local]
        keep = rng.random(rep.size) < p_visit[f_op[rep]]
        rep, c_op = rep[keep], c_op[keep]
        dup = rng.random(rep.size) < p_repeat
        rep = np.concatenate([rep, rep[dup]])
        c_op = np.concatenate([c_op, c_op[dup]])
        o = np.argsort(rep, kind="stable")
        rep, c_op = rep[o], c_op[o]
        new_ids = count + np.arange(rep.size, dtype=np.int64)
        tr.append(f_tr[rep]); op.append(c_op); par.append(f_id[rep])
        lvl.append(np.full(rep.size, level, dtype=np.int8))
        f_tr, f_op, f_id = f_tr[rep], c_op, new_ids
        count += rep.size
    return (np.concatenate(tr), np.concatenate(op), np.concatenate(par), np.concatenate(lvl))


def gen_spans(topo: Topology, n_traces: int, seed: int = 0, *, t0_ns: int = 1_700_000_000 * 10**9,
              minutes: float = 5.0, branch: float = 1.6, p_max: float = 0.7, p_repeat: float = 0.1,
              fault_op: Optional[int] = None, fault_frac: float = 0.0, fault_ms: float = 2500.0,
              dup_span_frac: float = 0.0, broken_frac: float = 0.0, names: bool = True,
              span_times: bool = False) -> SpanTable:
    """Generate ``n_traces`` traces.  Trace codes are assigned in sorted traceID order.

    ``span_times``: startTime / endTime per SPAN (a child starts after its parent, ends after
    its own duration) instead of the trace-level TraceStart / TraceEnd the reference's CSVs
    carry (online_rca.py:229-230), so traces near a window edge straddle it: the detector's
    window (preprocess_data.py:13) then keeps only some rows of a trace, while the graph of the
    trace takes all of them (online_rca.py:180,185)."""
    rng = np.random.default_rng([seed, 0x5A])
    tr, op, par, lvl = _walk(topo, n_traces, rng, branch, p_max, p_repeat)
    S = tr.size
    # durations (µs): self time + sum of children, computed bottom-up
    self_ms = rng.normal(topo.base_ms[op], 0.1 * topo.base_ms[op]).clip(0.5, None)
    if fault_op is not None and fault_frac > 0:
        faulty_trace = rng.random(n_traces) < fault_frac
        hit = (op == fault_op) & faulty_trace[tr]
        self_ms[hit] += fault_ms
    dur = self_ms.copy()
    for level in range(int(lvl.max()), 0, -1):
        m = lvl == level
        np.add.at(dur, par[m], dur[m])
    dur_us = np.rint(dur * 1000.0).astype(np.int64)
    # broken traces: drop one non-root span (children become orphans, T11)
    keep = np.ones(S, dtype=bool)
    if broken_frac > 0:
        bt = rng.random(n_traces) < broken_frac
        cand = np.flatnonzero(bt[tr] & (lvl > 0))
        if cand.size:
            # drop the first non-root span of each broken trace
            _, first = np.unique(tr[cand], return_index=True)
            keep[cand[first]] = False
    # trace timing: start uniform in the window, end = start + root duration
    tstart_tr = t0_ns + np.sort(rng.random(n_traces)) * (minutes * 0.97 * NS_PER_MIN)
    tstart_tr = tstart_tr.astype(np.int64)
    root_dur = np.zeros(n_traces, dtype=np.int64)
    root_dur[tr[lvl == 0]] = dur_us[lvl == 0]
    tend_tr = tstart_tr + root_dur * 1000
    if span_times:
        # per span: the parent's start + a 0..2 ms offset per level, end = start + duration
        off = np.zeros(S, dtype=np.int64)
        jit = rng.integers(0, 2_000_000, size=S)
        for level in range(1, int(lvl.max()) + 1):
            m = lvl == level
            off[m] = off[par[m]] + jit[m]
        sp_start = tstart_tr[tr] + off
        sp_end = sp_start + dur_us * 1000
    # traceIDs: random 128-bit hex; code = rank in sorted order
    hi = rng.integers(0, 2**63, size=n_traces, dtype=np.int64)
    trace_rank = np.argsort(np.argsort(hi, kind="stable"), kind="stable").astype(np.int32)
    # row order: by trace start time, then level (a trace's spans are contiguous)
    row = np.lexsort((lvl, tr))
    row = row[keep[row]]
    new_pos = np.full(S, -1, dtype=np.int64)
    new_pos[row] = np.arange(row.size)
    span_code = new_pos[row]
    parent_code = np.where(par[row] >= 0, new_pos[np.maximum(par[row], 0)], -1)
    if dup_span_frac > 0 and row.size > 1:
        # cross-trace duplicated spanIDs (T11): a span reuses another span's ID
        nd = int(dup_span_frac * row.size)
        a = rng.integers(0, row.size, size=nd)
        b = rng.integers(0, row.size, size=nd)
        span_code = span_code.copy()
        span_code[a] = span_code[b]
    pods = topo.pods_per_service
    pod_k = rng.integers(0, pods, size=S)[row] if pods > 1 else np.zeros(row.size, dtype=np.int64)
    op_r = op[row]
    # podop / svcop codes via the name dictionaries (sorted string order)
    st = SpanTable(trace=trace_rank[tr[row]], podop=None, svcop=None, span=span_code.astype(np.int64),
                   parent=parent_code.astype(np.int64), duration=dur_us[row],
                   tstart=sp_start[row] if span_times else tstart_tr[tr[row]],
                   tend=sp_end[row] if span_times else tend_tr[tr[row]])
    svc_of = topo.service[op_r]
    svcop_str = np.array([f"{topo.svc_names[s]}_{topo.op_names[o]}" for s, o in
                          zip(topo.service, range(topo.n_ops))], dtype=object)
    sv_names, sv_code = np.unique(svcop_str, return_inverse=True)
    st.svcop = sv_code.astype(np.int32)[op_r]
    st.svcop_names = list(sv_names)
    pod_names = np.array([f"{topo.svc_names[s]}-{(s * 2654435761) % 99991:05d}-{k}"
                          for s in range(len(topo.svc_names)) for k in range(pods)], dtype=object)
    podop_key = op_r.astype(np.int64) * pods + pod_k
    all_podop = np.array([f"{pod_names[topo.service[o] * pods + k]}_{topo.op_names[o]}"
                          for o in range(topo.n_ops) for k in range(pods)], dtype=object)
    pn, pcode = np.unique(all_podop, return_inverse=True)
    st.podop = pcode.astype(np.int32)[podop_key]
    st.podop_names = list(pn)
    if names:
        order_hi = np.sort(hi)
        lo = np.random.default_rng([seed, 0x11]).integers(0, 2**63, size=n_traces, dtype=np.int64)
        st.trace_names = [f"{int(h):016x}{int(l):016x}" for h, l in zip(order_hi, lo)]
    st.meta = dict(pod_k=pod_k.astype(np.int32), op=op_r, svc=svc_of, seed=seed, n_gen_traces=n_traces)
    return st


def to_dataframe(st: SpanTable, topo: Topology, seed: int = 0):
    """Materialise the reference string schema (online_rca.py:221-248 after rename)."""
    import pandas as pd

    rng = np.random.default_rng([seed, 0x33])
    op = st.meta["op"]
    svc = st.meta["svc"]
    pods = topo.pods_per_service
    opn = np.array(topo.op_names, dtype=object)[op]
    ui = svc == 0
    if ui.any():  # REST id segment that the naming rule strips
        ids = rng.integers(1000, 99999, size=int(ui.sum()))
        opn = opn.copy()
        opn[ui] = [f"{a}/{b}" for a, b in zip(opn[ui], ids)]
    # spanID strings: distinct 16-hex per span code
    sp_hex = {}
    span_ids = np.array([f"{(int(c) * 0x9E3779B97F4A7C15 + 0x1234567) & 0xFFFFFFFFFFFFFFFF:016x}"
                         for c in st.span], dtype=object)
    par_ids = np.array([f"{(int(c) * 0x9E3779B97F4A7C15 + 0x1234567) & 0xFFFFFFFFFFFFFFFF:016x}"
                        if c >= 0 else None for c in st.parent], dtype=object)
    del sp_hex
    pod_names = [f"{topo.svc_names[s]}-{(s * 2654435761) % 99991:05d}-{k}"
                 for s in range(len(topo.svc_names)) for k in range(pods)]
    podn = np.array([pod_names[s * pods + k] for s, k in zip(svc, st.meta["pod_k"])], dtype=object)
    df = pd.DataFrame({
        "traceID": np.array(st.trace_names, dtype=object)[st.trace],
        "spanID": span_ids,
        "ParentSpanId": par_ids,
        "serviceName": np.array(topo.svc_names, dtype=object)[svc],
        "operationName": opn,
        "podName": podn,
        "duration": st.duration.astype(np.int64),
        "startTime": pd.to_datetime(st.tstart, unit="ns"),
        "endTime": pd.to_datetime(st.tend, unit="ns"),
    })
    return df


def fault_op_of(topo: Topology) -> int:
    """The faulty operation: the root's first child (visited by most traces)."""
    return int(topo.child_ids[topo.child_off[0]]) if topo.child_off[1] > 0 else 0


def window_pair(n_ops: int, n_traces: int, seed: int, *, pods: int = 1, dup: float = 0.0,
                broken: float = 0.0, branch: float = 4.0, p_max: float = 0.7, zipf_s: float = 0.0,
                fault_frac: float = 0.4, fault_ms: float = 4000.0, names: bool = True, span_times: bool = False,
                minutes: float = 5.0):
    """(topology, normal SpanTable for the SLO, abnormal SpanTable with a fault) -- SURVEY §8.2."""
    topo = make_topology(n_ops, seed, pods_per_service=pods, zipf_s=zipf_s)
    normal = gen_spans(topo, n_traces, seed + 1, branch=branch, p_max=p_max, names=names, span_times=span_times,
                       minutes=minutes)
    abnormal = gen_spans(topo, n_traces, seed + 2, branch=branch, p_max=p_max,
                         fault_op=fault_op_of(topo), fault_frac=fault_frac, fault_ms=fault_ms,
                         dup_span_frac=dup,
                         broken_frac=broken, names=names, span_times=span_times, minutes=minutes)
    return topo, normal, abnormal


def window_dataframes(n_ops: int, n_traces: int, seed: int, **kw):
    topo, normal, abnormal = window_pair(n_ops, n_traces, seed, **kw)
    return to_dataframe(normal, topo, seed + 1), to_dataframe(abnormal, topo, seed + 2)


def stream_dataframes(n_ops: int, n_traces: int, seed: int, *, minutes: float = 60.0, fault_frac: float = 0.003,
                      gap_after_min: Optional[float] = None, gap_min: float = 0.0, **kw):
    """A long span stream for the driver's window sweep (online_rca.py:161-216): normal frame for
    the SLO and an abnormal frame of ``minutes`` of traffic with a rare fault, so that some 5-minute
    windows trigger and some do not.  ``gap_after_min``: traces starting that many minutes after
    the first one are shifted ``gap_min`` minutes later (a silent gap: an empty window, T2)."""
    ndf, adf = window_dataframes(n_ops, n_traces, seed, minutes=minutes, fault_frac=fault_frac, **kw)
    if gap_after_min is not None:
        cut = adf["startTime"].min() + pd_timedelta(minutes=gap_after_min)
        late = adf["startTime"] >= cut
        shift = pd_timedelta(minutes=gap_min)
        adf.loc[late, "startTime"] = adf.loc[late, "startTime"] + shift
        adf.loc[late, "endTime"] = adf.loc[late, "endTime"] + shift
    return ndf, adf


def pd_timedelta(**kw):
    import pandas as pd

    return pd.Timedelta(**kw)


def frame_digest(df) -> str:
    """sha256 over the reference-schema columns, so a fixture can check that the
    generator re-created exactly the frame the reference was run on."""
    import hashlib

    h = hashlib.sha256()
    for c in ("traceID", "spanID", "ParentSpanId", "serviceName", "operationName", "podName"):
        h.update("\x1f".join("" if v is None else str(v) for v in df[c].tolist()).encode())
    for c in ("duration", "startTime", "endTime"):
        h.update(np.ascontiguousarray(df[c].to_numpy().astype(np.int64)).tobytes())
    return h.hexdigest()


SLO_SIZES = (1, 7, 8, 9, 127, 128, 129, 1000, 8191, 8192, 8193, 16384, 16385, 24577, 50001, 131075)


def slo_frame(seed: int = 7, sizes=SLO_SIZES):
    """Spans of ops sized around numpy's 8192-element reduction buffer and its pairwise
    block (128), rows interleaved at random: the SLO variance depends on the row order inside
    each op and on the buffer chunking of np.std (preprocess_data.py:66-73)."""
    import pandas as pd

    rng = np.random.default_rng(seed)
    op = np.repeat(np.arange(len(sizes)), sizes)
    rng.shuffle(op)
    n = op.size
    # heavy-tailed integer durations (microseconds), large enough that rounding matters
    dur = (rng.lognormal(8.0, 1.5, n) + rng.integers(0, 1000, n)).astype(np.int64)
    t0 = np.int64(1_700_000_000_000_000_000)
    start = t0 + np.arange(n, dtype=np.int64) * 1000
    return pd.DataFrame({
        "traceID": [f"s{i // 4:07d}" for i in range(n)],
        "spanID": [f"x{i:08d}" for i in range(n)],
        "ParentSpanId": [None] * n,
        "serviceName": [f"svc{o % 3}" for o in op],
        "operationName": [f"op{o:02d}" for o in op],
        "podName": [f"svc{o % 3}-pod" for o in op],
        "duration": dur,
        "startTime": pd.to_datetime(start),
        "endTime": pd.to_datetime(start + dur * 1000),
    })


_BIG_CHUNK = 1 << 21   # traces per generation chunk of big_graph


def _big_chunk(job):
    """Traces of one big_graph chunk: (len_t, len_o partial, distinct ops per trace, sorted ops)."""
    rng, T, N, cdf, spans_mean = job
    if not isinstance(rng, np.random.Generator):
        rng = np.random.default_rng(rng)
    k = np.maximum(rng.poisson(spans_mean - 1.0, T), 1).astype(np.int64) + 1        # spans per trace
    S = int(k.sum())
    trace = np.repeat(np.arange(T, dtype=np.int64), k)
    op = np.searchsorted(cdf, rng.random(S), side="right").clip(0, N - 1).astype(np.int64)
    op[np.r_[0, np.cumsum(k)[:-1]]] = 0                                              # root span
    len_o = np.bincount(op, minlength=N)
    key = np.unique(trace * N + op)
    del trace, op
    return k.astype(np.int32), len_o, np.bincount(key // N, minlength=T), (key % N).astype(np.int32)


def big_graph(n_ops: int, n_traces: int, seed: int = 11, spans_mean: float = 19.0, zipf_s: float = 1.1,
              fp_dup: float = 0.25, shard: tuple | None = None):
    """A C4/C5-scale op<->trace graph generated directly as incidence lists (no span table):
    per trace ~Poisson(spans_mean) spans whose ops follow a power law (zipf_s) over n_ops, the
    root op in every trace, duplicates within a trace allowed (len_t counts spans, the incidence
    keeps distinct ops); a random call tree over the ops.  Returns a graph.HostGraph with
    ``nodes``/``traces`` as ranges (names are not needed for timing).

    ``shard=(rank, world)``: this rank's n_traces traces of a trace-sharded graph:
    traces from a per-rank stream, the call tree from ``seed`` (the same on every rank); len_o is
    this rank's partial span count and the call edges / children counts sit on rank 0, which is
    what mr_pagerank_sharded expects."""
    from .graph import HostGraph

    rank, world = shard if shard is not None else (0, 1)
    rng = np.random.default_rng(seed if shard is None else (seed, rank, world))
    T, N = int(n_traces), int(n_ops)
    w = 1.0 / np.arange(1, N + 1, dtype=np.float64) ** zipf_s
    cdf = np.cumsum(w / w.sum())
    if T <= _BIG_CHUNK:
        parts = [_big_chunk((rng, T, N, cdf, spans_mean))]
    else:   # C5-sized graphs (10^8 traces, 2x10^9 spans): chunks with their own streams, in parallel
        from concurrent.futures import ProcessPoolExecutor

        jobs = [((seed, rank, world, c), min(_BIG_CHUNK, T - c0), N, cdf, spans_mean)
                for c, c0 in enumerate(range(0, T, _BIG_CHUNK))]
        with ProcessPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
            parts = list(ex.map(_big_chunk, jobs))
    len_t = np.concatenate([p[0] for p in parts])
    len_o = np.sum([p[1] for p in parts], axis=0).astype(np.int32)
    sr_off = np.zeros(T + 1, np.int64)
    np.cumsum(np.concatenate([p[2] for p in parts]), out=sr_off[1:])
    sr_ops = np.concatenate([p[3] for p in parts])
    del parts
    # call tree: every op but the root has one parent of smaller index
    trng = rng if shard is None else np.random.default_rng(seed)
    child = np.arange(1, N, dtype=np.int64)
    parent = (trng.random(N - 1) * child).astype(np.int64)
    if rank != 0:
        child, parent = child[:0], parent[:0]
    order = np.lexsort((parent, child))
    ss_off = np.zeros(N + 1, np.int64)
    np.cumsum(np.bincount(child[order], minlength=N), out=ss_off[1:])
    ss_par = parent[order].astype(np.int32)
    nchild = np.bincount(parent, minlength=N).astype(np.int32)
    return HostGraph(range(N), range(T), sr_off, sr_ops, None, None, len_t, len_o, ss_off, ss_par, nchild,
                     None, None)


_SPAN_SLOTS = 32   # C4 span tables: at most this many spans per trace (global row = trace * 32 + j)


def big_spans(n_ops: int, n_traces: int, seed: int = 11, spans_mean: float = 19.0,
              dup_frac: float = 0.01, broken_frac: float = 0.05, shard: tuple | None = None) -> SpanTable:
    """A C4-scale SPAN table (codes only), generated vectorised for K1-inclusive benchmarks.
    Ops form a random call tree (op o > 0 has one parent op < o, the same tree on every rank);
    per trace ~Poisson(spans_mean) spans (capped at 32): the first is the root op, each later
    span picks a uniformly chosen earlier span of the trace as its parent and one of the parent
    op's child ops (a leaf op's child: the next op code -- edges off the tree, at most n_ops).
    ``broken_frac`` of the traces lose one non-root span (orphans, T11) and ``dup_frac`` of the
    rows reuse the spanID of a random trace's root span -- often a trace of another rank, so the
    ParentSpanId join crosses shards (T11).  Pod-op = service-op = op.

    ``shard=(rank, world)``: this rank's share of the n_traces traces (a contiguous trace-code
    range) with global codes; rows are trace-major and ``row`` = trace * 32 + span slot (a
    monotone global row index: first appearance, T10)."""
    rank, world = shard if shard is not None else (0, 1)
    base, rem = divmod(n_traces, world)
    t_lo = rank * base + min(rank, rem)
    T = base + (1 if rank < rem else 0)
    N = int(n_ops)
    trng = np.random.default_rng(seed)                                 # the op tree: every rank alike
    child = np.arange(1, N, dtype=np.int64)
    par_op = (trng.random(N - 1) * child).astype(np.int64)
    order = np.argsort(par_op, kind="stable")
    ch_list = child[order]
    ch_off = np.zeros(N + 1, np.int64)
    np.cumsum(np.bincount(par_op, minlength=N), out=ch_off[1:])
    rng = np.random.default_rng((seed, rank, world))
    k = np.clip(rng.poisson(spans_mean - 1.0, T) + 1, 1, _SPAN_SLOTS).astype(np.int64)
    M = np.zeros((T, _SPAN_SLOTS), np.int32)                           # op of slot j of each trace
    P = np.full((T, _SPAN_SLOTS), -1, np.int8)                         # parent slot
    for j in range(1, _SPAN_SLOTS):
        live = np.flatnonzero(k > j)
        if live.size == 0:
            break
        pj = (rng.random(live.size) * j).astype(np.int64)
        po = M[live, pj].astype(np.int64)
        nch = ch_off[po + 1] - ch_off[po]
        pick = ch_off[po] + (rng.random(live.size) * np.maximum(nch, 1)).astype(np.int64)
        M[live, j] = np.where(nch > 0, ch_list[np.minimum(pick, ch_list.size - 1)], (po + 1) % N).astype(np.int32)
        P[live, j] = pj.astype(np.int8)
    S0 = int(k.sum())
    valid = np.arange(_SPAN_SLOTS)[None, :] < k[:, None]
    tr = np.repeat(np.arange(T, dtype=np.int64), k)
    j = np.nonzero(valid)[1].astype(np.int64)
    gtr = tr + t_lo
    op = M[valid]
    pslot = P[valid].astype(np.int64)
    del M, P, valid
    code = gtr * _SPAN_SLOTS + j                                       # spanID code = global row slot
    parent = np.where(pslot >= 0, gtr * _SPAN_SLOTS + pslot, -1)
    start = np.zeros(T + 1, np.int64)
    np.cumsum(k, out=start[1:])
    keep = np.ones(S0, bool)
    bt = np.flatnonzero((rng.random(T) < broken_frac) & (k > 1))
    keep[start[bt] + 1 + (rng.random(bt.size) * (k[bt] - 1)).astype(np.int64)] = False
    if dup_frac > 0:
        d = np.flatnonzero(rng.random(S0) < dup_frac)
        code[d] = rng.integers(0, n_traces, d.size) * _SPAN_SLOTS      # a root spanID, any rank
    dur = rng.integers(1_000, 2_000_000, S0)
    t_start = (1_700_000_000 * 10**9 + gtr * 1000).astype(np.int64)
    sl = keep
    return SpanTable(trace=gtr[sl].astype(np.int32), podop=op[sl], svcop=op[sl], span=code[sl],
                     parent=parent[sl], duration=dur[sl], tstart=t_start[sl], tend=t_start[sl] + dur[sl] * 1000,
                     trace_names=range(n_traces), podop_names=range(N), svcop_names=range(N),
                     row=(gtr[sl] * _SPAN_SLOTS + j[sl]).astype(np.int32))
