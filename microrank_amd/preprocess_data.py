"""Drop-in for the reference module ``preprocess_data`` (preprocess_data.py).

* ``get_pagerank_graph`` builds the op<->trace graph on the GPU (K1,
  csrc/mr_graph_build.hip) from the int-coded span table and returns four lazy mappings
  with the reference's key order and list contents.  Passing them straight to
  ``pagerank.trace_pagerank`` (what ``online_anomaly_detect_RCA`` does) keeps the graph in
  HBM: no dict is ever materialised.
* ``get_operation_slo`` runs the SLO reduction on the GPU (K4, csrc/mr_slo.hip).
* ``get_span``, ``get_service_operation_list`` and ``get_operation_duration_data`` are
  DataFrame utilities with the reference's behaviour (including the added ``operation``
  column side effect).

A DataFrame is factorised into a :class:`SpanTable` once and uploaded once; the result is
cached per DataFrame object (see :func:`span_table`).
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import weakref
from collections.abc import Mapping

import numpy as np
import pandas as pd

from . import _lib
from ._lib import SpanCols, ptr
from .spans import UI_SERVICE, IngestedTable, SpanTable, _as_ns, arrow_columns, op_display

ROOT_INDEX = "root"   # preprocess_data.py:7


# ------------------------------------------------------------------------ span table cache
def span_strings(df: pd.DataFrame, arrays):
    """The mr_span_strings view of a DataFrame's Arrow string columns (no copies of the string
    bytes) plus the host arrays it points into: (struct, keep-alive, duration, tstart, tend)."""
    S = len(df)
    ss = _lib.SpanStrings()
    ss.n_spans = S
    keep = {"arrays": arrays}
    for field, col in (("trace_id", "traceID"), ("span_id", "spanID"), ("parent_id", "ParentSpanId"),
                       ("service", "serviceName"), ("operation", "operationName"), ("pod", "podName")):
        a = arrays[col]
        validity, offsets, data = a.buffers()[:3]
        sc = getattr(ss, field)
        if offsets is None:   # an all-null column (no ParentSpanId): zero offsets, no bytes
            z = np.zeros(S + 1, np.int64)
            keep[col] = z
            sc.offsets = ptr(z, C.c_int64)
            sc.bytes = None
        else:
            sc.offsets = C.cast(C.c_void_p(offsets.address + 8 * a.offset), C.POINTER(C.c_int64))
            sc.bytes = data.address if data is not None and data.size else None
        if a.null_count:
            vb = np.unpackbits(np.frombuffer(validity, np.uint8), bitorder="little")[a.offset:a.offset + S]
            v = np.packbits(vb, bitorder="little")
            keep[col + ".valid"] = v
            sc.valid = v.ctypes.data
        else:
            sc.valid = None
    dur = np.ascontiguousarray(df["duration"].to_numpy(dtype=np.int64))
    ss.duration = ptr(dur, C.c_int64)
    ts = te = None
    if "startTime" in df and "endTime" in df:
        ts, te = np.ascontiguousarray(_as_ns(df["startTime"])), np.ascontiguousarray(_as_ns(df["endTime"]))
        ss.tstart, ss.tend = ptr(ts, C.c_int64), ptr(te, C.c_int64)
    return ss, keep, dur, ts, te


class DeviceSpans:
    """An mr_spans handle: the span columns resident in HBM."""

    @classmethod
    def ingest(cls, ctx, df: pd.DataFrame, arrays):
        """The table built on the device from the DataFrame's strings (mr_spans_ingest, SURVEY 8(f)
        f2): factorisation, name rules and dictionaries in HBM.  Returns (IngestedTable, DeviceSpans)."""
        ss, _keep, dur, ts, te = span_strings(df, arrays)
        h = _lib.P()
        ctx.check(_lib.load().mr_spans_ingest(ctx.h, C.byref(ss), C.byref(h)), "mr_spans_ingest")
        dev = cls.__new__(cls)
        dev.ctx, dev.h = ctx, h
        table = IngestedTable(dev, arrays, dur, ts, te)
        dev.table = table
        return table, dev

    def __init__(self, ctx, table: SpanTable):
        lib = _lib.load()
        table.check()
        cols = SpanCols()
        cols.n_spans = table.n_spans
        cols.n_traces, cols.n_podops, cols.n_svcops = table.n_traces, table.n_podops, table.n_svcops
        keep = {}
        for name, ct in (("trace", C.c_int32), ("podop", C.c_int32), ("svcop", C.c_int32), ("span", C.c_int64),
                         ("parent", C.c_int64), ("duration", C.c_int64), ("tstart", C.c_int64), ("tend", C.c_int64),
                         ("row", C.c_int32)):
            a = getattr(table, name, None)
            if a is None:
                continue
            a = np.ascontiguousarray(a, dtype=np.int32 if ct is C.c_int32 else np.int64)
            keep[name] = a
            setattr(cols, name, ptr(a, ct))
        h = _lib.P()
        ctx.check(lib.mr_spans_upload(ctx.h, C.byref(cols), C.byref(h)), "mr_spans_upload")
        self.ctx, self.h, self.table = ctx, h, table

    def close(self):
        # a destroyed context has freed its handles already (mr_ctx_destroy)
        if getattr(self, "h", None) and getattr(getattr(self, "ctx", None), "h", None):
            _lib.load().mr_spans_free(self.h)
        self.h = None

    def __del__(self):  # pragma: no cover
        if sys.is_finalizing():   # the owning context may already be destroyed
            return
        try:
            self.close()
        except Exception:
            pass


_CACHE: dict = {}
# MR_HOST_FACTORIZE=1: factorise the DataFrame's strings on the host (SpanTable.from_dataframe)
# instead of on the device (A/B and parity tests)
_HOST_FACTORIZE = os.environ.get("MR_HOST_FACTORIZE", "") not in ("", "0")
# every column SpanTable.from_dataframe reads: an in-place edit of any of them (the reference's own
# get_operation_duration_data rewrites operationName, preprocess_data.py:100) must rebuild the table
_TABLE_COLUMNS = ("traceID", "spanID", "ParentSpanId", "serviceName", "operationName", "podName", "duration",
                  "startTime", "endTime")


_memcmp = C.CDLL(None).memcmp
_memcmp.restype = C.c_int
_memcmp.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]


class _ColumnSnapshot:
    """What a column held when the device table was built, held so that "unchanged" is decided
    exactly, never by sampling (an in-place cell edit outside a sample must
    rebuild the table, as the reference -- which has no cache -- would see the edit):
      * Arrow-backed columns: the ChunkedArray itself (immutable: an in-place edit replaces it, and
        holding the old one keeps its buffers from being reused at the same addresses);
      * NumPy columns: a copy of the values -- for object columns a copy of the pointer array, which
        also holds a reference to every string, so equal pointers mean the same (immutable) string
        objects: a word-by-word compare of 8 B per row decides it."""

    def __init__(self, s: pd.Series):
        arr = s.array
        self.pa = getattr(arr, "_pa_array", None)
        self.np = self.mask = self.boxed = None
        if self.pa is None:
            data, mask = _masked_parts(arr)
            if data is not None:   # nullable (masked) columns, e.g. Int64 with pd.NA: values + mask
                self.np, self.mask = data.copy(), mask.copy()
                return
            a = getattr(arr, "_ndarray", None)
            if a is None:   # another extension array: np.asarray boxes new objects per call
                self.boxed = s.copy()
            else:
                self.np = np.array(a, copy=True)

    def matches(self, s: pd.Series) -> bool:
        arr = s.array
        pa_arr = getattr(arr, "_pa_array", None)
        if self.pa is not None or pa_arr is not None:
            return pa_arr is self.pa
        if self.boxed is not None:   # compared by value (NA equal to NA), not by object identity
            return s.dtype == self.boxed.dtype and bool(s.reset_index(drop=True).equals(self.boxed.reset_index(drop=True)))
        data, mask = _masked_parts(arr)
        if self.mask is not None or data is not None:
            return self.mask is not None and data is not None and _same_values(data, self.np) and \
                _same_values(mask, self.mask)
        a = getattr(arr, "_ndarray", None)
        return a is not None and _same_values(a, self.np)


def _masked_parts(arr):
    """(values, mask) of a pandas masked extension array (BaseMaskedArray: Int64, Float64,
    boolean ...), else (None, None)."""
    data, mask = getattr(arr, "_data", None), getattr(arr, "_mask", None)
    if isinstance(data, np.ndarray) and isinstance(mask, np.ndarray):
        return data, mask
    return None, None


def _same_values(a: np.ndarray, b: np.ndarray) -> bool:
    """a equals the snapshot b: values, or an object column's pointers (the snapshot holds a
    reference to every object, so equal pointers are the same immutable objects)."""
    if a.dtype != b.dtype or a.shape != b.shape:
        return False
    if a.flags.c_contiguous and b.flags.c_contiguous:
        # memcmp (ctypes releases the GIL)
        return a.nbytes == 0 or _memcmp(C.c_void_p(a.ctypes.data), C.c_void_p(b.ctypes.data), C.c_size_t(a.nbytes)) == 0
    return bool(np.array_equal(a, b)) if a.dtype != object else all(u is v for u, v in zip(a.tolist(), b.tolist()))


class _FrameSnapshot:
    """Exact cache key of the columns a span table is built from: row count, column set, this
    module's mutation version and a _ColumnSnapshot per column.  A lookup compares 8 B per row and
    column (the columns in parallel: the compares release the GIL) -- O(rows) like the reference's
    own per-window DataFrame filtering (preprocess_data.py:13), and exact."""

    def __init__(self, df: pd.DataFrame):
        self.cols = tuple(c for c in _TABLE_COLUMNS if c in df.columns)
        self.n = len(df)
        self.version = df.attrs.get("_mr_version", 0)
        self.parts = [_ColumnSnapshot(df[c]) for c in self.cols]

    def matches(self, df: pd.DataFrame, reads=None) -> bool:
        """reads: the columns the caller's result depends on (None: all) -- only those are compared
        word by word, so a call whose own columns are unchanged reuses the table even when another
        column was edited (its result cannot see that column; the next call that reads it rebuilds)."""
        cols = tuple(c for c in _TABLE_COLUMNS if c in df.columns)
        if cols != self.cols or len(df) != self.n or df.attrs.get("_mr_version", 0) != self.version:
            return False
        if self.n == 0:
            return True
        pick = [i for i, c in enumerate(cols) if reads is None or c in reads]
        parts, series = [self.parts[i] for i in pick], [df[cols[i]] for i in pick]
        if self.n < 65536:
            return all(p.matches(x) for p, x in zip(parts, series))
        return all(list(_pool().map(lambda px: px[0].matches(px[1]), zip(parts, series))))


_POOL = None


def _pool():
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor

        _POOL = ThreadPoolExecutor(max_workers=len(_TABLE_COLUMNS), thread_name_prefix="mr-fp")
    return _POOL


def _fingerprint(df: pd.DataFrame) -> _FrameSnapshot:
    """The exact snapshot of df's span-table columns (``_fingerprint(df).matches(df)`` until any of
    them changes, in place or by replacement)."""
    return _FrameSnapshot(df)


def invalidate(df: pd.DataFrame) -> None:
    """Drop the cached device span table of ``df``; the next drop-in call rebuilds it.  Not needed
    for correctness (every lookup compares the columns exactly); frees the device table early."""
    df.attrs["_mr_version"] = df.attrs.get("_mr_version", 0) + 1
    for k in [k for k in _CACHE if k[0] == id(df)]:
        _CACHE.pop(k, None)


# the columns each drop-in call's result depends on (the cache compares only those, span_table)
DETECT_READS = ("traceID", "serviceName", "operationName", "duration", "startTime", "endTime")
GRAPH_READS = ("traceID", "spanID", "ParentSpanId", "serviceName", "operationName", "podName")


def span_table(df: pd.DataFrame, ctx=None, reads=None):
    """(SpanTable, DeviceSpans) for a DataFrame, built once per (DataFrame, Context) and rebuilt
    when a column it reads changed -- of the columns in `reads` (the ones the caller's result
    depends on; None: every column the table is built from).  The device table belongs to the
    context that uploaded it (mr_spans handles are per mr_ctx), so two contexts sharing a DataFrame
    get a handle each."""
    ctx = ctx or _lib.default_context()
    key = (id(df), id(ctx))
    hit = _CACHE.get(key)
    if hit is not None and hit[0]() is df and hit[1]() is ctx and hit[2].matches(df, reads):
        return hit[3], hit[4]
    fp = _fingerprint(df)   # (taken before the build: the table is built from these values)
    arrays = None if _HOST_FACTORIZE else arrow_columns(df)
    if arrays is not None:   # strings -> codes on the device
        table, dev = DeviceSpans.ingest(ctx, df, arrays)
    else:                    # non-string / null-bearing columns: the host factorisation
        table = SpanTable.from_dataframe(df)
        dev = DeviceSpans(ctx, table)
    try:
        ref = weakref.ref(df, lambda _r, k=key: _CACHE.pop(k, None))
        cref = weakref.ref(ctx, lambda _r, k=key: _CACHE.pop(k, None))
    except TypeError:  # pragma: no cover - DataFrames and Contexts are weak-referenceable
        ref, cref = (lambda: df), (lambda: ctx)
    _CACHE[key] = (ref, cref, fp, table, dev)
    return table, dev


class StreamedTable(IngestedTable):
    """IngestedTable of a table built by mr_spans_append: names are read from the chunk that holds
    each code's first row (mr_spans_dict_sources gives its stream row number)."""

    def __init__(self, dev, chunks):
        super().__init__(dev, None, None, None, None)
        self._chunks = chunks   # [(first stream row, rows, Arrow columns)], ascending

    def _rows(self, which):
        n = (self.n_traces, self.n_podops, self.n_svcops)[which]
        src = np.zeros(max(n, 1), np.int64)
        self._dev.ctx.check(_lib.load().mr_spans_dict_sources(self._dev.h, which, ptr(src, C.c_int64)),
                            "mr_spans_dict_sources")
        return src[:n]

    def _take(self, col, rows):
        import pyarrow as pa

        rows = np.asarray(rows, np.int64)
        bases = np.array([c[0] for c in self._chunks], np.int64)
        which = np.searchsorted(bases, rows, side="right") - 1
        out = [None] * rows.size
        for ci in np.unique(which):
            sel = np.flatnonzero(which == ci)
            base, _n, arrays = self._chunks[ci]
            vals = arrays[col].take(pa.array(rows[sel] - base)).to_pylist()
            for k, v in zip(sel, vals):
                out[k] = v
        return out


class SpanStream:
    """an append-only device span table (mr_spans_append).  Each append keeps the
    resident rows whose trace starts at or after ``keep_from`` and adds the chunk's rows; only the
    chunk's strings cross PCIe and only its Arrow columns are built on the host, so the host cost of
    an append scales with the chunk, not with the resident table.  The resulting table equals
    :func:`span_table` of the concatenated, filtered DataFrame row for row."""

    def __init__(self, ctx=None):
        self.ctx = ctx or _lib.default_context()
        self.dev = None
        self.table = None
        self.chunks = []        # (first stream row, rows, Arrow columns, largest trace start)
        self.next = 0

    @staticmethod
    def accepts(chunk: pd.DataFrame):
        """Arrow string columns for a chunk the device append can take (string columns, datetime
        trace times), else None."""
        if len(chunk) == 0 or not all(c in chunk.columns and np.issubdtype(chunk[c].dtype, np.datetime64)
                                      for c in ("startTime", "endTime")):
            return None
        return arrow_columns(chunk)

    def append(self, chunk: pd.DataFrame, keep_from_ns: int, arrays=None):
        arrays = arrays if arrays is not None else self.accepts(chunk)
        if arrays is None:
            raise ValueError("SpanStream.append: the chunk needs string columns and datetime startTime/endTime")
        ss, _keep, _dur, ts, _te = span_strings(chunk, arrays)
        h = _lib.P()
        self.ctx.check(_lib.load().mr_spans_append(self.ctx.h, self.dev.h if self.dev is not None else None,
                                                   int(keep_from_ns), C.byref(ss), C.byref(h)), "mr_spans_append")
        if self.dev is not None:
            self.dev.close()
        dev = DeviceSpans.__new__(DeviceSpans)
        dev.ctx, dev.h = self.ctx, h
        self.chunks.append((self.next, len(chunk), arrays, int(ts.max())))
        self.next += len(chunk)
        # chunks whose every trace started before keep_from hold no resident row any more
        self.chunks = [c for c in self.chunks if c[3] >= keep_from_ns]
        self.dev = dev
        self.table = StreamedTable(dev, [c[:3] for c in self.chunks])
        dev.table = self.table
        return self.table, dev

    def frame(self, keep_from_ns: int, frames):
        """The resident rows as a DataFrame (the per-window fallback's input), from the chunk frames."""
        df = pd.concat(frames, ignore_index=True) if len(frames) > 1 else frames[0]
        keep = _as_ns(df["startTime"]) >= keep_from_ns
        return df[keep].reset_index(drop=True) if not keep.all() else df

    def close(self):
        if self.dev is not None:
            self.dev.close()
        self.dev = self.table = None


# ------------------------------------------------------------------------ reference utilities
def get_span(df, start=None, end=None):
    """preprocess_data.py:10-14 -- inclusive trace-level window (T15)."""
    if start and end:
        df = df[(df["startTime"] >= start) & (df["endTime"] <= end)]
    return df


def _svc_op_names(span_df: pd.DataFrame) -> np.ndarray:
    svc = span_df["serviceName"].to_numpy(dtype=object)
    op = op_display(svc, span_df["operationName"].to_numpy(dtype=object))
    return np.array([f"{a}_{b}" for a, b in zip(svc, op)], dtype=object)


def get_service_operation_list(span_df: pd.DataFrame):
    """preprocess_data.py:26-33: adds the ``operation`` column, returns its distinct values in
    first-appearance order."""
    span_df["operation"] = _svc_op_names(span_df)
    return span_df["operation"].drop_duplicates().tolist()


def get_operation_slo(service_operation_list, span_df: pd.DataFrame, *, ctx=None):
    """preprocess_data.py:50-78 on the GPU (K4): {svc_op: [round(mean/1000,4), round(std/1000,4)]}
    for the ops of the DataFrame that are in ``service_operation_list``, keys in sorted order."""
    span_df["operation"] = _svc_op_names(span_df)
    ctx = ctx or _lib.default_context()
    table, dev = span_table(span_df, ctx)
    n = table.n_svcops
    mean = np.empty(n, np.float64)
    std = np.empty(n, np.float64)
    cnt = np.empty(n, np.int64)
    ctx.check(_lib.load().mr_slo(ctx.h, dev.h, ptr(mean, C.c_double), ptr(std, C.c_double), ptr(cnt, C.c_int64)),
              "mr_slo")
    keep = set(service_operation_list)
    out = {}
    for code, name in enumerate(table.svcop_names):   # codes are in sorted name order
        if cnt[code] > 0 and name in keep:
            out[name] = [np.float64(mean[code]), np.float64(std[code])]
    return out


def get_operation_duration_data(operation_list, span_df: pd.DataFrame):
    """preprocess_data.py:97-122 -- {traceID: {svc_op: count, ..., 'duration': max}} (sorted
    keys, traces with max duration <= 0 dropped).  Mutates ``operationName`` of ``span_df``
    like the reference.  The detector itself runs on the GPU (anormaly_detector.py)."""
    span_df["operationName"] = _svc_op_names(span_df)
    span_df.attrs["_mr_version"] = span_df.attrs.get("_mr_version", 0) + 1   # a table column changed
    counts = span_df.groupby(["traceID", "operationName"]).size().unstack(fill_value=0)
    counts["duration"] = span_df.groupby("traceID")["duration"].max()
    counts = counts.dropna(subset=["duration"])
    counts = counts[counts["duration"] > 0]
    return counts.to_dict(orient="index")


# ------------------------------------------------------------------------ K1 graph + lazy dicts
class PagerankGraph:
    """Device graph of one ``get_pagerank_graph`` call and its four reference-shaped views."""

    def __init__(self, ctx, table: SpanTable, dev: DeviceSpans, trace_mask: np.ndarray):
        lib = _lib.load()
        mask = np.ascontiguousarray(trace_mask, dtype=np.uint8)
        h = _lib.P()
        ctx.check(lib.mr_graph_build(ctx.h, dev.h, ptr(mask, C.c_uint8), C.byref(h)), "mr_graph_build")
        from .graph import DeviceGraph

        n, t, nnz, e = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int64()
        lib.mr_graph_info(h, C.byref(n), C.byref(t), C.byref(nnz), C.byref(e))
        self.N, self.T = n.value, t.value
        self.node_podop = np.empty(self.N, np.int32)
        self.trace_code = np.empty(self.T, np.int32)
        ctx.check(lib.mr_graph_nodes(h, ptr(self.node_podop, C.c_int32), ptr(self.trace_code, C.c_int32)),
                  "mr_graph_nodes")
        self.table, self.mask = table, mask.astype(bool)
        nodes = [table.podop_names[c] for c in self.node_podop]
        # the trace keys (sorted traceIDs, T of them) are built when something reads them: the
        # driver's window body never does (trace_pagerank ranks the device graph)
        self._dg = DeviceGraph(ctx, h, nodes, None, self.N, self.T)
        self.nodes, self._traces = nodes, None
        self._lists = None
        self.operation_operation = GraphDicts(self, "operation_operation")
        self.operation_trace = GraphDicts(self, "operation_trace")
        self.trace_operation = GraphDicts(self, "trace_operation")
        self.pr_trace = GraphDicts(self, "pr_trace")

    def device_graph(self):
        return self._dg

    @property
    def traces(self):
        if self._traces is None:
            tb = self.table
            names = tb.meta.get("trace_names_arr")
            if names is None:
                names = tb.meta["trace_names_arr"] = np.asarray(tb.trace_names, dtype=object)
            self._traces = names[self.trace_code].tolist()
            self._dg.traces = self._traces
        return self._traces

    def as_tuple(self):
        return self.operation_operation, self.operation_trace, self.trace_operation, self.pr_trace

    def _materialise(self):
        """List contents (one entry per span, DataFrame row order) for code that inspects the
        dicts; the key order comes from the device graph."""
        if self._lists is not None:
            return self._lists
        tb = self.table
        rows = np.flatnonzero(self.mask[tb.trace])
        node_of = {int(c): i for i, c in enumerate(self.node_podop)}
        rn = np.array([node_of[int(c)] for c in tb.podop[rows]], dtype=np.int64)
        tr_of = {int(c): i for i, c in enumerate(self.trace_code)}
        rt = np.array([tr_of[int(c)] for c in tb.trace[rows]], dtype=np.int64)
        ot = {k: [] for k in self.traces}
        tnames, nnames = self.traces, self.nodes
        for t, n in zip(rt, rn):
            ot[tnames[t]].append(nnames[n])
        to = {k: [] for k in sorted(nnames)}
        for t, n in zip(rt, rn):
            to[nnames[n]].append(tnames[t])
        # children: merge of ParentSpanId == spanID, left (child) row order, then right row order
        oo = {k: [] for k in nnames}
        sp = tb.span[rows]
        order = np.argsort(sp, kind="stable")
        srt = sp[order]
        par = tb.parent[rows]
        lo = np.searchsorted(srt, par, "left")
        hi = np.searchsorted(srt, par, "right")
        for i in range(rows.size):
            if par[i] < 0:
                continue
            for j in order[lo[i]:hi[i]]:
                oo[nnames[rn[j]]].append(nnames[rn[i]])
        self._lists = {"operation_operation": oo, "operation_trace": ot, "trace_operation": to, "pr_trace": ot}
        return self._lists


class GraphDicts(Mapping):
    """Read-only mapping with the reference's key order; list values materialise on demand."""

    def __init__(self, owner: PagerankGraph, kind: str):
        self.owner = owner
        self.kind = kind

    def _keys(self):
        o = self.owner
        if self.kind == "operation_operation":
            return o.nodes
        if self.kind == "trace_operation":
            return sorted(o.nodes)
        return o.traces

    def __iter__(self):
        return iter(self._keys())

    def __len__(self):
        if self.kind in ("operation_trace", "pr_trace"):
            return self.owner.T
        return len(self._keys())

    def __getitem__(self, k):
        return self.owner._materialise()[self.kind][k]

    def __contains__(self, k):
        return k in self.owner._materialise()[self.kind]

    def keys(self):
        return list(self._keys())

    def __repr__(self):
        return f"<GraphDicts {self.kind}: {len(self)} keys on {self.owner._dg.ctx.device}>"


def get_pagerank_graph(trace_list, span_df: pd.DataFrame, *, ctx=None):
    """preprocess_data.py:146-171 on the GPU (K1).  Returns (operation_operation,
    operation_trace, trace_operation, pr_trace) as lazy mappings backed by the device graph."""
    ctx = ctx or _lib.default_context()
    table, dev = span_table(span_df, ctx, GRAPH_READS)
    mask = np.zeros(table.n_traces, np.uint8)
    codes = trace_list.codes_for(table) if hasattr(trace_list, "codes_for") else None
    if codes is not None:   # a list system_anomaly_detect returned for this table: its codes
        mask[codes] = 1
    else:
        index = table.meta.get("trace_index")
        if index is None:
            index = table.meta["trace_index"] = {n: i for i, n in enumerate(table.trace_names)}
        for t in trace_list:
            i = index.get(t)
            if i is not None:
                mask[i] = 1
    return PagerankGraph(ctx, table, dev, mask).as_tuple()
