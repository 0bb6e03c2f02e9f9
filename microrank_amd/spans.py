"""Int-coded columnar span table: the wire format between pandas and the HIP kernels.

The reference keeps spans in a pandas DataFrame of strings (schema renamed at
``online_rca.py:221-244`` from the OTel export of ``collect_data.py:35-46``) and
re-derives operation names with string concatenation in every function
(``preprocess_data.py:26-32, 53-57, 100-104, 151-155``).  Here that work is
done ONCE per DataFrame: every string column becomes an int32/int64 code whose
integer order equals the code-point (Python ``str``) order of the strings, so
"sorted by name" in the reference (pandas ``groupby`` sort, T10) is "sorted by
code" on the device.

Two operation namespaces exist (T10):
  * ``svcop`` = ``serviceName + '_' + op``  -- SLO / detector (preprocess_data.py:29-30,55-56,102-103)
  * ``podop`` = ``podName + '_' + op``      -- PageRank graph    (preprocess_data.py:151-155)
where ``op`` drops the last ``/segment`` for service ``ts-ui-dashboard``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

UI_SERVICE = "ts-ui-dashboard"


def op_display(service: np.ndarray, operation: np.ndarray) -> np.ndarray:
    """Operation part of a name: ``rsplit('/', 1)[0]`` for ts-ui-dashboard spans
    (preprocess_data.py:28-30), the raw operationName otherwise."""
    out = np.array(operation, dtype=object, copy=True)
    ui = np.asarray(service, dtype=object) == UI_SERVICE
    if ui.any():
        out[ui] = [s.rsplit("/", 1)[0] if isinstance(s, str) else s for s in out[ui]]
    return out


def _factorize_sorted(values: np.ndarray):
    """codes, uniques with uniques in Python string order (what pandas' groupby sort uses)."""
    import pandas as pd

    codes, uniques = pd.factorize(pd.Series(values, dtype=object), sort=True)
    return codes.astype(np.int32), list(uniques)


@dataclass
class SpanTable:
    """Columns are in DataFrame row order (row order fixes first-appearance order, T10)."""

    trace: np.ndarray                 # int32  trace code, rank of traceID in sorted order
    podop: np.ndarray                 # int32  podName_op code (graph node namespace)
    svcop: np.ndarray                 # int32  serviceName_op code (SLO namespace)
    span: np.ndarray                  # int64  spanID code (duplicates share a code)
    parent: np.ndarray                # int64  code of ParentSpanId in the spanID dictionary, -1 if none
    duration: np.ndarray              # int64  span duration (reference divides by 1000 -> ms)
    tstart: Optional[np.ndarray] = None   # int64 ns, trace-level start (renamed TraceStart)
    tend: Optional[np.ndarray] = None     # int64 ns, trace-level end (renamed TraceEnd)
    trace_names: Optional[Sequence[str]] = None
    podop_names: Optional[Sequence[str]] = None
    svcop_names: Optional[Sequence[str]] = None
    meta: dict = field(default_factory=dict)
    row: Optional[np.ndarray] = None      # int32 global row index (a shard of a larger table), else None

    @property
    def n_spans(self) -> int:
        return int(self.trace.shape[0])

    @property
    def n_traces(self) -> int:
        return len(self.trace_names) if self.trace_names is not None else int(self.trace.max()) + 1

    @property
    def n_podops(self) -> int:
        return len(self.podop_names) if self.podop_names is not None else int(self.podop.max()) + 1

    @property
    def n_svcops(self) -> int:
        return len(self.svcop_names) if self.svcop_names is not None else int(self.svcop.max()) + 1

    def check(self) -> None:
        S = self.n_spans
        for name in ("trace", "podop", "svcop", "span", "parent", "duration"):
            a = getattr(self, name)
            if a.shape != (S,):
                raise ValueError(f"SpanTable.{name}: shape {a.shape} != ({S},)")
        if S and (self.trace.min() < 0 or self.podop.min() < 0 or self.svcop.min() < 0):
            raise ValueError("SpanTable: negative trace/op code")

    def take(self, rows: np.ndarray) -> "SpanTable":
        """Row subset (keeps dictionaries, so codes stay comparable)."""
        pick = lambda a: None if a is None else a[rows]
        return SpanTable(self.trace[rows], self.podop[rows], self.svcop[rows], self.span[rows],
                         self.parent[rows], self.duration[rows], pick(self.tstart), pick(self.tend),
                         self.trace_names, self.podop_names, self.svcop_names, dict(self.meta), pick(self.row))

    def shard(self, rank: int, world: int) -> "SpanTable":
        """This rank's traces (trace code % world == rank) with every span of each, codes and
        dictionaries global, and the global row index of each row (first appearance, T10): the
        per-rank table of a trace-sharded deployment (mr_graph_build_sharded)."""
        rows = np.flatnonzero(self.trace % world == rank)
        sub = self.take(rows)
        sub.row = (self.row[rows] if self.row is not None else rows).astype(np.int32)
        for attr, n in (("trace_names", self.n_traces), ("podop_names", self.n_podops), ("svcop_names", self.n_svcops)):
            if getattr(sub, attr) is None:   # code spaces stay the whole table's
                setattr(sub, attr, range(n))
        return sub

    # ------------------------------------------------------------------ ingest
    @classmethod
    def from_dataframe(cls, df) -> "SpanTable":
        """Factorise a reference-schema DataFrame (traceID, spanID, ParentSpanId, serviceName,
        operationName, podName, duration[, startTime, endTime])."""
        svc = df["serviceName"].to_numpy(dtype=object)
        op = op_display(svc, df["operationName"].to_numpy(dtype=object))
        svcop = np.array([f"{a}_{b}" for a, b in zip(svc, op)], dtype=object)
        pod = df["podName"].to_numpy(dtype=object)
        podop = np.array([f"{a}_{b}" for a, b in zip(pod, op)], dtype=object)
        tcode, tnames = _factorize_sorted(df["traceID"].to_numpy(dtype=object))
        pcode, pnames = _factorize_sorted(podop)
        scode, snames = _factorize_sorted(svcop)
        import pandas as pd

        sid_codes, sid_uniques = pd.factorize(df["spanID"])
        par = pd.Index(sid_uniques).get_indexer(df["ParentSpanId"]) if "ParentSpanId" in df else \
            np.full(len(df), -1)
        tstart = tend = None
        if "startTime" in df and "endTime" in df:
            tstart = _as_ns(df["startTime"])
            tend = _as_ns(df["endTime"])
        return cls(tcode, pcode, scode, sid_codes.astype(np.int64), np.asarray(par, dtype=np.int64),
                   df["duration"].to_numpy(dtype=np.int64), tstart, tend, tnames, pnames, snames)


# ------------------------------------------------------------------ the OTel CSV export (f2)
# collect_data.py:35-46 exports TraceId, SpanId, ParentSpanId, SpanName, ServiceName, PodName,
# Duration, TraceStart, TraceEnd (plus Timestamp, SpanKind); online_rca.py:221-232 renames them
OTEL_RENAME = {"TraceId": "traceID", "ServiceName": "serviceName", "SpanName": "operationName", "PodName": "podName",
               "SpanId": "spanID", "Duration": "duration", "TraceStart": "startTime", "TraceEnd": "endTime"}


def read_traces_csv(path):
    """``pd.read_csv(path).rename(columns=...)`` + ``pd.to_datetime`` of online_rca.py:221-248
    through pyarrow's multithreaded CSV reader: the string columns stay Arrow-backed
    (``string[pyarrow]``), so the device ingest (mr_spans_ingest) takes their buffers without a
    Python-object round trip.  Empty fields read as missing, as pandas reads them."""
    import pandas as pd
    import pyarrow as pa
    import pyarrow.csv as pv

    t = pv.read_csv(path, convert_options=pv.ConvertOptions(strings_can_be_null=True))
    t = t.rename_columns([OTEL_RENAME.get(c, c) for c in t.column_names])
    df = t.to_pandas(types_mapper=lambda ty: pd.ArrowDtype(ty) if pa.types.is_string(ty) or pa.types.is_large_string(ty)
                     else None)
    for c in ("startTime", "endTime"):
        if c in df and not np.issubdtype(df[c].dtype, np.datetime64):
            df[c] = pd.to_datetime(df[c])
    return df


# ------------------------------------------------------------------ device ingest
_STR_COLS = ("traceID", "spanID", "ParentSpanId", "serviceName", "operationName", "podName")


def arrow_columns(df):
    """The string columns as Arrow large_string arrays (C++ conversion, no per-row Python), or
    None when a column is not all strings or a required one has nulls (the host factorisation of
    :meth:`SpanTable.from_dataframe` then builds the table)."""
    try:
        import pyarrow as pa
    except ImportError:  # pragma: no cover
        return None
    if any(c not in df.columns for c in _STR_COLS if c != "ParentSpanId") or len(df) == 0:
        return None
    out = {}
    for c in _STR_COLS:
        if c not in df.columns:   # no ParentSpanId column: every span a root
            out[c] = pa.nulls(len(df), type=pa.large_string())
            continue
        try:
            a = pa.array(df[c], type=pa.large_string(), from_pandas=True)
        except (pa.ArrowInvalid, pa.ArrowTypeError, TypeError):
            return None
        if isinstance(a, pa.ChunkedArray):
            a = a.combine_chunks()
        if c != "ParentSpanId" and a.null_count:
            return None
        out[c] = a
    return out


class IngestedTable:
    """SpanTable-compatible view of a table built on the device from strings (mr_spans_ingest):
    sizes and name lists come from the device dictionaries (the first row of each code); the code
    columns are copied back only if something asks for them (PagerankGraph list materialisation)."""

    def __init__(self, dev, arrays, duration, tstart, tend):
        from . import _lib

        self._dev, self._arrays = dev, arrays
        self.duration, self.tstart, self.tend = duration, tstart, tend
        self.meta, self.row = {}, None
        S, nt, npo, nsv = C_i64(), C_i32(), C_i32(), C_i32()
        _lib.load().mr_spans_info(dev.h, S, nt, npo, nsv)
        self.n_spans, self.n_traces, self.n_podops, self.n_svcops = S.value, nt.value, npo.value, nsv.value
        self._names = {}
        self._codes = None

    def _rows(self, which):
        import ctypes as C

        from . import _lib

        n = (self.n_traces, self.n_podops, self.n_svcops)[which]
        rows = np.zeros(max(n, 1), np.int32)
        self._dev.ctx.check(_lib.load().mr_spans_dict_rows(self._dev.h, which, rows.ctypes.data_as(C.POINTER(C.c_int32))),
                            "mr_spans_dict_rows")
        return rows[:n]

    def _take(self, col, rows):
        """Values of string column ``col`` at ``rows`` (as returned by :meth:`_rows`), a list."""
        import pyarrow as pa

        return self._arrays[col].take(pa.array(rows)).to_pylist()

    def _op_names(self, rows):
        svc = np.array(self._take("serviceName", rows), dtype=object)
        op = np.array(self._take("operationName", rows), dtype=object)
        return svc, op_display(svc, op)

    @property
    def trace_names(self):
        if "trace" not in self._names:
            self._names["trace"] = self._take("traceID", self._rows(0))
        return self._names["trace"]

    @property
    def podop_names(self):
        if "podop" not in self._names:
            rows = self._rows(1)
            _, op = self._op_names(rows)
            pod = self._take("podName", rows)
            self._names["podop"] = [f"{a}_{b}" for a, b in zip(pod, op)]
        return self._names["podop"]

    @property
    def svcop_names(self):
        if "svcop" not in self._names:
            rows = self._rows(2)
            svc, op = self._op_names(rows)
            self._names["svcop"] = [f"{a}_{b}" for a, b in zip(svc, op)]
        return self._names["svcop"]

    def _code_cols(self):
        if self._codes is None:
            import ctypes as C

            from . import _lib

            S = self.n_spans
            cols = [np.empty(S, np.int32), np.empty(S, np.int32), np.empty(S, np.int32), np.empty(S, np.int64),
                    np.empty(S, np.int64)]
            ptrs = [a.ctypes.data_as(C.POINTER(C.c_int32 if a.dtype == np.int32 else C.c_int64)) for a in cols]
            self._dev.ctx.check(_lib.load().mr_spans_codes(self._dev.h, *ptrs), "mr_spans_codes")
            self._codes = cols
        return self._codes

    trace = property(lambda self: self._code_cols()[0])
    podop = property(lambda self: self._code_cols()[1])
    svcop = property(lambda self: self._code_cols()[2])
    span = property(lambda self: self._code_cols()[3])
    parent = property(lambda self: self._code_cols()[4])

    def check(self) -> None:
        pass


def C_i64():
    import ctypes as C

    return C.c_int64()


def C_i32():
    import ctypes as C

    return C.c_int32()


def _as_ns(col) -> np.ndarray:
    import pandas as pd

    if np.issubdtype(col.dtype, np.datetime64):
        return col.to_numpy(dtype="datetime64[ns]").astype(np.int64)
    return pd.to_datetime(col).to_numpy(dtype="datetime64[ns]").astype(np.int64)


def to_ns(t) -> int:
    """A window boundary (pandas Timestamp / datetime64 / int ns) as int64 ns."""
    import pandas as pd

    if isinstance(t, (int, np.integer)):
        return int(t)
    return int(pd.Timestamp(t).value)
