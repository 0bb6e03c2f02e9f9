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
