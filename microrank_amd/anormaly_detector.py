"""Drop-in for the reference module ``anormaly_detector`` (anormaly_detector.py).

* ``get_slo`` -- the reference version is broken (T16: it passes ``span_list=`` to
  ``get_operation_slo`` and treats ``start_time`` as the DataFrame, anormaly_detector.py:22-27).
  Here it takes the span DataFrame (optionally windowed) and returns what
  ``get_operation_slo(get_service_operation_list(df), df)`` returns, computed on the GPU (K4).
* ``system_anomaly_detect`` -- the 3-sigma trace detector (anormaly_detector.py:44-84) on the
  GPU (K5): same prints, same return value (``(flag, abnormal, normal)``, or ``False`` for an
  empty window), same list order (sorted traceIDs).
* ``trace_anormaly_detect`` / ``trace_list_partition`` -- the reference's unused per-trace
  helpers (anormaly_detector.py:101-139), kept for API completeness (host dict logic).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import ptr
from .preprocess_data import DETECT_READS, get_operation_slo, get_service_operation_list, get_span, span_table
from .spans import to_ns


def get_slo(span_df, start_time=None, end_time=None, *, ctx=None):
    """SLO of every service operation of ``span_df`` (optionally restricted to the window)."""
    df = get_span(span_df, start_time, end_time)
    df = df.copy() if df is not span_df else df
    operation_list = get_service_operation_list(df)
    return get_operation_slo(operation_list, df, ctx=ctx)


def slo_arrays(table, slo):
    """a3[op] = mean + 3 * std per service-op code (the detector's per-op expectation)."""
    n = table.n_svcops
    a3 = np.zeros(n, np.float64)
    ok = np.zeros(n, np.uint8)
    for code, name in enumerate(table.svcop_names):
        v = slo.get(name) if isinstance(slo, dict) else None
        if v is None:
            continue
        try:
            a3[code] = v[0] + 3 * v[1]          # anormaly_detector.py:64-65
            ok[code] = 1
        except Exception:                        # the reference's bare except adds 0
            pass
    return a3, ok


def detect_states(data, start_time, end_time, slo, *, ctx=None):
    """(state per trace code, n_abnormal, n_normal, table) or None for an empty window."""
    ctx = ctx or _lib.default_context()
    table, dev = span_table(data, ctx, DETECT_READS)
    a3, ok = slo_arrays(table, slo)
    state = np.zeros(table.n_traces, np.uint8)
    na, nn, nin = C.c_int32(), C.c_int32(), C.c_int64()
    rc = _lib.load().mr_detect(ctx.h, dev.h, to_ns(start_time), to_ns(end_time), ptr(a3, C.c_double),
                               ptr(ok, C.c_uint8), ptr(state, C.c_uint8), C.byref(na), C.byref(nn), C.byref(nin))
    if rc == _lib.MR_ERR_VALUE and nin.value == 0:
        return None
    ctx.check(rc, "mr_detect")
    return state, na.value, nn.value, table


class TraceList(list):
    """The detector's trace lists: plain lists of traceIDs (sorted, as the reference returns them)
    that also remember their trace codes in the span table they came from, so the driver's next
    call, get_pagerank_graph(list, data), selects them without a Python lookup per trace."""

    __slots__ = ("_mr_codes", "_mr_table")

    @classmethod
    def of(cls, table, codes):
        names = table.meta.get("trace_names_arr")
        if names is None:
            names = table.meta["trace_names_arr"] = np.asarray(table.trace_names, dtype=object)
        out = cls(names[codes].tolist())
        out._mr_codes, out._mr_table = codes, table
        return out

    def codes_for(self, table):
        """The trace codes when this list is unchanged and from ``table``, else None."""
        c = getattr(self, "_mr_codes", None)
        if c is None or getattr(self, "_mr_table", None) is not table or len(self) != c.size:
            return None
        if c.size and (self[0] != table.trace_names[c[0]] or self[-1] != table.trace_names[c[-1]]):
            return None
        return c


def system_anomaly_detect(data, start_time, end_time, slo, operation_list, *, ctx=None):
    """anormaly_detector.system_anomaly_detect on the GPU (anormaly_detector.py:44-84)."""
    res = detect_states(data, start_time, end_time, slo, ctx=ctx)
    if res is None:
        print("Error: Current span list is empty ")
        return False
    state, na, nn, table = res
    abnormal_list = TraceList.of(table, np.flatnonzero(state == 2))
    normal_list = TraceList.of(table, np.flatnonzero(state == 1))
    print("anormaly_trace", na)
    print("total_trace", na + nn)
    print()
    return (True if na else False), abnormal_list, normal_list


def trace_anormaly_detect(operation_list, slo):
    """anormaly_detector.py:101-113 (unused by the driver)."""
    expect_duration = 0.0
    real_duration = float(operation_list["duration"]) / 1000.0
    for operation in operation_list:
        if operation == "duration":
            continue
        expect_duration += operation_list[operation] * (slo[operation][0] + slo[operation][1])
    return real_duration > expect_duration + 50


def trace_list_partition(operation_count, slo):
    """anormaly_detector.py:128-139 (unused by the driver)."""
    abnormal_list, normal_list = [], []
    for traceid in operation_count:
        (abnormal_list if trace_anormaly_detect(operation_count[traceid], slo) else normal_list).append(traceid)
    return abnormal_list, normal_list
