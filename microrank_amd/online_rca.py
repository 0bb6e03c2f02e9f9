"""Drop-in for the reference module ``online_rca`` (online_rca.py).

* ``calculate_spectrum_without_delay_list`` -- the weighted spectrum scores and the stable
  top list (online_rca.py:33-152), computed on the GPU (K3, csrc/mr_spectrum.hip); printing,
  argument names and return types as in the reference.
* ``online_anomaly_detect_RCA`` -- the sliding-window driver (online_rca.py:155-216), line for
  line the same control flow, with every ranking step on the GPU.
* ``rca_window`` -- one whole window (detect -> 2 graphs -> 2 PageRanks -> spectrum) in a
  single C-ABI call with every intermediate resident in HBM (used by bench.py).
"""
from __future__ import annotations

import csv
import ctypes as C
import math
import time

import numpy as np
import pandas as pd

from . import _lib
from ._lib import SPECTRUM_METHODS, ptr
from .anormaly_detector import slo_arrays, system_anomaly_detect, trace_list_partition  # noqa: F401
from .pagerank import trace_pagerank
from .preprocess_data import (SpanStream, get_operation_duration_data, get_operation_slo, get_pagerank_graph,  # noqa: F401
                              get_service_operation_list, get_span, span_table)
from .spans import to_ns


def timestamp(datetime):
    """online_rca.py:26-30."""
    return int(time.mktime(time.strptime(str(datetime), "%Y-%m-%d %H:%M:%S"))) * 1000


def _is_np(v) -> bool:
    return isinstance(v, np.generic)


def calculate_spectrum_without_delay_list(anomaly_result, normal_result, anomaly_list_len, normal_list_len, top_max,
                                          normal_num_list, anomaly_num_list, spectrum_method, *, ctx=None):
    """online_rca.calculate_spectrum_without_delay_list on MI355X."""
    nodes = list(anomaly_result)
    nodes += [k for k in normal_result if k not in anomaly_result]
    n = len(nodes)
    has_a = np.zeros(n, np.uint8)
    has_n = np.zeros(n, np.uint8)
    a_w = np.zeros(n, np.float64)
    n_w = np.zeros(n, np.float64)
    a_num = np.zeros(n, np.int64)
    n_num = np.zeros(n, np.int64)
    kinds = []   # (a numpy-typed, n numpy-typed) per node, for the result type
    for i, node in enumerate(nodes):
        ta = tn = False
        if node in anomaly_result:
            w = anomaly_result[node]
            a_w[i] = w
            a_num[i] = anomaly_num_list[node]          # KeyError as in the reference (:49)
            ta = _is_np(w)
            has_a[i] = 1 | (2 if ta else 0)
        if node in normal_result:
            w = normal_result[node]
            n_w[i] = w
            n_num[i] = normal_num_list[node]
            tn = _is_np(w)
            has_n[i] = 1 | (2 if tn else 0)
        kinds.append((ta, tn))
    try:
        method = SPECTRUM_METHODS.index(spectrum_method)
    except ValueError:
        return [], []                                  # no branch matched: empty result (:77-142)
    if n == 0:
        return [], []
    ctx = ctx or _lib.default_context()
    k = max(0, min(n, top_max + 6))
    idx = np.zeros(max(k, 1), np.int32)
    sc = np.zeros(max(k, 1), np.float64)
    n_out, zd = C.c_int32(), C.c_int32()
    ctx.check(_lib.load().mr_spectrum(ctx.h, n, ptr(has_a, C.c_uint8), ptr(a_w, C.c_double), ptr(a_num, C.c_int64),
                                      ptr(has_n, C.c_uint8), ptr(n_w, C.c_double), ptr(n_num, C.c_int64),
                                      int(anomaly_list_len), int(normal_list_len), method, k, ptr(idx, C.c_int32),
                                      ptr(sc, C.c_double), C.byref(n_out), C.byref(zd)), "mr_spectrum")
    if zd.value:
        raise ZeroDivisionError("float division by zero")
    top_list, score_list = [], []
    for j in range(n_out.value):
        i = int(idx[j])
        ta, tn = kinds[i]
        ha, hn = bool(has_a[i] & 1), bool(has_n[i] & 1)
        if spectrum_method == "ochiai":          # ef / math.sqrt(...): the type of ef decides
            res_np = ta if ha else False
        else:
            res_np = (ta or (tn and hn)) if ha else tn
        s = np.float64(sc[j]) if res_np else float(sc[j])
        top_list.append(nodes[i])
        score_list.append(s)
        print("%-50s: %.8f" % (nodes[i], s))
    return top_list, score_list


def _write_result(top_list, score_list):
    ranked = sorted(zip(top_list, score_list), key=lambda x: x[1], reverse=True)
    with open("result.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["level", "result", "rank", "confidence"])
        for rank, (service, score) in enumerate(ranked, start=1):
            w.writerow(["span", service, rank, float(score)])


def sweep_plan(ctx, table, dev, a3, ok, t_begin: int, t_end: int, step_normal: int, step_abnormal: int):
    """SURVEY 8(f) f3 on a resident span table: the detector counts of every window start the
    driver's chain can reach (online_rca.py:161-216: starts t_begin + m * grain while < t_end,
    grain = gcd of the two steps) from ONE device pass (mr_detect_sweep).  None when the table's
    window times vary within a trace (the per-window loop applies then)."""
    grain = math.gcd(step_normal, step_normal + step_abnormal)
    n_win = -(-(t_end - t_begin) // grain)
    if n_win <= 0 or n_win > 1 << 24:
        return None
    na, nn, rows = np.zeros(n_win, np.int32), np.zeros(n_win, np.int32), np.zeros(n_win, np.int64)
    rc = _lib.load().mr_detect_sweep(ctx.h, dev.h, t_begin, grain, step_normal, n_win, ptr(a3, C.c_double),
                                     ptr(ok, C.c_uint8), None, ptr(na, C.c_int32), ptr(nn, C.c_int32),
                                     ptr(rows, C.c_int64))
    if rc == _lib.MR_ERR_STATE:
        return None
    ctx.check(rc, "mr_detect_sweep")
    return dict(ctx=ctx, table=table, dev=dev, a3=a3, ok=ok, t_begin=t_begin, grain=grain,
                step_n=step_normal // grain, step_a=step_abnormal // grain, n_win=n_win, na=na, nn=nn, rows=rows)


def sweep_chain(plan):
    """Walk the driver's window chain over the sweep's counts -- only the counts decide the next
    start: ("window", m, n_abnormal, n_normal, ranked) per visited window, ("empty", m) where the
    reference's detector returns False (T2) and the chain stops."""
    events, m = [], 0
    while m < plan["n_win"]:
        if plan["rows"][m] == 0:
            events.append(("empty", m))
            break
        na, nn = int(plan["na"][m]), int(plan["nn"][m])
        ranked = na > 0 and nn > 0
        events.append(("window", m, na, nn, ranked))
        m += plan["step_n"] + (plan["step_a"] if ranked else 0)
    plan["next_m"] = m   # where the chain goes on (RCAStream)
    return events


def sweep_rank(plan, events, precision="fp64"):
    """Every ranked window of the chain in ONE mr_windows_batch call: {m: (codes, scores, ...)}."""
    todo = [e[1] for e in events if e[0] == "window" and e[4]]
    width = plan["step_n"] * plan["grain"]
    if not todo:
        return {}
    wins = [(plan["dev"], plan["t_begin"] + mm * plan["grain"], plan["t_begin"] + mm * plan["grain"] + width,
             plan["a3"], plan["ok"]) for mm in todo]
    return dict(zip(todo, rank_windows(plan["ctx"], wins, precision=precision)))


def _sweep_plan(data, slo, start, end, window_normal, window_abnormal, ctx):
    """The driver's sweep plan for a DataFrame (None: not applicable -- no datetime window columns,
    an empty frame, or times that vary within a trace)."""
    if len(data) == 0 or not all(np.issubdtype(data[c].dtype, np.datetime64) for c in ("startTime", "endTime")):
        return None
    if pd.isna(start) or pd.isna(end) or not start < end:
        return None
    ctx = ctx or _lib.default_context()
    table, dev = span_table(data, ctx)
    return _sweep_plan_dev(table, dev, slo, start, end, window_normal, window_abnormal, ctx)


def _sweep_plan_dev(table, dev, slo, start, end, window_normal, window_abnormal, ctx):
    """_sweep_plan over a resident device table (RCAStream's appended one)."""
    if pd.isna(start) or pd.isna(end) or not start < end:
        return None
    a3, ok = slo_arrays(table, slo)
    return sweep_plan(ctx, table, dev, a3, ok, int(pd.Timestamp(start).value), int(pd.Timestamp(end).value),
                      int(window_normal.value), int(window_abnormal.value))


def _sweep_run(plan):
    """The chain, one batched ranking of its triggered windows, then the driver's output replayed
    in window order; an empty window raises the reference's TypeError (T2) after the output of
    the windows before it."""
    events = sweep_chain(plan)
    _sweep_emit(plan, events, sweep_rank(plan, events))


def _sweep_emit(plan, events, results):
    names = plan["table"].podop_names
    for e in events:
        if e[0] == "empty":
            print("Error: Current span list is empty ")
            anomaly_flag, normal_list, abnormal_list = False   # noqa: F841 -- TypeError, as the reference (T2)
        _, mm, na, nn, ranked = e
        print("anormaly_trace", na)                       # anormaly_detector.py:74-76
        print("total_trace", na + nn)
        print()
        if not na:
            continue
        print("anomaly_list", nn)                         # T1: the driver's abnormal_list is the
        print("normal_list", na)                          # detector's normal list
        print("total", na + nn)
        if not ranked:
            continue
        codes, scores, r_na, r_nn, _edges, status = results[mm]
        if status != _lib.MR_OK or (r_na, r_nn) != (na, nn):
            raise RuntimeError(f"window {mm}: batch ranking disagrees with the sweep (status {status})")
        top_list = [names[c] for c in codes] if names is not None else codes.tolist()
        score_list = [np.float64(x) for x in scores]    # dstar2 over np.float64 weights
        for node, sc in zip(top_list, score_list):
            print("%-50s: %.8f" % (node, sc))             # online_rca.py:151
        print(top_list, score_list)
        _write_result(top_list, score_list)


def online_anomaly_detect_RCA(data, slo, operation_list, *, ctx=None):
    """online_rca.online_anomaly_detect_RCA (online_rca.py:155-216): 5-minute windows, a triggered
    window advances by 9 minutes; the detector's lists are unpacked swapped (T1), an empty
    window makes the unpacking raise TypeError (T2); result.csv is rewritten per trigger.

    With trace-level window times (the renamed TraceStart/TraceEnd, online_rca.py:229-230) the
    whole sweep runs as one device detector pass, one batched ranking of the triggered windows
    and a replay of the output (f3, :func:`_sweep_run`); otherwise window by window."""
    window_normal = pd.Timedelta(minutes=5)
    window_abnormal = pd.Timedelta(minutes=4)
    start = data["startTime"].min()
    end = data["endTime"].max()
    plan = _sweep_plan(data, slo, start, end, window_normal, window_abnormal, ctx)
    if plan is not None:
        return _sweep_run(plan)
    _window_loop(data, slo, operation_list, start, end)


def _window_loop(data, slo, operation_list, current_time, end):
    """online_rca.py:164-216 window by window from current_time while it is before end; returns
    where the chain goes on."""
    window_normal = pd.Timedelta(minutes=5)
    window_abnormal = pd.Timedelta(minutes=4)
    while current_time < end:
        start_time = current_time
        end_time = current_time + window_normal
        anomaly_flag, normal_list, abnormal_list = system_anomaly_detect(
            data, start_time=start_time, end_time=end_time, slo=slo, operation_list=operation_list)
        if anomaly_flag:
            print("anomaly_list", len(abnormal_list))
            print("normal_list", len(normal_list))
            print("total", len(normal_list) + len(abnormal_list))
            if not abnormal_list or not normal_list:
                current_time += window_normal
                continue
            n_graph = get_pagerank_graph(normal_list, data)
            normal_trace_result, normal_num_list = trace_pagerank(*n_graph, False)
            a_graph = get_pagerank_graph(abnormal_list, data)
            anomaly_trace_result, anomaly_num_list = trace_pagerank(*a_graph, True)
            top_list, score_list = calculate_spectrum_without_delay_list(
                anomaly_result=anomaly_trace_result, normal_result=normal_trace_result,
                anomaly_list_len=len(abnormal_list), normal_list_len=len(normal_list), top_max=5,
                anomaly_num_list=anomaly_num_list, normal_num_list=normal_num_list, spectrum_method="dstar2")
            print(top_list, score_list)
            _write_result(top_list, score_list)
            current_time += window_abnormal
        current_time += window_normal
    return current_time


class RCAStream:
    """SURVEY 8(f) f3, online: online_anomaly_detect_RCA (online_rca.py:161-216) over spans that
    arrive in chunks.  Each chunk holds whole traces and chunks come in trace-start order (the
    OTel export's TraceStart order); push() ranks every window of the driver's chain that the data
    seen so far completes (a window [t, t + 5 min] is complete once a trace starting after t + 5 min
    has arrived), close() the rest up to the last endTime, as the offline driver would.  The
    output -- prints, result.csv, the T2 TypeError -- equals the offline driver's on the
    concatenated chunks.  Spans of traces that start before the chain's next window are dropped,
    so the resident table stays a few windows long; each push re-ingests that table on the device
    (mr_spans_ingest) and runs the chain's new windows as one sweep + one batched ranking."""

    WINDOW = pd.Timedelta(minutes=5)
    STEP_ABNORMAL = pd.Timedelta(minutes=4)

    def __init__(self, slo, operation_list, *, ctx=None, device_append=True):
        self.slo, self.operation_list = slo, operation_list
        self.ctx = ctx or _lib.default_context()
        self.data = None          # retained spans as a DataFrame (host mode only)
        self.cur = None           # the chain's next window start (pd.Timestamp)
        self.watermark = None     # largest trace start seen
        self.end = None           # largest trace end seen (the offline driver's loop bound)
        self.dead = False         # an empty window ended the driver (T2)
        # device mode (default): the resident table lives in HBM and grows by mr_spans_append, so
        # a push costs O(chunk) on the host and across PCIe; the chunk frames are kept (by
        # reference) only for the per-window fallback.  Host mode: pd.concat + a full re-ingest.
        self._stream = SpanStream(self.ctx) if device_append else None
        self._frames = []         # (chunk, its largest trace start) of the device mode
        self._empty = None        # a zero-row frame with the chunks' columns

    def push(self, chunk: pd.DataFrame):
        if self.dead:
            raise RuntimeError("RCAStream: the driver ended at an empty window")
        if len(chunk) == 0:
            return
        lo, hi, e = chunk["startTime"].min(), chunk["startTime"].max(), chunk["endTime"].max()
        if self.cur is None:
            self.cur = lo
        elif self.watermark is not None and lo < self.watermark:
            raise ValueError("RCAStream.push: chunks must arrive in trace-start order")
        self.watermark = hi if self.watermark is None else max(self.watermark, hi)
        self.end = e if self.end is None else max(self.end, e)
        arrays = SpanStream.accepts(chunk) if self._stream is not None else None
        if arrays is not None:
            self._stream.append(chunk, int(pd.Timestamp(self.cur).value), arrays)
            self._frames.append((chunk, hi))
            self._empty = chunk.iloc[:0]
        else:
            if self._stream is not None:   # a chunk the device append cannot take: host mode from here
                self.data = self._frame()
                self._stream.close()
                self._stream, self._frames = None, []
            self.data = chunk if self.data is None else pd.concat([self.data, chunk], ignore_index=True)
        # complete windows: start + 5 min < watermark
        self._advance(self.watermark - self.WINDOW, final=False)

    def close(self):
        if self.dead or (self.data is None if self._stream is None else self._stream.dev is None):
            return
        self._advance(self.end, final=True)

    def _frame(self):
        """The resident spans as a DataFrame (device mode: from the kept chunk frames)."""
        if self._stream is None:
            return self.data
        if not self._frames:
            return self._empty
        df = pd.concat([f for f, _ in self._frames], ignore_index=True) if len(self._frames) > 1 else self._frames[0][0]
        keep = df["startTime"] >= self.cur
        return df if keep.all() else df[keep].reset_index(drop=True)

    def _advance(self, limit, final):
        if not self.cur < limit:
            return
        try:
            if self._stream is not None:
                plan = _sweep_plan_dev(self._stream.table, self._stream.dev, self.slo, self.cur, limit, self.WINDOW,
                                       self.STEP_ABNORMAL, self.ctx)
            else:
                plan = _sweep_plan(self.data, self.slo, self.cur, limit, self.WINDOW, self.STEP_ABNORMAL, self.ctx)
            if plan is None:   # window times vary within a trace: window by window
                data = self._frame()
                if final:
                    self.cur = _window_loop(data, self.slo, self.operation_list, self.cur, limit)
                else:
                    self.cur = self._loop_complete(data, limit)
            else:
                events = sweep_chain(plan)
                _sweep_emit(plan, events, sweep_rank(plan, events))
                self.cur = self.cur + pd.Timedelta(plan["next_m"] * plan["grain"], unit="ns")
        except TypeError:
            self.dead = True
            raise
        if self._stream is not None:   # frames whose every trace started before the next window go
            self._frames = [(f, h) for f, h in self._frames if h >= self.cur]
            return
        keep = self.data["startTime"] >= self.cur   # traces before the next window leave the table
        if not keep.all():
            self.data = self.data[keep].reset_index(drop=True)

    def _loop_complete(self, data, limit):
        """The window loop for per-span times, one window at a time while its start is before limit."""
        cur = self.cur
        while cur < limit:
            nxt = _window_loop(data, self.slo, self.operation_list, cur, cur + pd.Timedelta(1, unit="ns"))
            cur = nxt
        return cur


def rca_window(data, start_time, end_time, slo, *, top_max=5, spectrum_method="dstar2", precision="fp64", ctx=None,
               table=None, dev=None):
    """One RCA window entirely on the device (mr_rca_window).  Returns a dict with the top list
    (pod-op names), scores, the detector counts and the edges traversed by the two PageRanks."""
    ctx = ctx or _lib.default_context()
    if table is None or dev is None:
        table, dev = span_table(data, ctx)
    a3, ok = slo_arrays(table, slo)
    k = max(top_max + 6, 1)
    codes = np.zeros(k, np.int32)
    scores = np.zeros(k, np.float64)
    n_out, na, nn, edges = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64()
    method = SPECTRUM_METHODS.index(spectrum_method)
    prec = _lib.MR_FP32 if precision == "fp32" else _lib.MR_FP64
    ctx.check(_lib.load().mr_rca_window(ctx.h, dev.h, to_ns(start_time), to_ns(end_time), ptr(a3, C.c_double),
                                        ptr(ok, C.c_uint8), method, top_max, prec, ptr(codes, C.c_int32),
                                        ptr(scores, C.c_double), C.byref(n_out), C.byref(edges), C.byref(na),
                                        C.byref(nn)), "mr_rca_window")
    m = n_out.value
    names = table.podop_names
    return {"top": [names[c] for c in codes[:m]] if names is not None else codes[:m].tolist(),
            "score": scores[:m].tolist(), "n_abnormal": na.value, "n_normal": nn.value, "edges": edges.value}


def rank_windows(ctx, windows, *, top_max=5, spectrum_method="dstar2", precision="fp64"):
    """C3: many RCA windows in one call (mr_windows_batch).  ``windows``: a list of
    (DeviceSpans, t0_ns, t1_ns, a3, a3_valid) (the SLO arrays over the table's service-op
    codes).  Returns per window (top pod-op codes, scores, n_abnormal, n_normal, edges, status);
    status MR_ERR_VALUE marks an empty window (the reference raises TypeError there, T2)."""
    n = len(windows)
    k = max(top_max + 6, 1)
    keep = [np.ascontiguousarray(w[3], np.float64) for w in windows] + \
           [np.ascontiguousarray(w[4], np.uint8) for w in windows]
    spans = (_lib.P * max(n, 1))(*[w[0].h for w in windows])
    t0 = np.array([int(w[1]) for w in windows], np.int64)
    t1 = np.array([int(w[2]) for w in windows], np.int64)
    a3 = (C.c_void_p * max(n, 1))(*[a.ctypes.data for a in keep[:n]])
    ok = (C.c_void_p * max(n, 1))(*[a.ctypes.data for a in keep[n:]])
    codes = np.zeros(max(n, 1) * k, np.int32)
    scores = np.zeros(max(n, 1) * k, np.float64)
    n_out, edges, na, nn, status = (np.zeros(max(n, 1), t) for t in (np.int32, np.int64, np.int32, np.int32, np.int32))
    method = SPECTRUM_METHODS.index(spectrum_method)
    prec = _lib.MR_FP32 if precision == "fp32" else _lib.MR_FP64
    ctx.check(_lib.load().mr_windows_batch(ctx.h, n, spans, ptr(t0, C.c_int64), ptr(t1, C.c_int64), a3, ok, method,
                                           top_max, prec, ptr(codes, C.c_int32), ptr(scores, C.c_double),
                                           ptr(n_out, C.c_int32), ptr(edges, C.c_int64), ptr(na, C.c_int32),
                                           ptr(nn, C.c_int32), ptr(status, C.c_int32)), "mr_windows_batch")
    return [(codes[i * k:i * k + n_out[i]].copy(), scores[i * k:i * k + n_out[i]].copy(), int(na[i]), int(nn[i]),
             int(edges[i]), int(status[i])) for i in range(n)]
