"""Capture golden vectors by running the REFERENCE (/root/reference) in this container.

Run from the repo root:  python tests/golden/make_golden.py
The reference is imported read-only (no bytecode written) and never travels: only the
inputs (parquet / JSON) and the outputs it produced are committed under tests/golden/.
Floats are stored as ``float.hex`` strings so fixtures are bit-exact.

Environment recorded in ``manifest.json`` (numpy / pandas / OpenBLAS versions), because
the reference pins none of them.
"""
from __future__ import annotations

import contextlib
import io
import json
import math
import os
import sys
import tempfile
import time

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference")

import anormaly_detector as ref_det  # noqa: E402
import online_rca as ref_rca  # noqa: E402
import pagerank as ref_pr  # noqa: E402
import preprocess_data as ref_pp  # noqa: E402

from microrank_amd import synth  # noqa: E402

METHODS = ["dstar2", "ochiai", "jaccard", "sorensendice", "m1", "m2", "goodman", "tarantula",
           "russellrao", "hamann", "dice", "simplematcing", "rogers", "nosuchmethod"]


def fhex(x) -> str:
    return float(x).hex()


def dump_pr(weight, num):
    return {"keys": list(weight.keys()), "weight": [fhex(v) for v in weight.values()],
            "num_keys": list(num.keys()), "num": [int(v) for v in num.values()]}


def dump_graph(g, trace_names=None):
    """Compact form: ops as indices into ``nodes`` (the operation_operation key order), traces as
    indices into ``trace_names`` (sorted traceIDs of the DataFrame) when given."""
    oo, ot, to, pt = g
    nodes = list(oo.keys())
    if trace_names is None:
        return {"operation_operation": {k: list(v) for k, v in oo.items()},
                "operation_trace": {k: list(v) for k, v in ot.items()},
                "trace_operation": {k: list(v) for k, v in to.items()},
                "pr_trace": {k: list(v) for k, v in pt.items()}}
    ni = {n: i for i, n in enumerate(nodes)}
    ti = {n: i for i, n in enumerate(trace_names)}
    flat = lambda d, kmap, vmap: {"keys": [kmap[k] for k in d],
                                  "len": [len(v) for v in d.values()],
                                  "vals": [vmap[x] for v in d.values() for x in v]}
    return {"nodes": nodes,
            "operation_operation": flat(oo, ni, ni),
            "operation_trace": flat(ot, ti, ni),
            "trace_operation": flat(to, ni, ti),
            "pr_trace_is_operation_trace": all(list(pt[k]) == list(ot[k]) for k in ot) and list(pt) == list(ot)}


def run_spectrum_all(a_w, n_w, a_len, n_len, a_num, n_num):
    out = {}
    for m in METHODS:
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf), np.errstate(all="ignore"):
            try:
                top, score = ref_rca.calculate_spectrum_without_delay_list(
                    anomaly_result=a_w, normal_result=n_w, anomaly_list_len=a_len,
                    normal_list_len=n_len, top_max=5, normal_num_list=n_num,
                    anomaly_num_list=a_num, spectrum_method=m)
                out[m] = {"top": list(top), "score": [fhex(s) for s in score], "stdout": buf.getvalue()}
            except Exception as e:  # ZeroDivisionError etc. are part of the contract
                out[m] = {"error": type(e).__name__, "stdout": buf.getvalue()}
    return out


# --------------------------------------------------------------------------- dict-level cases
def fig3_dicts():
    """Paper Fig. 3 (pagerank.py:143-159 commented matrices) as the equivalent dicts."""
    oo = {"front": ["recommend", "checkout", "product"], "recommend": ["product"],
          "checkout": ["product"], "product": []}
    ot = {"t0": ["front", "product"], "t1": ["front", "checkout", "product"],
          "t2": ["front", "recommend", "product"]}
    to = {"front": ["t0", "t1", "t2"], "recommend": ["t2"], "checkout": ["t1"],
          "product": ["t0", "t1", "t2"]}
    return oo, ot, to, dict(ot)


def dict_edge_cases():
    cases = {}
    cases["fig3"] = fig3_dicts()
    # self loop, duplicated children (multiset), repeated ops inside a trace, identical traces
    oo = {"a": ["b", "b", "c", "a"], "b": ["d"], "c": [], "d": [], "e": []}
    ot = {"x1": ["a", "b", "b", "d"], "x2": ["a", "b", "b", "d"], "x3": ["a", "c"],
          "x4": ["a", "a", "c", "e"], "x5": ["e"]}
    to = {"a": ["x1", "x2", "x3", "x4", "x4"], "b": ["x1", "x1", "x2", "x2"], "c": ["x3", "x4"],
          "d": ["x1", "x2"], "e": ["x4", "x5"]}
    cases["multiset_selfloop"] = (oo, ot, to, dict(ot))
    # pr_trace differs from operation_trace: a subset with different lengths
    pt = {"x2": ["a", "b"], "x4": ["a", "a", "c", "e", "e", "e"], "x5": ["e"]}
    cases["pr_subset"] = (oo, ot, to, pt)
    # single op, single trace
    cases["single"] = ({"only": []}, {"t": ["only"]}, {"only": ["t"]}, {"t": ["only"]})
    # trace_operation incidence differs from operation_trace (not produced by the graph builder)
    to2 = dict(to)
    to2["e"] = ["x5"]
    cases["asym_incidence"] = (oo, ot, to2, dict(ot))
    return cases


# --------------------------------------------------------------------------- span-level cases
def make_windows(n_ops, n_traces, seed, **kw):
    """microrank_amd.synth.window_pair with the params recorded in the fixture."""
    return synth.window_dataframes(n_ops, n_traces, seed, **kw)


def span_case(name, params, outdir, driver=True):
    ndf, adf = make_windows(**params)
    res = {"name": name, "params": params}
    t0 = time.perf_counter()
    span_df = ndf.copy()
    op_list = ref_pp.get_service_operation_list(span_df)
    slo = ref_pp.get_operation_slo(op_list, span_df)
    res["operation_list"] = op_list
    res["slo"] = {k: [fhex(v[0]), fhex(v[1])] for k, v in slo.items()}
    start = adf["startTime"].min()
    end = start + pd.Timedelta(minutes=5)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        det = ref_det.system_anomaly_detect(adf, start_time=start, end_time=end, slo=slo,
                                            operation_list=op_list)
    flag, abn, nor = det
    tn = sorted(adf["traceID"].unique())
    ti = {n: i for i, n in enumerate(tn)}
    res["detect"] = {"flag": bool(flag), "abnormal": [ti[x] for x in abn], "normal": [ti[x] for x in nor],
                     "stdout": buf.getvalue(), "start_ns": int(start.value), "end_ns": int(end.value)}
    # the driver swaps the lists (T1): "normal" graph is built from the abnormal list
    g_n = ref_pp.get_pagerank_graph(abn, adf)
    g_a = ref_pp.get_pagerank_graph(nor, adf)
    tnames = sorted(adf["traceID"].unique())
    res["graph_swapped_normal"] = dump_graph(g_n, tnames)
    res["graph_swapped_anomaly"] = dump_graph(g_a, tnames)
    t1 = time.perf_counter()
    w_n, c_n = ref_pr.trace_pagerank(*g_n, False)
    w_a, c_a = ref_pr.trace_pagerank(*g_a, True)
    t2 = time.perf_counter()
    res["pr_normal"] = dump_pr(w_n, c_n)
    res["pr_anomaly"] = dump_pr(w_a, c_a)
    res["spectrum"] = run_spectrum_all(w_a, w_n, len(nor), len(abn), c_a, c_n)
    # both flavours on the un-swapped lists too
    for flag_, lst, key in ((True, abn, "pr_abn_true"), (False, nor, "pr_nor_false")):
        g = ref_pp.get_pagerank_graph(lst, adf)
        w, c = ref_pr.trace_pagerank(*g, flag_)
        res[key] = dump_pr(w, c)
    if driver:
        cwd = os.getcwd()
        with tempfile.TemporaryDirectory() as td:
            os.chdir(td)
            buf = io.StringIO()
            try:
                with contextlib.redirect_stdout(buf):
                    ref_rca.online_anomaly_detect_RCA(adf.copy(), slo, op_list)
                res["driver_stdout"] = buf.getvalue()
                res["driver_error"] = None
            except Exception as e:
                res["driver_stdout"] = buf.getvalue()
                res["driver_error"] = type(e).__name__
            res["result_csv"] = open("result.csv").read() if os.path.exists("result.csv") else None
            os.chdir(cwd)
    res["timing_s"] = {"detect+graphs": t1 - t0, "trace_pagerank_x2": t2 - t1}
    res["input_digest"] = {"normal": synth.frame_digest(ndf), "abnormal": synth.frame_digest(adf)}
    with open(os.path.join(outdir, f"{name}.json"), "w") as f:
        json.dump(res, f, indent=0)
    print(name, "traces", adf.traceID.nunique(), "spans", len(adf), "abn", len(abn), "nor", len(nor),
          "pr time %.2fs" % (t2 - t1))


def edge_span_df():
    """Hand-built spans hitting T5/T10/T11/T14: duplicate spanIDs across traces, orphans,
    self-loop, ts-ui-dashboard naming, zero-duration trace, op missing from the SLO."""
    T0 = pd.Timestamp("2024-01-01 00:00:00")
    rows = []

    def add(tr, sid, par, svc, op, pod, dur, t_off=0.0, t_len=2.0):
        rows.append(dict(traceID=tr, spanID=sid, ParentSpanId=par, serviceName=svc, operationName=op,
                         podName=pod, duration=dur, startTime=T0 + pd.Timedelta(seconds=t_off),
                         endTime=T0 + pd.Timedelta(seconds=t_off + t_len)))
    ui = "ts-ui-dashboard"
    for i in range(12):
        tr = f"tr{i:03d}"
        base = 1000 * (i + 1)
        add(tr, f"{tr}-r", None, ui, f"GET /api/orders/{100 + i}", "ui-pod-0", 40000 + base, i)
        add(tr, f"{tr}-a", f"{tr}-r", "svc-a", "query", "a-pod-0", 20000 + base, i)
        add(tr, f"{tr}-b", f"{tr}-a", "svc-b", "fetch", "b-pod-%d" % (i % 2), 9000 + base, i)
        if i % 3 == 0:  # self loop a->a and a repeated child
            add(tr, f"{tr}-a2", f"{tr}-a", "svc-a", "query", "a-pod-0", 5000, i)
            add(tr, f"{tr}-b2", f"{tr}-a", "svc-b", "fetch", "b-pod-0", 4000, i)
        if i % 4 == 1:  # orphan: parent id never seen
            add(tr, f"{tr}-o", "missing-parent", "svc-c", "orphan", "c-pod-0", 3000, i)
        if i % 5 == 2:  # op absent from the SLO training set
            add(tr, f"{tr}-n", f"{tr}-b", "svc-new", "novel", "n-pod-0", 2000000, i)
    # duplicated spanID across traces: tr001-a reuses tr000-a's id
    for r in rows:
        if r["traceID"] == "tr001" and r["spanID"] == "tr001-a":
            r["spanID"] = "tr000-a"
        if r["traceID"] == "tr001" and r["ParentSpanId"] == "tr001-a":
            r["ParentSpanId"] = "tr000-a"
    # zero-duration trace is dropped by the detector (preprocess_data.py:117)
    add("trzero", "z-r", None, ui, "GET /api/orders/1", "ui-pod-0", 0, 3)
    return pd.DataFrame(rows)


def slo_large(outdir):
    """get_operation_slo on ops straddling numpy's 8192-element reduction buffer."""
    df = synth.slo_frame()
    sdf = df.copy()
    ol = ref_pp.get_service_operation_list(sdf)
    slo = ref_pp.get_operation_slo(ol, sdf)
    out = {"seed": 7, "sizes": list(synth.SLO_SIZES), "digest": synth.frame_digest(df), "operation_list": ol,
           "slo": {k: [fhex(v[0]), fhex(v[1])] for k, v in slo.items()}}
    with open(os.path.join(outdir, "slo_large.json"), "w") as f:
        json.dump(out, f, indent=0)


def span_times_case(outdir):
    """Per-span startTime / endTime (synth span_times): traces at the window's end straddle it, so
    the detector sees some of their rows (get_span, preprocess_data.py:10-14) while the driver's
    graphs take all rows of the selected traces (online_rca.py:180,185 pass the whole frame)."""
    span_case("span_times", dict(n_ops=40, n_traces=1500, seed=400, span_times=True, minutes=5.2), outdir)


STREAM_CASES = {
    # 60 minutes of traffic, a rare fault: a mix of quiet, triggered and one-list-empty windows
    "stream": dict(n_ops=40, n_traces=6000, seed=500, minutes=60.0, fault_frac=0.006),
    # the same with a silent 15-minute gap after minute 30: the sweep ends in the empty-window
    # TypeError (T2) after the windows before it
    "stream_gap": dict(n_ops=40, n_traces=6000, seed=510, minutes=60.0, fault_frac=0.003, gap_after_min=30.0,
                       gap_min=15.0),
}


def stream_case(name, params, outdir):
    """The reference driver over a multi-window stream (online_rca.py:161-216): stdout, error and
    result.csv."""
    ndf, adf = synth.stream_dataframes(**params)
    span_df = ndf.copy()
    op_list = ref_pp.get_service_operation_list(span_df)
    slo = ref_pp.get_operation_slo(op_list, span_df)
    res = {"name": name, "params": params, "operation_list": op_list,
           "slo": {k: [fhex(v[0]), fhex(v[1])] for k, v in slo.items()}}
    cwd = os.getcwd()
    t0 = time.perf_counter()
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        buf = io.StringIO()
        try:
            with contextlib.redirect_stdout(buf):
                ref_rca.online_anomaly_detect_RCA(adf.copy(), slo, op_list)
            res["driver_error"] = None
        except Exception as e:
            res["driver_error"] = type(e).__name__
        res["driver_stdout"] = buf.getvalue()
        res["result_csv"] = open("result.csv").read() if os.path.exists("result.csv") else None
        os.chdir(cwd)
    res["timing_s"] = time.perf_counter() - t0
    res["input_digest"] = {"normal": synth.frame_digest(ndf), "abnormal": synth.frame_digest(adf)}
    with open(os.path.join(outdir, f"{name}.json"), "w") as f:
        json.dump(res, f, indent=0)
    print(name, "traces", adf.traceID.nunique(), "error", res["driver_error"], "windows ranked",
          res["driver_stdout"].count("anomaly_list"), "time %.1fs" % res["timing_s"])


C3_WINDOW = dict(n_ops=500, n_traces=20_000, seed=4242, branch=1.9, p_max=0.8, fault_ms=6000.0)


def c3_window_case(outdir):
    """One C3-sized window (BASELINE configs[2]: 500 ops / 20k traces) through the reference's
    per-window body (online_rca.py:167-201): detector, the two swapped graphs (T1), both
    trace_pagerank calls and the DStar2 spectrum.  Lean on purpose (no extra flavours, no driver
    re-run): the two trace_pagerank calls alone take minutes (O(T^2) kinds, pagerank.py:54-66).
    Only outputs are stored; the inputs are re-created by synth from the recorded params."""
    ndf, adf = make_windows(**C3_WINDOW)
    res = {"name": "c3_window", "params": C3_WINDOW}
    span_df = ndf.copy()
    op_list = ref_pp.get_service_operation_list(span_df)
    slo = ref_pp.get_operation_slo(op_list, span_df)
    res["operation_list"] = op_list
    res["slo"] = {k: [fhex(v[0]), fhex(v[1])] for k, v in slo.items()}
    start = adf["startTime"].min()
    end = start + pd.Timedelta(minutes=5)
    buf = io.StringIO()
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(buf):
        flag, abn, nor = ref_det.system_anomaly_detect(adf, start_time=start, end_time=end, slo=slo,
                                                       operation_list=op_list)
    tn = sorted(adf["traceID"].unique())
    ti = {n: i for i, n in enumerate(tn)}
    res["detect"] = {"flag": bool(flag), "abnormal": [ti[x] for x in abn], "normal": [ti[x] for x in nor],
                     "stdout": buf.getvalue(), "start_ns": int(start.value), "end_ns": int(end.value)}
    g_n = ref_pp.get_pagerank_graph(abn, adf)
    g_a = ref_pp.get_pagerank_graph(nor, adf)
    res["nodes_normal"] = list(g_n[0].keys())
    res["nodes_anomaly"] = list(g_a[0].keys())
    t1 = time.perf_counter()
    w_n, c_n = ref_pr.trace_pagerank(*g_n, False)
    w_a, c_a = ref_pr.trace_pagerank(*g_a, True)
    t2 = time.perf_counter()
    res["pr_normal"] = dump_pr(w_n, c_n)
    res["pr_anomaly"] = dump_pr(w_a, c_a)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        top, score = ref_rca.calculate_spectrum_without_delay_list(
            anomaly_result=w_a, normal_result=w_n, anomaly_list_len=len(nor), normal_list_len=len(abn), top_max=5,
            normal_num_list=c_n, anomaly_num_list=c_a, spectrum_method="dstar2")
    res["spectrum_dstar2"] = {"top": list(top), "score": [fhex(s) for s in score], "stdout": buf.getvalue()}
    res["timing_s"] = {"detect+graphs": t1 - t0, "trace_pagerank_x2": t2 - t1}
    res["input_digest"] = {"normal": synth.frame_digest(ndf), "abnormal": synth.frame_digest(adf)}
    with open(os.path.join(outdir, "c3_window.json"), "w") as f:
        json.dump(res, f, indent=0)
    print("c3_window traces", adf.traceID.nunique(), "spans", len(adf), "abn", len(abn), "nor", len(nor),
          "pr time %.1fs" % (t2 - t1))


def main():
    outdir = HERE
    if sys.argv[1:] == ["c3_window"]:
        c3_window_case(outdir)
        return
    if sys.argv[1:] == ["stream"]:
        for name, params in STREAM_CASES.items():
            stream_case(name, params, outdir)
        return
    if sys.argv[1:] == ["slo_large"]:
        slo_large(outdir)
        return
    if sys.argv[1:] == ["span_times"]:
        span_times_case(outdir)
        return
    man = {"numpy": np.__version__, "pandas": pd.__version__, "python": sys.version.split()[0]}
    try:
        cfg = np.show_config(mode="dicts")
        man["blas"] = cfg["Build Dependencies"]["blas"]
    except Exception:
        pass
    # dict cases
    dres = {}
    for name, (oo, ot, to, pt) in dict_edge_cases().items():
        entry = {"input": {"operation_operation": oo, "operation_trace": ot, "trace_operation": to,
                           "pr_trace": pt}}
        for anomaly in (False, True):
            try:
                w, c = ref_pr.trace_pagerank(oo, ot, to, pt, anomaly)
                entry[f"anomaly={anomaly}"] = dump_pr(w, c)
            except Exception as e:
                entry[f"anomaly={anomaly}"] = {"error": type(e).__name__}
        dres[name] = entry
    # raw pageRank on the paper matrices (illustrative)
    ap_ss = np.array([[0, 0, 0, 0], [1 / 3, 0, 0, 0], [1 / 3, 0, 0, 0], [1 / 3, 1, 1, 0]])
    ap_sr = np.array([[1 / 2, 1 / 3, 1 / 3], [0, 0, 1 / 3], [0, 1 / 3, 0], [1 / 2, 1 / 3, 1 / 3]])
    ap_rs = np.array([[1 / 3, 0, 0, 1 / 3], [1 / 3, 0, 1, 1 / 3], [1 / 3, 1, 0, 1 / 3]])
    a_v = np.array([[1], [1 / 3], [1 / 3]])
    dres["paper_pageRank"] = {"result": [fhex(x) for x in ref_pr.pageRank(ap_ss, ap_sr, ap_rs, a_v, 4, 3)[:, 0]]}
    # spectrum edge cases: zero denominators, ties, normal-only / anomaly-only nodes
    a_w = {"p": 0.5, "q": 0.5, "r": 0.0, "s": 1.0}
    n_w = {"q": 0.25, "s": 0.0, "t": 0.75}
    a_n = {"p": 3, "q": 3, "r": 0, "s": 4}
    n_n = {"q": 2, "s": 5, "t": 1}
    dres["spectrum_edges"] = {"input": {"a_w": a_w, "n_w": n_w, "a_n": a_n, "n_n": n_n, "A": 4, "N": 5},
                              "out": run_spectrum_all(a_w, n_w, 4, 5, a_n, n_n)}
    with open(os.path.join(outdir, "dict_cases.json"), "w") as f:
        json.dump(dres, f, indent=0)
    # span-level: hand-built edges
    edf = edge_span_df()
    e = {}
    sdf = edf.copy()
    ol = ref_pp.get_service_operation_list(sdf)
    slo = ref_pp.get_operation_slo(ol[:-1], sdf)  # drop one op from the SLO list
    e["operation_list"] = ol
    e["slo"] = {k: [fhex(v[0]), fhex(v[1])] for k, v in slo.items()}
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        flag, abn, nor = ref_det.system_anomaly_detect(edf, start_time=edf.startTime.min(),
                                                       end_time=edf.startTime.min() + pd.Timedelta(minutes=5),
                                                       slo=slo, operation_list=ol)
    e["detect"] = {"flag": bool(flag), "abnormal": abn, "normal": nor, "stdout": buf.getvalue()}
    all_tr = sorted(edf.traceID.unique())
    for key, lst in (("all", all_tr), ("subset", all_tr[::2] + ["not-a-trace"])):
        g = ref_pp.get_pagerank_graph(lst, edf)
        e[f"graph_{key}"] = dump_graph(g)
        for flag_ in (False, True):
            w, c = ref_pr.trace_pagerank(*g, flag_)
            e[f"pr_{key}_{flag_}"] = dump_pr(w, c)
    edf.to_parquet(os.path.join(outdir, "edges_spans.parquet"), index=False)
    with open(os.path.join(outdir, "edges.json"), "w") as f:
        json.dump(e, f, indent=0)
    # synthetic windows
    span_case("c1", dict(n_ops=40, n_traces=2000, seed=100), outdir)
    span_case("pods_dup_broken", dict(n_ops=30, n_traces=600, seed=200, pods=2, dup=0.01, broken=0.05), outdir)
    slo_large(outdir)
    span_case("ops200", dict(n_ops=200, n_traces=1500, seed=300, branch=1.9, p_max=0.8, fault_ms=6000.0), outdir, driver=False)
    span_times_case(outdir)
    for name, params in STREAM_CASES.items():
        stream_case(name, params, outdir)
    with open(os.path.join(outdir, "manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
