"""Pin the oracle (oracle/oracle.py) to the reference's own outputs (tests/golden/*.json).

The fixtures were produced by importing /root/reference in the dev container
(tests/golden/make_golden.py).  Tolerances: graph structure, counts, key orders and
top lists exact; trace_pagerank weights 1e-12 relative (the reference's dense
OpenBLAS dgemv sums in an order no sparse code reproduces bit for bit); spectrum,
SLO and detector bit-exact (same IEEE operation sequence).
"""
import math

import numpy as np
import pandas as pd
import pytest

import oracle as orc
from conftest import load_golden, regen_window, unhex
from microrank_amd.spans import SpanTable

SPAN_CASES = ["c1", "pods_dup_broken", "ops200", "span_times"]


def check_pr(got, exp, rtol=1e-12):
    w, num = got
    assert list(w.keys()) == exp["keys"]
    assert list(num.keys()) == exp["num_keys"]
    assert [int(v) for v in num.values()] == exp["num"]
    gw = np.array([float(v) for v in w.values()])
    ew = unhex(exp["weight"])
    np.testing.assert_allclose(gw, ew, rtol=rtol, atol=0)


@pytest.mark.parametrize("case", ["fig3", "multiset_selfloop", "pr_subset", "single", "asym_incidence"])
@pytest.mark.parametrize("anomaly", [False, True])
def test_dict_cases(case, anomaly):
    d = load_golden("dict_cases.json")[case]
    inp = d["input"]
    exp = d[f"anomaly={anomaly}"]
    args = (inp["operation_operation"], inp["operation_trace"], inp["trace_operation"], inp["pr_trace"])
    if "error" in exp:
        with pytest.raises(getattr(__builtins__, exp["error"], Exception) if isinstance(__builtins__, dict)
                           else Exception):
            orc.trace_pagerank(*args, anomaly)
        return
    check_pr(orc.trace_pagerank(*args, anomaly), exp)


def test_paper_example_survey_values():
    # anomaly weights of the Fig. 3 dicts through the reference
    d = load_golden("dict_cases.json")["fig3"]
    w = unhex(d["anomaly=True"]["weight"])
    np.testing.assert_allclose(w, [0.65681832483573, 0.21988528611506, 0.21988528611506, 0.66330495471105],
                               rtol=1e-12)


def _spans(df):
    return SpanTable.from_dataframe(df)


@pytest.mark.parametrize("name", SPAN_CASES)
def test_span_graph_matches_reference(name):
    case = load_golden(f"{name}.json")
    _, adf = regen_window(case)
    st = _spans(adf)
    tnames = list(st.trace_names)
    ti = {n: i for i, n in enumerate(tnames)}
    for key, lst in (("graph_swapped_normal", case["detect"]["abnormal"]),
                     ("graph_swapped_anomaly", case["detect"]["normal"])):
        exp = case[key]
        sel = np.zeros(len(tnames), dtype=bool)
        sel[lst] = True
        sg = orc.span_graph(st.trace, st.podop, st.span, st.parent, sel)
        nodes = [st.podop_names[c] for c in sg.node_podop]
        assert nodes == exp["nodes"]
        # children multisets
        oo = exp["operation_operation"]
        N = len(nodes)
        exp_nchild = np.zeros(N, dtype=np.int64)
        exp_pairs = set()
        pos = 0
        for k, ln in zip(oo["keys"], oo["len"]):
            exp_nchild[k] = ln
            for c in oo["vals"][pos:pos + ln]:
                exp_pairs.add((c, k))
            pos += ln
        assert oo["keys"] == list(range(N))
        np.testing.assert_array_equal(sg.nchild, exp_nchild)
        assert set(zip(sg.ss_c.tolist(), sg.ss_p.tolist())) == exp_pairs
        # operation_trace: sorted trace keys, list lengths, distinct op sets
        ot = exp["operation_trace"]
        assert list(sg.trace_codes) == ot["keys"]
        np.testing.assert_array_equal(sg.len_t, ot["len"])
        exp_sr = set()
        pos = 0
        for t_i, (k, ln) in enumerate(zip(ot["keys"], ot["len"])):
            for o in ot["vals"][pos:pos + ln]:
                exp_sr.add((t_i, o))
            pos += ln
        assert set(zip(sg.sr_t.tolist(), sg.sr_o.tolist())) == exp_sr
        to = exp["trace_operation"]
        len_o = dict(zip(to["keys"], to["len"]))
        assert [len_o[i] for i in range(N)] == sg.len_o.tolist()
        assert exp["pr_trace_is_operation_trace"]


@pytest.mark.parametrize("name", SPAN_CASES)
def test_span_pagerank_matches_reference(name):
    case = load_golden(f"{name}.json")
    _, adf = regen_window(case)
    st = _spans(adf)
    for lst_key, anomaly, exp_key in (("abnormal", False, "pr_normal"), ("normal", True, "pr_anomaly"),
                                      ("abnormal", True, "pr_abn_true"), ("normal", False, "pr_nor_false")):
        sel = np.zeros(st.n_traces, dtype=bool)
        sel[case["detect"][lst_key]] = True
        sg = orc.span_graph(st.trace, st.podop, st.span, st.parent, sel)
        g = sg.as_graph()
        g.nodes = [st.podop_names[c] for c in sg.node_podop]
        kind = orc.trace_kinds(g)
        v = orc.preference(g, kind, anomaly)
        s = orc.power_iteration(g, v)
        check_pr(orc.weights(g, s), case[exp_key])


@pytest.mark.parametrize("name", SPAN_CASES)
def test_spectrum_matches_reference(name):
    case = load_golden(f"{name}.json")
    a = case["pr_anomaly"]
    n = case["pr_normal"]
    a_w = dict(zip(a["keys"], unhex(a["weight"])))
    n_w = dict(zip(n["keys"], unhex(n["weight"])))
    a_n = dict(zip(a["num_keys"], a["num"]))
    n_n = dict(zip(n["num_keys"], n["num"]))
    A = len(case["detect"]["normal"])     # T1: the driver's anomaly list is the detector's normal list
    Nn = len(case["detect"]["abnormal"])
    for m, exp in case["spectrum"].items():
        top, score, lines = orc.spectrum(a_w, n_w, A, Nn, 5, n_n, a_n, m)
        assert top == exp["top"]
        assert [float(x).hex() for x in score] == exp["score"]
        assert "".join(l + "\n" for l in lines) == exp["stdout"]


def test_spectrum_edge_cases():
    d = load_golden("dict_cases.json")["spectrum_edges"]
    i = d["input"]
    for m, exp in d["out"].items():
        if "error" in exp:
            with pytest.raises(ZeroDivisionError):
                orc.spectrum(i["a_w"], i["n_w"], i["A"], i["N"], 5, i["n_n"], i["a_n"], m)
            continue
        top, score, lines = orc.spectrum(i["a_w"], i["n_w"], i["A"], i["N"], 5, i["n_n"], i["a_n"], m)
        assert top == exp["top"]
        assert [float(x).hex() for x in score] == exp["score"]


@pytest.mark.parametrize("name", SPAN_CASES)
def test_slo_and_detector_match_reference(name):
    case = load_golden(f"{name}.json")
    ndf, adf = regen_window(case)
    nst = _spans(ndf)
    slo = orc.operation_slo(nst.svcop, nst.duration, nst.svcop_names, case["operation_list"])
    assert list(slo.keys()) == list(case["slo"].keys())
    for k, v in slo.items():
        assert [float(v[0]).hex(), float(v[1]).hex()] == case["slo"][k]
    ast = _spans(adf)
    a3 = {}
    for code, name_ in enumerate(ast.svcop_names):
        if name_ in slo:
            a3[code] = slo[name_][0] + 3 * slo[name_][1]
    flag, ab, no = orc.detect(ast.trace, ast.svcop, ast.duration, ast.tstart, ast.tend,
                              case["detect"]["start_ns"], case["detect"]["end_ns"], a3)
    assert ab == case["detect"]["abnormal"]
    assert no == case["detect"]["normal"]
    assert flag == case["detect"]["flag"]


def test_edge_spans():
    e = load_golden("edges.json")
    df = pd.read_parquet(f"{__import__('conftest').GOLDEN}/edges_spans.parquet")
    st = _spans(df)
    slo_list = e["operation_list"][:-1]
    slo = orc.operation_slo(st.svcop, st.duration, st.svcop_names, slo_list)
    assert {k: [float(v[0]).hex(), float(v[1]).hex()] for k, v in slo.items()} == e["slo"]
    a3 = {c: slo[n][0] + 3 * slo[n][1] for c, n in enumerate(st.svcop_names) if n in slo}
    t0 = int(df.startTime.min().value)
    flag, ab, no = orc.detect(st.trace, st.svcop, st.duration, st.tstart, st.tend, t0,
                              t0 + 5 * 60 * 10**9, a3)
    assert [st.trace_names[t] for t in ab] == e["detect"]["abnormal"]
    assert [st.trace_names[t] for t in no] == e["detect"]["normal"]
    all_tr = sorted(df.traceID.unique())
    for key, lst in (("all", all_tr), ("subset", all_tr[::2] + ["not-a-trace"])):
        sel = np.isin(np.array(st.trace_names, dtype=object), lst)
        sg = orc.span_graph(st.trace, st.podop, st.span, st.parent, sel)
        exp = e[f"graph_{key}"]
        nodes = [st.podop_names[c] for c in sg.node_podop]
        assert nodes == list(exp["operation_operation"].keys())
        for p, ch in exp["operation_operation"].items():
            pi = nodes.index(p)
            assert sg.nchild[pi] == len(ch)
            assert {(nodes.index(c), pi) for c in ch} == {(c, p_) for c, p_ in zip(sg.ss_c, sg.ss_p) if p_ == pi}
        for flag_ in (False, True):
            g = sg.as_graph()
            g.nodes = nodes
            w = orc.weights(g, orc.power_iteration(g, orc.preference(g, orc.trace_kinds(g), flag_)))
            check_pr(w, e[f"pr_{key}_{flag_}"])


def test_slo_large_ops_numpy_buffering():
    """Ops larger than numpy's 8192-element reduction buffer: np.std sums the buffers
    sequentially (oracle.numpy_reduce_sum); plain pairwise summation over the whole op differs
    in the last bits for some of them."""
    from microrank_amd import synth

    case = load_golden("slo_large.json")
    df = synth.slo_frame(case["seed"], tuple(case["sizes"]))
    assert synth.frame_digest(df) == case["digest"]
    st = _spans(df)
    slo = orc.operation_slo(st.svcop, st.duration, st.svcop_names, case["operation_list"])
    assert {k: [float(v[0]).hex(), float(v[1]).hex()] for k, v in slo.items()} == case["slo"]
    assert list(slo) == sorted(case["slo"])


@pytest.mark.parametrize("name", ["stream", "stream_gap"])
def test_driver_sweep_matches_reference(name):
    """The oracle's window chain (online_rca.py:161-216) reproduces every detector line of the
    reference driver over a multi-window stream, and where it ends (T2)."""
    from microrank_amd import synth

    case = load_golden(f"{name}.json")
    ndf, adf = synth.stream_dataframes(**case["params"])
    assert synth.frame_digest(ndf) == case["input_digest"]["normal"], "generator drifted (normal)"
    assert synth.frame_digest(adf) == case["input_digest"]["abnormal"], "generator drifted (abnormal)"
    ast = _spans(adf)
    slo = {k: (float.fromhex(a), float.fromhex(b)) for k, (a, b) in case["slo"].items()}
    a3 = {c: slo[n][0] + 3 * slo[n][1] for c, n in enumerate(ast.svcop_names) if n in slo}
    events, empty = orc.driver_sweep(ast.trace, ast.svcop, ast.duration, ast.tstart, ast.tend, a3)
    lines = []
    for _t, flag, ab, no, _ranked in events:
        lines += [f"anormaly_trace {len(ab)}", f"total_trace {len(ab) + len(no)}"]
        if flag:
            lines += [f"anomaly_list {len(no)}", f"normal_list {len(ab)}"]
    if empty:
        lines.append("Error: Current span list is empty")
    exp = [ln.rstrip() for ln in case["driver_stdout"].splitlines()
           if ln.startswith(("anormaly_trace", "total_trace", "anomaly_list", "normal_list", "Error"))]
    assert lines == exp
    assert empty == (case["driver_error"] == "TypeError")


def test_read_traces_csv_equals_pandas(tmp_path):
    """f2: the OTel export (collect_data.py:35-46) read through pyarrow (Arrow-backed strings) holds
    what pandas' read_csv + rename + to_datetime (online_rca.py:221-248) holds, and factorises
    to the same codes."""
    import pandas as pd

    from microrank_amd import synth
    from microrank_amd.spans import OTEL_RENAME, SpanTable, read_traces_csv

    case = load_golden("pods_dup_broken.json")
    _, adf = regen_window(case)
    inv = {v: k for k, v in OTEL_RENAME.items()}
    p = tmp_path / "traces.csv"
    adf.rename(columns=inv).to_csv(p, index=False)
    ref = pd.read_csv(p).rename(columns=OTEL_RENAME)
    ref["startTime"] = pd.to_datetime(ref["startTime"])
    ref["endTime"] = pd.to_datetime(ref["endTime"])
    got = read_traces_csv(p)
    assert list(got.columns) == list(ref.columns)
    for c in ref.columns:
        a, b = got[c].to_numpy(dtype=object), ref[c].to_numpy(dtype=object)
        same = [(pd.isna(x) and pd.isna(y)) if (pd.isna(x) or pd.isna(y)) else x == y for x, y in zip(a, b)]
        assert all(same), c
    h1, h2 = SpanTable.from_dataframe(ref), SpanTable.from_dataframe(got)
    for c in ("trace", "podop", "svcop", "span", "parent", "duration", "tstart", "tend"):
        assert np.array_equal(getattr(h1, c), getattr(h2, c)), c
    assert synth.frame_digest(adf) == case["input_digest"]["abnormal"]
