"""GPU parity of K1 (get_pagerank_graph on the device) against the oracle and the reference
fixtures: node order, trace order, incidence, span counts and call edges bit-exact."""
import ctypes as C

import numpy as np
import pytest

import oracle as orc
from conftest import load_golden, regen_window, unhex

pytestmark = pytest.mark.gpu


def _export(pg):
    from microrank_amd import _lib
    from microrank_amd._lib import ptr

    info = pg.device_graph().info()
    N, T, nnz, E = info["N"], info["T"], info["nnz"], info["E"]
    sr_off = np.empty(T + 1, np.int64)
    sr_ops = np.empty(nnz, np.int32)
    len_t = np.empty(T, np.int32)
    len_o = np.empty(N, np.int32)
    ss_off = np.empty(N + 1, np.int64)
    ss_par = np.empty(E, np.int32)
    nchild = np.empty(N, np.int32)
    dg = pg.device_graph()
    dg.ctx.check(_lib.load().mr_graph_export(dg.h, ptr(sr_off, C.c_int64), ptr(sr_ops, C.c_int32),
                                             ptr(len_t, C.c_int32), ptr(len_o, C.c_int32), ptr(ss_off, C.c_int64),
                                             ptr(ss_par, C.c_int32), ptr(nchild, C.c_int32)))
    return dict(sr_off=sr_off, sr_ops=sr_ops, len_t=len_t, len_o=len_o, ss_off=ss_off, ss_par=ss_par, nchild=nchild)


def _check_against_oracle(table, dev, sel):
    from microrank_amd import _lib
    from microrank_amd.preprocess_data import PagerankGraph

    ctx = _lib.default_context()
    pg = PagerankGraph(ctx, table, dev, sel.astype(np.uint8))
    sg = orc.span_graph(table.trace, table.podop, table.span, table.parent, sel)
    np.testing.assert_array_equal(pg.node_podop, sg.node_podop)
    np.testing.assert_array_equal(pg.trace_code, sg.trace_codes)
    ex = _export(pg)
    np.testing.assert_array_equal(ex["len_t"], sg.len_t)
    np.testing.assert_array_equal(ex["len_o"], sg.len_o)
    np.testing.assert_array_equal(ex["nchild"], sg.nchild)
    t_of = np.repeat(np.arange(sg.trace_codes.size), np.diff(ex["sr_off"]))
    np.testing.assert_array_equal(t_of, sg.sr_t)
    np.testing.assert_array_equal(ex["sr_ops"], sg.sr_o)
    c_of = np.repeat(np.arange(sg.node_podop.size), np.diff(ex["ss_off"]))
    np.testing.assert_array_equal(c_of, sg.ss_c)
    np.testing.assert_array_equal(ex["ss_par"], sg.ss_p)
    return pg, sg


@pytest.mark.parametrize("name", ["c1", "pods_dup_broken", "ops200", "span_times"])
def test_graph_build_matches_reference(name):
    from microrank_amd import _lib
    from microrank_amd.pagerank import trace_pagerank
    from microrank_amd.preprocess_data import get_pagerank_graph, span_table

    case = load_golden(f"{name}.json")
    _, adf = regen_window(case)
    table, dev = span_table(adf, _lib.default_context())
    for lst_key, gkey, anomaly, pkey in (("abnormal", "graph_swapped_normal", False, "pr_normal"),
                                         ("normal", "graph_swapped_anomaly", True, "pr_anomaly")):
        sel = np.zeros(table.n_traces, bool)
        sel[case["detect"][lst_key]] = True
        _check_against_oracle(table, dev, sel)
        tnames = sorted(adf["traceID"].unique())
        g = get_pagerank_graph([tnames[i] for i in case["detect"][lst_key]], adf)
        assert list(g[0].keys()) == case[gkey]["nodes"]
        w, num = trace_pagerank(*g, anomaly)
        exp = case[pkey]
        assert list(w) == exp["keys"] and list(num.values()) == exp["num"]
        np.testing.assert_allclose(list(w.values()), unhex(exp["weight"]), rtol=1e-10)


def test_graph_views_materialise_like_reference():
    """The lazy dicts, when read, hold the reference's lists (row order, merge order)."""
    from microrank_amd.preprocess_data import get_pagerank_graph

    case = load_golden("pods_dup_broken.json")
    _, adf = regen_window(case)
    tnames = sorted(adf["traceID"].unique())
    g = get_pagerank_graph([tnames[i] for i in case["detect"]["abnormal"]], adf)
    exp = case["graph_swapped_normal"]
    nodes = exp["nodes"]
    d = exp["operation_operation"]
    pos = 0
    for k, ln in zip(d["keys"], d["len"]):
        assert g[0][nodes[k]] == [nodes[v] for v in d["vals"][pos:pos + ln]]
        pos += ln
    d = exp["operation_trace"]
    pos = 0
    for k, ln in zip(d["keys"], d["len"]):
        assert g[1][tnames[k]] == [nodes[v] for v in d["vals"][pos:pos + ln]]
        pos += ln
    assert list(g[2].keys()) == [nodes[k] for k in exp["trace_operation"]["keys"]]


def test_edge_spans_graph():
    import pandas as pd

    from conftest import GOLDEN
    from microrank_amd.pagerank import trace_pagerank
    from microrank_amd.preprocess_data import get_pagerank_graph

    e = load_golden("edges.json")
    df = pd.read_parquet(f"{GOLDEN}/edges_spans.parquet")
    all_tr = sorted(df.traceID.unique())
    for key, lst in (("all", all_tr), ("subset", all_tr[::2] + ["not-a-trace"])):
        g = get_pagerank_graph(lst, df)
        exp = e[f"graph_{key}"]
        assert list(g[0].keys()) == list(exp["operation_operation"].keys())
        for p, ch in exp["operation_operation"].items():
            assert g[0][p] == ch
        for flag_ in (False, True):
            w, num = trace_pagerank(*g, flag_)
            ex = e[f"pr_{key}_{flag_}"]
            assert list(w) == ex["keys"] and list(num.values()) == ex["num"]
            np.testing.assert_allclose(list(w.values()), unhex(ex["weight"]), rtol=1e-10)


def test_empty_selection_raises_like_reference():
    from microrank_amd.pagerank import trace_pagerank
    from microrank_amd.preprocess_data import get_pagerank_graph

    case = load_golden("c1.json")
    _, adf = regen_window(case)
    g = get_pagerank_graph([], adf)
    assert len(g[0]) == 0 and len(g[1]) == 0
    with pytest.raises(ValueError):
        trace_pagerank(*g, False)


@pytest.mark.parametrize("dup,broken,pods", [(0.0, 0.0, 1), (0.02, 0.05, 3)])
def test_c2_scale_graph_build(dup, broken, pods):
    """1k ops / 200k traces (C2), with and without duplicated spanIDs / broken traces."""
    from microrank_amd import _lib, synth
    from microrank_amd.preprocess_data import DeviceSpans

    topo = synth.make_topology(1000, 11, pods_per_service=pods)
    st = synth.gen_spans(topo, 200_000, 12, branch=1.9, p_max=0.8, dup_span_frac=dup, broken_frac=broken, names=False)
    st.trace_names = [str(i) for i in range(st.meta["n_gen_traces"])]
    dev = DeviceSpans(_lib.default_context(), st)
    rng = np.random.default_rng(5)
    sel = rng.random(st.n_traces) < 0.6
    _check_against_oracle(st, dev, sel)


def test_graph_sees_in_place_column_edits():
    """The reference's get_operation_duration_data rewrites operationName on the frame it gets
    (preprocess_data.py:100); a later get_pagerank_graph on that frame names its nodes from the
    rewritten column.  The device span table must be rebuilt, not served from the cache."""
    from microrank_amd.preprocess_data import get_operation_duration_data, get_pagerank_graph

    case = load_golden("c1.json")
    _, adf = regen_window(case)
    df = adf.copy()
    tnames = sorted(df["traceID"].unique())
    lst = [tnames[i] for i in case["detect"]["normal"]]
    before = list(get_pagerank_graph(lst, df)[0].keys())
    assert before == case["graph_swapped_anomaly"]["nodes"]
    get_operation_duration_data(case["operation_list"], df)   # mutates df["operationName"]
    after = list(get_pagerank_graph(lst, df)[0].keys())
    assert after != before
    # the oracle on the rewritten frame (ts-ui-dashboard names lose one more '/segment', so some
    # nodes merge -- as in the reference, whose get_pagerank_graph re-applies the rsplit rule)
    from microrank_amd.spans import SpanTable

    st = SpanTable.from_dataframe(df)
    sel = np.isin(np.array(st.trace_names, dtype=object), lst)
    sg = orc.span_graph(st.trace, st.podop, st.span, st.parent, sel)
    assert after == [st.podop_names[c] for c in sg.node_podop]
    from microrank_amd.preprocess_data import _fingerprint

    fp = _fingerprint(df)
    df.loc[df.index[0], "duration"] += 1   # any used column, in place
    assert not fp.matches(df)


def test_in_place_cell_edit_anywhere_reranks():
    """one in-place cell edit at an interior row (no sample would see it) --
    a span's operationName and another span's duration -- must reach the next drop-in call: the
    ranking equals the one computed on a fresh copy of the edited frame (a cache miss by
    construction), not the stale device table's."""
    from microrank_amd.pagerank import trace_pagerank
    from microrank_amd.preprocess_data import get_pagerank_graph

    case = load_golden("c1.json")
    _, adf = regen_window(case)
    df = adf.copy()
    tnames = sorted(df["traceID"].unique())
    lst = [tnames[i] for i in case["detect"]["normal"]]
    w0, c0 = trace_pagerank(*get_pagerank_graph(lst, df), False)
    rows = np.flatnonzero(df["traceID"].isin(lst).to_numpy())
    r = df.index[rows[len(rows) // 2 + 3]]   # an interior span of a listed trace
    df.loc[r, "operationName"] = "edited_operation"
    w1, c1 = trace_pagerank(*get_pagerank_graph(lst, df), False)
    fresh = df.copy()
    w2, c2 = trace_pagerank(*get_pagerank_graph(lst, fresh), False)
    assert list(w1) == list(w2) and c1 == c2
    assert [float(x) for x in w1.values()] == [float(x) for x in w2.values()]
    assert list(w1) != list(w0)   # the edited span's node appears
    assert any(k.endswith("_edited_operation") for k in w1)


def test_two_contexts_share_one_dataframe():
    """One Context per thread (the bench's streams): each context gets its own device span table
    for the same DataFrame (mr_spans handles belong to the context that uploaded them)."""
    from microrank_amd import _lib
    from microrank_amd.pagerank import trace_pagerank
    from microrank_amd.preprocess_data import get_pagerank_graph, span_table

    case = load_golden("c1.json")
    _, adf = regen_window(case)
    tnames = sorted(adf["traceID"].unique())
    lst = [tnames[i] for i in case["detect"]["abnormal"]]
    c1, c2 = _lib.Context(0), _lib.Context(0)
    t1, d1 = span_table(adf, c1)
    t2, d2 = span_table(adf, c2)
    assert d1 is not d2 and d1.ctx is c1 and d2.ctx is c2
    w1, _ = trace_pagerank(*get_pagerank_graph(lst, adf, ctx=c1), False, ctx=c1)
    w2, _ = trace_pagerank(*get_pagerank_graph(lst, adf, ctx=c2), False, ctx=c2)
    assert list(w1) == list(w2) and [float(x) for x in w1.values()] == [float(x) for x in w2.values()]
    np.testing.assert_allclose(list(w1.values()), unhex(case["pr_normal"]["weight"]), rtol=1e-10)


def test_edge_count_in_edge_id_order_equals_per_entry_count(monkeypatch):
    """Large tables keep their edge entries in edge-id order too (mr_spans.eb_*) and a build counts
    edges by a segmented sum per id (k_ix_ecount) instead of an atomic / hash probe per entry:
    forced on a small table (MR_IX_EB=force) the dense build (mr_graph_build) and the sharded one
    (mr_graph_build_sharded, one rank: the per-id counts inserted into its hash set) give the same
    graphs and bitwise the same weights as the per-entry count (MR_IX_EB=0), with a trace_list
    that is not every trace and broken / duplicated traces."""
    from microrank_amd import _lib, shard, synth
    from microrank_amd._lib import ptr
    from microrank_amd.graph import DeviceGraph
    from microrank_amd.preprocess_data import DeviceSpans

    st = synth.big_spans(3000, 20_000, seed=5, dup_frac=0.01, broken_frac=0.05)
    sel = np.ones(st.n_traces, np.uint8)
    sel[::5] = 0
    ctx = _lib.default_context()
    lib = _lib.load()
    out = {}
    for mode in ("0", "force"):
        monkeypatch.setenv("MR_IX_EB", mode)
        dev = DeviceSpans(ctx, st)
        h = _lib.P()
        ctx.check(lib.mr_graph_build(ctx.h, dev.h, ptr(sel, C.c_uint8), C.byref(h)), "mr_graph_build")
        n, t, nnz, e = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int64()
        lib.mr_graph_info(h, C.byref(n), C.byref(t), C.byref(nnz), C.byref(e))
        node = np.empty(n.value, np.int32)
        tcode = np.empty(t.value, np.int32)
        ctx.check(lib.mr_graph_nodes(h, ptr(node, C.c_int32), ptr(tcode, C.c_int32)), "mr_graph_nodes")
        dg = DeviceGraph(ctx, h, node, tcode, n.value, t.value)
        dg.pagerank(True)
        w, cov = dg.fetch()
        sg = shard.build_graph(dev, sel)
        ws, covs = shard.sharded_pagerank(sg, True)
        out[mode] = ((n.value, t.value, nnz.value, e.value), node.copy(), tcode.copy(), w.copy(), cov.copy(),
                     sg.info(), np.asarray(ws).copy(), np.asarray(covs).copy())
        assert e.value > 0
        dg.close()
        sg.close()
        dev.close()
    a, b = out["0"], out["force"]
    assert a[0] == b[0] and a[5] == b[5]
    for x, y in zip(a[1:5] + a[6:], b[1:5] + b[6:]):
        assert x.tobytes() == y.tobytes()
