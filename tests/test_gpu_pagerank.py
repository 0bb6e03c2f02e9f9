"""GPU parity of K2 (trace_pagerank) against the reference fixtures and the oracle.

Tolerances (BASELINE.json north star): fp64 scores within 1e-6 relative (we assert 1e-10:
the only difference from the reference is the summation order of its dense dgemv),
fp32 within 1e-4; coverage counts, key order and kinds exact.
"""
import numpy as np
import pytest

import oracle as orc
from conftest import load_golden, unhex
from gpu_util import c2_graph, golden_graph_dicts, host_graph_from_oracle

pytestmark = pytest.mark.gpu

RTOL64 = 1e-10
RTOL32 = 1e-4


def _check(got, exp, rtol):
    w, num = got
    assert list(w.keys()) == exp["keys"]
    assert list(num.keys()) == exp["num_keys"]
    assert [int(v) for v in num.values()] == exp["num"]
    assert all(isinstance(v, np.float64) for v in w.values())
    np.testing.assert_allclose(np.array(list(w.values())), unhex(exp["weight"]), rtol=rtol, atol=0)


@pytest.mark.parametrize("case", ["fig3", "multiset_selfloop", "pr_subset", "single", "asym_incidence"])
@pytest.mark.parametrize("anomaly", [False, True])
@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_dict_cases(case, anomaly, precision):
    from microrank_amd.pagerank import trace_pagerank

    d = load_golden("dict_cases.json")[case]
    inp = d["input"]
    got = trace_pagerank(inp["operation_operation"], inp["operation_trace"], inp["trace_operation"],
                         inp["pr_trace"], anomaly, precision=precision)
    _check(got, d[f"anomaly={anomaly}"], RTOL64 if precision == "fp64" else RTOL32)


def test_unknown_key_raises_value_error():
    from microrank_amd.pagerank import trace_pagerank

    with pytest.raises(ValueError):
        trace_pagerank({"a": ["zz"]}, {"t": ["a"]}, {"a": ["t"]}, {"t": ["a"]}, False)
    with pytest.raises(ValueError):
        trace_pagerank({}, {}, {}, {}, False)
    with pytest.raises(ZeroDivisionError):
        trace_pagerank({"a": []}, {"t": ["a"], "u": ["a"]}, {"a": ["t", "u"]}, {"t": ["a"], "u": []}, True)


@pytest.mark.parametrize("name", ["c1", "pods_dup_broken", "ops200", "span_times"])
def test_span_case_graphs(name):
    """The reference's own graph dicts for each window -> trace_pagerank on the GPU."""
    from microrank_amd.pagerank import trace_pagerank

    case = load_golden(f"{name}.json")
    from conftest import regen_window

    _, adf = regen_window(case)
    tnames = sorted(adf["traceID"].unique())
    for gkey, anomaly, pkey in (("graph_swapped_normal", False, "pr_normal"),
                                ("graph_swapped_anomaly", True, "pr_anomaly")):
        dicts = golden_graph_dicts(case[gkey], tnames)
        _check(trace_pagerank(*dicts, anomaly), case[pkey], RTOL64)
        _check(trace_pagerank(*dicts, anomaly, precision="fp32"), case[pkey], RTOL32)


@pytest.fixture(scope="module")
def c2():
    return c2_graph()


@pytest.mark.parametrize("anomaly", [False, True])
def test_c2_scale_against_oracle(c2, anomaly):
    """1k ops / 200k traces: GPU vs oracle; kinds exact, weights 1e-10 (fp64) / 1e-4 (fp32),
    and bitwise-identical reruns (fixed-order reductions)."""
    from microrank_amd import _lib
    from microrank_amd.graph import DeviceGraph

    st, sg = c2
    g = sg.as_graph()
    kind = orc.trace_kinds(g) if g.T <= 300_000 else None
    v = orc.preference(g, kind, anomaly)
    s = orc.power_iteration(g, v)
    w_ref, cov_ref = orc.weights(g, s)
    ctx = _lib.default_context()
    dg = DeviceGraph.upload(ctx, host_graph_from_oracle(g))
    dg.pagerank(anomaly)
    w, cov, k, pref = dg.fetch(kinds=True)
    np.testing.assert_array_equal(k, kind)
    np.testing.assert_allclose(pref, v, rtol=1.2e-7, atol=0)   # tree vs sequential sum: <=1 fp32 ulp
    np.testing.assert_array_equal(cov, np.array(list(cov_ref.values())))
    np.testing.assert_allclose(w, np.array(list(w_ref.values())), rtol=RTOL64, atol=0)
    dg.pagerank(anomaly)
    w2, _ = dg.fetch()
    assert w2.tobytes() == w.tobytes(), "rerun not bitwise identical"
    dg.pagerank(anomaly, precision="fp32")
    w3, _ = dg.fetch()
    np.testing.assert_allclose(w3, np.array(list(w_ref.values())), rtol=RTOL32, atol=0)
    dg.close()


@pytest.mark.parametrize("part_min", ["0", "1000000000"])
def test_kinds_partition_and_table_paths(c2, part_min, monkeypatch):
    """Both kinds paths (the per-partition LDS tables of large graphs, forced here with
    MR_KIND_PART_MIN=0, and the global hash table) give the oracle's kinds exactly on the C2
    graph (hot kinds: thousands of traces on one call path), and the same weights bitwise."""
    from microrank_amd import _lib
    from microrank_amd.graph import DeviceGraph

    monkeypatch.setenv("MR_KIND_PART_MIN", part_min)
    st, sg = c2
    g = sg.as_graph()
    kind = orc.trace_kinds(g)
    ctx = _lib.default_context()
    dg = DeviceGraph.upload(ctx, host_graph_from_oracle(g))
    dg.pagerank(True)
    w, cov, k, pref = dg.fetch(kinds=True)
    np.testing.assert_array_equal(k, kind)
    monkeypatch.setenv("MR_KIND_PART_MIN", "1000000000" if part_min == "0" else "0")
    dg.pagerank(True)
    w2, _ = dg.fetch()
    assert w2.tobytes() == w.tobytes()
    # the partition path's two ways of grouping records by partition (two passes of its bits with
    # the classes written back to each record's slot, the default; a device cursor per partition,
    # MR_KIND_GROUP=cursor): the same classes and representatives
    monkeypatch.setenv("MR_KIND_PART_MIN", "0")
    for grouping in ("two", "cursor"):
        monkeypatch.setenv("MR_KIND_GROUP", grouping)
        dg.pagerank(True)
        w3, _, k3, _ = dg.fetch(kinds=True)
        np.testing.assert_array_equal(k3, kind)
        assert w3.tobytes() == w.tobytes()
    dg.close()


@pytest.mark.parametrize("anomaly", [False, True])
def test_trace_order_preference_equals_position_order(c2, anomaly, monkeypatch):
    """The trace-order preference form (k_pref_apply_t: large graphs, c_tp scattered through the
    inverse of tperm) against the position-order form on the C2 graph: the same pref vector and
    the same weights, bitwise; and the oracle's preference within 1 fp32 ulp."""
    from microrank_amd import _lib
    from microrank_amd.graph import DeviceGraph

    st, sg = c2
    g = sg.as_graph()
    v = orc.preference(g, orc.trace_kinds(g), anomaly)
    ctx = _lib.default_context()
    dg = DeviceGraph.upload(ctx, host_graph_from_oracle(g))
    monkeypatch.setenv("MR_PREF_T_MIN", "1000000000")   # position order
    dg.pagerank(anomaly)
    w0, _c0, _k0, p0 = dg.fetch(kinds=True)
    monkeypatch.setenv("MR_PREF_T_MIN", "0")            # trace order
    dg.pagerank(anomaly)
    w1, _c1, _k1, p1 = dg.fetch(kinds=True)
    assert p1.tobytes() == p0.tobytes()
    assert w1.tobytes() == w0.tobytes()
    np.testing.assert_allclose(p1, v, rtol=1.2e-7, atol=0)
    dg.close()


@pytest.mark.parametrize("n_ops", [9000, 12000])
def test_call_graph_terms_in_walk_kernel_bitwise(n_ops, monkeypatch):
    """The call-graph terms computed by k_tr_a's waves that finished their walk (MR_TR_SSV=1, large
    graphs) instead of k_fx_b: bitwise the same weights; N = 12000 is relabelled (su of the hot
    ops in LDS), so the terms are in column order there.  Write-through rows (MR_TR_ROW_WT) too."""
    from microrank_amd import _lib, synth
    from microrank_amd.graph import DeviceGraph

    hg = synth.big_graph(n_ops, 200_000, seed=8)
    ctx = _lib.default_context()
    dg = DeviceGraph.upload(ctx, hg)
    out = {}
    for ssv, wt in (("0", "0"), ("1", "0"), ("1", "1")):
        monkeypatch.setenv("MR_TR_SSV", ssv)
        monkeypatch.setenv("MR_TR_ROW_WT", wt)
        dg.pagerank(True)
        out[(ssv, wt)] = dg.fetch()
    for k in (("1", "0"), ("1", "1")):
        assert out[k][0].tobytes() == out[("0", "0")][0].tobytes(), k
        np.testing.assert_array_equal(out[k][1], out[("0", "0")][1])
    dg.close()


def _oracle_graph_from_host(hg) -> "orc.Graph":
    T, N = hg.T, hg.N
    sr_t = np.repeat(np.arange(T, dtype=np.int64), np.diff(hg.sr_off))
    ss_c = np.repeat(np.arange(N, dtype=np.int64), np.diff(hg.ss_off))
    return orc.Graph(list(range(N)), list(range(T)), sr_t, hg.sr_ops.astype(np.int64), sr_t,
                     hg.sr_ops.astype(np.int64), hg.len_t.astype(np.int64), hg.len_o.astype(np.int64), ss_c,
                     hg.ss_par.astype(np.int64), hg.nchild.astype(np.int64), np.arange(T, dtype=np.int64),
                     hg.len_t.astype(np.int64))


def _with_long_traces(hg, n_long, width, seed):
    """Append n_long traces of `width` distinct ops each: their tiles exceed the staged-id cap and
    take the fused kernel's long-tile path."""
    from microrank_amd.graph import HostGraph

    rng = np.random.default_rng(seed)
    ops = np.sort(np.stack([rng.choice(hg.N, width, replace=False) for _ in range(n_long)]), axis=1)
    sr_ops = np.concatenate([hg.sr_ops, ops.ravel().astype(np.int32)])
    sr_off = np.concatenate([hg.sr_off, hg.sr_off[-1] + width * np.arange(1, n_long + 1, dtype=np.int64)])
    len_t = np.concatenate([hg.len_t, np.full(n_long, width, np.int32)])
    len_o = hg.len_o + np.bincount(ops.ravel(), minlength=hg.N).astype(np.int32)
    T = hg.T + n_long
    return HostGraph(range(hg.N), range(T), sr_off, sr_ops, None, None, len_t, len_o, hg.ss_off, hg.ss_par,
                     hg.nchild, None, None)


@pytest.mark.parametrize("anomaly", [False, True])
def test_large_op_count_multi_tile_long_tiles(anomaly):
    """9k ops (su gathered from L2, not LDS), 250k traces (several tiles per block: the pipelined
    variant) plus 3k 60-op traces (tiles past the staged-id cap: the long-tile path), ragged last
    tile: GPU vs oracle at 1e-10, coverage exact, bitwise reruns."""
    from microrank_amd import _lib, synth
    from microrank_amd.graph import DeviceGraph

    hg = _with_long_traces(synth.big_graph(9000, 250_000, seed=5), 3000, 60, seed=6)
    g = _oracle_graph_from_host(hg)
    kind = orc.trace_kinds(g)
    v = orc.preference(g, kind, anomaly)
    s = orc.power_iteration(g, v)
    w_ref, cov_ref = orc.weights(g, s)
    ctx = _lib.default_context()
    dg = DeviceGraph.upload(ctx, hg)
    dg.pagerank(anomaly)
    w, cov = dg.fetch()
    np.testing.assert_array_equal(cov, np.array(list(cov_ref.values())))
    np.testing.assert_allclose(w, np.array(list(w_ref.values())), rtol=RTOL64, atol=0)
    dg.pagerank(anomaly)
    w2, _ = dg.fetch()
    assert w2.tobytes() == w.tobytes(), "rerun not bitwise identical"
    dg.close()


def _with_cold_traces(hg, n, lo, seed):
    """Append n traces of 1..3 distinct ops drawn from [lo, N): traces whose ops are all outside
    the wide path's hot set (a pad id in the LDS walk, every entry on the cold side)."""
    from microrank_amd.graph import HostGraph

    rng = np.random.default_rng(seed)
    width = rng.integers(1, 4, n)
    ops = [np.sort(rng.choice(np.arange(lo, hg.N), w, replace=False)) for w in width]
    flat = np.concatenate(ops).astype(np.int32)
    sr_ops = np.concatenate([hg.sr_ops, flat])
    sr_off = np.concatenate([hg.sr_off, hg.sr_off[-1] + np.cumsum(width).astype(np.int64)])
    len_t = np.concatenate([hg.len_t, width.astype(np.int32)])
    len_o = hg.len_o + np.bincount(flat, minlength=hg.N).astype(np.int32)
    return HostGraph(range(hg.N), range(hg.T + n), sr_off, sr_ops, None, None, len_t, len_o, hg.ss_off, hg.ss_par,
                     hg.nchild, None, None)


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_wide_fused_path_against_oracle(precision):
    """N = 50000 > 16384 (config C5's regime): the wide fused path -- hot ops through the LDS walk,
    cold entries through k_cold_trace / k_cold_ops over 3 op ranges -- plus 3k traces with no hot op
    at all.  GPU vs oracle (fp64 1e-10, fp32 1e-4), coverage exact, bitwise reruns."""
    from microrank_amd import _lib, synth
    from microrank_amd.graph import DeviceGraph

    hg = _with_cold_traces(synth.big_graph(50_000, 40_000, seed=9), 3000, 30_000, seed=10)
    g = _oracle_graph_from_host(hg)
    kind = orc.trace_kinds(g)
    s = orc.power_iteration(g, orc.preference(g, kind, True))
    w_ref, cov_ref = orc.weights(g, s)
    ctx = _lib.default_context()
    dg = DeviceGraph.upload(ctx, hg)
    dg.pagerank(True, precision=precision)
    w, cov = dg.fetch()
    tol = RTOL64 if precision == "fp64" else 1e-4
    np.testing.assert_array_equal(cov, np.array(list(cov_ref.values())))
    np.testing.assert_allclose(w, np.array(list(w_ref.values())), rtol=tol, atol=0)
    dg.pagerank(True, precision=precision)
    w2, _ = dg.fetch()
    assert w2.tobytes() == w.tobytes(), "rerun not bitwise identical"
    dg.close()


@pytest.mark.parametrize("part_min", [None, "0"])
def test_kind_hash_collision_retries_with_next_seed(monkeypatch, part_min):
    """MR_KIND_TEST_COLLIDE narrows the first attempt's kind keys to 2 bits, so distinct trace
    kinds share keys: the exact verification must catch it and the call must rerun with the next
    seed, giving the same kinds and weights as an uncollided run (pagerank.py:54-66)."""
    from microrank_amd.pagerank import trace_pagerank

    case = load_golden("c1.json")
    from conftest import regen_window

    _, adf = regen_window(case)
    tnames = sorted(adf["traceID"].unique())
    oo, ot, to, pt = golden_graph_dicts(case["graph_swapped_anomaly"], tnames)
    ref = trace_pagerank(oo, ot, to, pt, True)
    if part_min is not None:   # the partition path's verification (k_kind_final)
        monkeypatch.setenv("MR_KIND_PART_MIN", part_min)
    monkeypatch.setenv("MR_KIND_TEST_COLLIDE", "1")
    got = trace_pagerank(oo, ot, to, pt, True)
    assert list(got[0]) == list(ref[0]) and got[1] == ref[1]
    assert [float(x) for x in got[0].values()] == [float(x) for x in ref[0].values()]
    _check(got, case["pr_anomaly"], RTOL64)


def test_context_destroy_frees_its_handles():
    """A context destroyed before its graphs / span tables (garbage-collection order of a
    reference cycle) frees them itself; freeing the stale handles afterwards is a no-op."""
    from microrank_amd import _lib
    from microrank_amd.graph import DeviceGraph
    from microrank_amd.preprocess_data import DeviceSpans
    from conftest import regen_window
    from microrank_amd.spans import SpanTable

    d = load_golden("dict_cases.json")["fig3"]["input"]
    cx = _lib.Context(0)
    g = orc.graph_from_dicts(d["operation_operation"], d["operation_trace"], d["trace_operation"], d["pr_trace"])
    dg = DeviceGraph.upload(cx, host_graph_from_oracle(g))
    _, adf = regen_window(load_golden("c1.json"))
    sp = DeviceSpans(cx, SpanTable.from_dataframe(adf))
    h_graph, h_spans = dg.h, sp.h
    cx.close()
    lib = _lib.load()
    assert lib.mr_graph_free(h_graph) == 0 and lib.mr_spans_free(h_spans) == 0   # stale: no-op
    dg.close()
    sp.close()


@pytest.mark.parametrize("name", ["c1", "pods_dup_broken", "ops200", "span_times"])
def test_kind_compressed_matches_reference(name):
    """§8(f) f4: the kind-compressed ranking (one representative per kind, multiplicities in q
    and the preference sums) gives the reference fixtures' weights at 1e-10."""
    from microrank_amd.pagerank import trace_pagerank

    case = load_golden(f"{name}.json")
    from conftest import regen_window

    _, adf = regen_window(case)
    tnames = sorted(adf["traceID"].unique())
    for gkey, anomaly, pkey in (("graph_swapped_normal", False, "pr_normal"),
                                ("graph_swapped_anomaly", True, "pr_anomaly")):
        dicts = golden_graph_dicts(case[gkey], tnames)
        _check(trace_pagerank(*dicts, anomaly, compress_kinds=True), case[pkey], RTOL64)


@pytest.mark.parametrize("anomaly", [False, True])
@pytest.mark.parametrize("part_min", [None, "0"])
def test_kind_compressed_c2_matches_uncompressed(c2, anomaly, part_min, monkeypatch):
    """C2 graph (hot kinds): compressed weights within 1e-10 of the uncompressed ranking and of
    the oracle, coverage exact, for both kinds paths; far fewer kinds than traces."""
    from microrank_amd import _lib
    from microrank_amd.graph import DeviceGraph

    if part_min is not None:
        monkeypatch.setenv("MR_KIND_PART_MIN", part_min)
    st, sg = c2
    g = sg.as_graph()
    ctx = _lib.default_context()
    dg = DeviceGraph.upload(ctx, host_graph_from_oracle(g))
    dg.pagerank(anomaly)
    w0, cov0, k0, _ = dg.fetch(kinds=True)
    dg.pagerank(anomaly, compress_kinds=True)
    w1, cov1, k1, _ = dg.fetch(kinds=True)
    np.testing.assert_array_equal(cov1, cov0)
    np.testing.assert_array_equal(k1, k0)
    np.testing.assert_allclose(w1, w0, rtol=1e-10, atol=0)
    assert (1.0 / k0).sum() < 0.6 * g.T   # the C2 window repeats call paths (113k kinds of 200k traces)
    # a later call ranks the kept representatives' graph: with the other preference as well, bitwise
    # the same as a call that rebuilds it (MR_KC_NOCACHE), and within 1e-10 of the uncompressed one
    dg.pagerank(not anomaly, compress_kinds=True)
    w2, _ = dg.fetch()
    monkeypatch.setenv("MR_KC_NOCACHE", "1")
    dg.pagerank(not anomaly, compress_kinds=True)
    w3, _ = dg.fetch()
    monkeypatch.delenv("MR_KC_NOCACHE")
    assert w2.tobytes() == w3.tobytes()
    dg.pagerank(not anomaly)
    w4, _ = dg.fetch()
    np.testing.assert_allclose(w2, w4, rtol=1e-10, atol=0)
    dg.close()


def test_c4_full_scale_properties():
    """BASELINE configs[3] at full size (10k ops / 10M traces, fp64, one GPU): no oracle finishes
    at this size, so size-independent properties -- bitwise reruns, coverage summing to the pairs,
    the kind classes partitioning the traces, the weights' max-normalisation identity
    (pagerank.py:107: N * sum(w) = (N * max(w))^2 when max(s) = 1), and the kind-compressed
    ranking equal to the uncompressed one (1e-10, top-5 identical)."""
    from microrank_amd import _lib, synth
    from microrank_amd.graph import DeviceGraph

    hg = synth.big_graph(10_000, 10_000_000, seed=11)
    nnz = int(hg.sr_ops.size)
    ctx = _lib.default_context()
    dg = DeviceGraph.upload(ctx, hg)
    del hg
    dg.pagerank(True)
    w1, cov, kind, _ = dg.fetch(kinds=True)
    dg.pagerank(True)
    w2, _ = dg.fetch()
    assert w1.tobytes() == w2.tobytes()
    assert int(cov.astype(np.int64).sum()) == nnz
    n_kinds = float((1.0 / kind).sum())
    assert abs(n_kinds - round(n_kinds)) < 1e-6 * n_kinds and 1 <= round(n_kinds) <= 10_000_000
    N = w1.size
    np.testing.assert_allclose(N * w1.sum(), (N * w1.max()) ** 2, rtol=1e-9)
    dg.pagerank(True, compress_kinds=True)
    w3, _ = dg.fetch()
    np.testing.assert_allclose(w3, w1, rtol=1e-10, atol=0)
    assert list(np.argsort(-w3, kind="stable")[:5]) == list(np.argsort(-w1, kind="stable")[:5])
    dg.close()


def test_c5_full_scale_properties():
    """BASELINE configs[4] at its stated size: 100k ops / 100M traces (1.5G distinct pairs, power-law
    op popularity, the root op in every trace) -- the wide fused iteration (hot ops through k_tr_a,
    the cold tail through k_cold_trace / k_cold_ops).  No oracle finishes at this size, so
    size-independent properties: bitwise reruns in fp32 and fp64, coverage summing to the pairs,
    the max-normalisation identity (pagerank.py:107: N sum(w) = (N max(w))^2) in both precisions,
    fp32 within 1e-4 of fp64 (the north star's fp32 tolerance) with the same top-5."""
    from microrank_amd import _lib, synth
    from microrank_amd.graph import DeviceGraph

    hg = synth.big_graph(100_000, 100_000_000, seed=12)
    nnz = int(hg.sr_ops.size)
    assert nnz > 2**30
    ctx = _lib.default_context()
    dg = DeviceGraph.upload(ctx, hg)
    del hg
    res = {}
    for prec in ("fp32", "fp64"):
        dg.pagerank(True, precision=prec)
        w, cov = dg.fetch()
        dg.pagerank(True, precision=prec)
        w2, _ = dg.fetch()
        assert w.tobytes() == w2.tobytes(), prec
        assert int(cov.astype(np.int64).sum()) == nnz
        N = w.size
        np.testing.assert_allclose(N * w.sum(), (N * w.max()) ** 2, rtol=1e-9 if prec == "fp64" else 1e-5)
        res[prec] = w
    big = res["fp64"] > 1e-6 * res["fp64"].max()
    np.testing.assert_allclose(res["fp32"][big], res["fp64"][big], rtol=1e-4)
    assert list(np.argsort(-res["fp32"], kind="stable")[:5]) == list(np.argsort(-res["fp64"], kind="stable")[:5])
    dg.close()


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_wide_span_graph_with_broken_traces_against_oracle(precision):
    """C5's span form at oracle size: 60k ops / 40k traces of spans with 5 % broken traces (a
    dropped parent span: orphans, T11) and 1 % duplicated root spanIDs, built on the device (K1,
    mr_graph_build) into a graph wide enough for the wide fused iteration (N > 16384), then ranked:
    node order, coverage and weights against the oracle's span_graph + trace_pagerank (fp64 1e-10,
    fp32 1e-4)."""
    from microrank_amd import _lib, synth
    from microrank_amd.graph import DeviceGraph
    from microrank_amd.preprocess_data import DeviceSpans
    import ctypes as C
    from microrank_amd._lib import ptr

    st = synth.big_spans(60_000, 40_000, seed=21, dup_frac=0.01, broken_frac=0.05)
    # spread the non-root spans' ops over the op space (per-trace offsets), so ~59k ops appear
    op = st.podop.astype(np.int64)
    st.podop = st.svcop = np.where(st.parent < 0, op, (op + (st.trace.astype(np.int64) % 997) * 61) % 60_000
                                   ).astype(np.int32)
    sel = np.ones(st.n_traces, bool)
    sel[::7] = False                                    # a trace_list that is not every trace
    sg = orc.span_graph(st.trace, st.podop, st.span, st.parent, sel)
    g = sg.as_graph()
    assert g.N > 16384 and g.ss_c.size > 0
    s = orc.power_iteration(g, orc.preference(g, orc.trace_kinds(g), True))
    w_ref, cov_ref = orc.weights(g, s)
    ctx = _lib.default_context()
    dev = DeviceSpans(ctx, st)
    lib = _lib.load()
    mask = sel.astype(np.uint8)
    h = _lib.P()
    ctx.check(lib.mr_graph_build(ctx.h, dev.h, ptr(mask, C.c_uint8), C.byref(h)), "mr_graph_build")
    n, t, nnz, e = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int64()
    lib.mr_graph_info(h, C.byref(n), C.byref(t), C.byref(nnz), C.byref(e))
    node = np.empty(n.value, np.int32)
    tcode = np.empty(t.value, np.int32)
    ctx.check(lib.mr_graph_nodes(h, ptr(node, C.c_int32), ptr(tcode, C.c_int32)), "mr_graph_nodes")
    assert node.tolist() == list(sg.node_podop) and tcode.tolist() == list(sg.trace_codes)
    assert (nnz.value, e.value) == (g.sr_o.size, g.ss_c.size)
    dg = DeviceGraph(ctx, h, None, None, n.value, t.value)
    dg.pagerank(True, precision=precision)
    w, cov = dg.fetch()
    np.testing.assert_array_equal(cov, np.array(list(cov_ref.values())))
    np.testing.assert_allclose(w, np.array(list(w_ref.values())), rtol=RTOL64 if precision == "fp64" else RTOL32,
                               atol=0)
    dg.close()
    dev.close()


@pytest.mark.parametrize("anomaly", [False, True])
def test_config_keywords_against_oracle(anomaly):
    """d / alpha / iters / phi as keywords (pagerank.py:116-117, :82-84): non-default
    values on the c1 window's graph equal the oracle run with the same values (1e-10)."""
    from microrank_amd.pagerank import trace_pagerank
    from conftest import regen_window

    case = load_golden("c1.json")
    _, adf = regen_window(case)
    tnames = sorted(adf["traceID"].unique())
    dicts = golden_graph_dicts(case["graph_swapped_anomaly"], tnames)
    kw = dict(d=0.7, alpha=0.05, iters=10, phi=0.3)
    w, num = trace_pagerank(*dicts, anomaly, **kw)
    w_ref, num_ref = orc.trace_pagerank(*dicts, anomaly, **kw)
    assert list(w) == list(w_ref) and num == num_ref
    np.testing.assert_allclose(np.array(list(w.values())), np.array(list(w_ref.values())), rtol=1e-10, atol=0)
    w0, _ = trace_pagerank(*dicts, anomaly)
    assert [float(x) for x in w0.values()] != [float(x) for x in w.values()]
    with pytest.raises(ValueError):
        trace_pagerank(*dicts, anomaly, iters=-1)


def _with_hot_only_traces(hg, hot, seed):
    """Append traces made of hot ops only (1..len(hot) of them): with the hot ops stripped from the
    id chunks such a trace keeps its first hot op in the list (no empty traces)."""
    from microrank_amd.graph import HostGraph

    rng = np.random.default_rng(seed)
    ops = [np.sort(rng.choice(hot, k, replace=False)) for k in range(1, len(hot) + 1) for _ in range(40)]
    width = np.array([len(o) for o in ops])
    flat = np.concatenate(ops).astype(np.int32)
    sr_ops = np.concatenate([hg.sr_ops, flat])
    sr_off = np.concatenate([hg.sr_off, hg.sr_off[-1] + np.cumsum(width).astype(np.int64)])
    len_t = np.concatenate([hg.len_t, width.astype(np.int32)])
    len_o = hg.len_o + np.bincount(flat, minlength=hg.N).astype(np.int32)
    return HostGraph(range(hg.N), range(hg.T + len(ops)), sr_off, sr_ops, None, None, len_t, len_o, hg.ss_off,
                     hg.ss_par, hg.nchild, None, None)


@pytest.mark.parametrize("anomaly", [False, True])
def test_hot_op_layout_against_oracle(anomaly, monkeypatch):
    """Register-accumulated hot ops (the 8 most covered ops leave k_tr_a's id chunks; forced here
    on a 300k-trace graph with MR_TR_HOT_MIN=0): short tiles, long tiles (60-op traces: the general
    walk) and hot-only traces.  GPU vs oracle at 1e-10 (fp64) / 1e-4 (fp32), coverage exact, bitwise
    reruns, and within 1e-12 of the layout without hot ops (only the summation order differs)."""
    from microrank_amd import _lib, synth
    from microrank_amd.graph import DeviceGraph

    hg = _with_hot_only_traces(_with_long_traces(synth.big_graph(1000, 300_000, seed=21), 2000, 60, seed=22),
                               np.arange(8), seed=23)
    g = _oracle_graph_from_host(hg)
    kind = orc.trace_kinds(g)
    s = orc.power_iteration(g, orc.preference(g, kind, anomaly))
    w_ref, cov_ref = orc.weights(g, s)
    ctx = _lib.default_context()
    res = {}
    for hot in ("0", "8"):
        monkeypatch.setenv("MR_TR_HOT", hot)
        monkeypatch.setenv("MR_TR_HOT_MIN", "0")
        monkeypatch.setenv("MR_TR_HOT_FRAC", "0")
        dg = DeviceGraph.upload(ctx, hg)
        dg.pagerank(anomaly)
        w, cov = dg.fetch()
        np.testing.assert_array_equal(cov, np.array(list(cov_ref.values())))
        np.testing.assert_allclose(w, np.array(list(w_ref.values())), rtol=RTOL64, atol=0)
        dg.pagerank(anomaly)
        w2, _ = dg.fetch()
        assert w2.tobytes() == w.tobytes(), "rerun not bitwise identical"
        dg.pagerank(anomaly, precision="fp32")
        w3, _ = dg.fetch()
        np.testing.assert_allclose(w3, np.array(list(w_ref.values())), rtol=RTOL32, atol=0)
        res[hot] = w
        dg.close()
    np.testing.assert_allclose(res["8"], res["0"], rtol=1e-12, atol=0)


@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_wide_hot_op_layout_against_oracle(precision, monkeypatch):
    """The wide path (N = 50000) with the hot ops of its LDS walk register-accumulated (forced with
    MR_TR_HOT_MIN=0): GPU vs oracle, bitwise reruns."""
    from microrank_amd import _lib, synth
    from microrank_amd.graph import DeviceGraph

    monkeypatch.setenv("MR_TR_HOT_MIN", "0")
    monkeypatch.setenv("MR_TR_HOT_FRAC", "0")
    hg = _with_cold_traces(synth.big_graph(50_000, 40_000, seed=9), 3000, 30_000, seed=10)
    g = _oracle_graph_from_host(hg)
    kind = orc.trace_kinds(g)
    s = orc.power_iteration(g, orc.preference(g, kind, False))
    w_ref, cov_ref = orc.weights(g, s)
    ctx = _lib.default_context()
    dg = DeviceGraph.upload(ctx, hg)
    dg.pagerank(False, precision=precision)
    w, cov = dg.fetch()
    tol = RTOL64 if precision == "fp64" else 1e-4
    np.testing.assert_array_equal(cov, np.array(list(cov_ref.values())))
    np.testing.assert_allclose(w, np.array(list(w_ref.values())), rtol=tol, atol=0)
    dg.pagerank(False, precision=precision)
    w2, _ = dg.fetch()
    assert w2.tobytes() == w.tobytes(), "rerun not bitwise identical"
    dg.close()
