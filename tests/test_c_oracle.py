"""The C restatement (oracle/mr_oracle.c, bench.py's cpu_baseline) agrees with the numpy
oracle and with the reference's golden vectors."""
import numpy as np
import pytest

import c_oracle
import oracle as orc
from conftest import load_golden, regen_window, unhex
from microrank_amd.spans import SpanTable


@pytest.mark.parametrize("name", ["c1", "pods_dup_broken", "ops200", "span_times"])
def test_c_window_matches_reference(name):
    case = load_golden(f"{name}.json")
    ndf, adf = regen_window(case)
    st = SpanTable.from_dataframe(adf)
    slo = {k: (float.fromhex(a), float.fromhex(b)) for k, (a, b) in case["slo"].items()}
    a3 = np.array([slo[n][0] + 3 * slo[n][1] if n in slo else 0.0 for n in st.svcop_names])
    ok = np.array([n in slo for n in st.svcop_names], np.uint8)
    res = c_oracle.rca_window(st, case["detect"]["start_ns"], case["detect"]["end_ns"], a3, ok, nthreads=2)
    codes, scores, na, nn, _ = res
    assert na == len(case["detect"]["abnormal"]) and nn == len(case["detect"]["normal"])
    exp = case["spectrum"]["dstar2"]
    assert [st.podop_names[c] for c in codes] == exp["top"]
    np.testing.assert_allclose(scores, unhex(exp["score"]), rtol=1e-10)


@pytest.mark.parametrize("anomaly", [False, True])
def test_c_graph_pagerank_matches_numpy_oracle(anomaly):
    case = load_golden("pods_dup_broken.json")
    _, adf = regen_window(case)
    st = SpanTable.from_dataframe(adf)
    sel = np.zeros(st.n_traces, bool)
    sel[case["detect"]["normal"]] = True
    node, w, cov, nnz = c_oracle.graph_pagerank(st, sel, anomaly)
    sg = orc.span_graph(st.trace, st.podop, st.span, st.parent, sel)
    np.testing.assert_array_equal(node, sg.node_podop)
    g = sg.as_graph()
    wr, cr = orc.weights(g, orc.power_iteration(g, orc.preference(g, orc.trace_kinds(g), anomaly)))
    np.testing.assert_array_equal(cov, list(cr.values()))
    np.testing.assert_allclose(w, list(wr.values()), rtol=1e-12)


def _san_binary():
    import os
    import subprocess

    here = os.path.join(os.path.dirname(c_oracle.__file__))
    subprocess.run(["make", "-s", "san"], cwd=here, check=True)
    return os.path.join(here, "_build", "mr_oracle_san")


@pytest.mark.parametrize("name", ["pods_dup_broken", "span_times"])
def test_c_restatement_under_asan_ubsan(name, tmp_path):
    """the C restatement runs clean under AddressSanitizer + UndefinedBehaviorSanitizer
    (any report aborts the binary: -fno-sanitize-recover=all) and gives the unsanitised result."""
    import os
    import subprocess

    case = load_golden(f"{name}.json")
    _, adf = regen_window(case)
    st = SpanTable.from_dataframe(adf)
    slo = {k: (float.fromhex(a), float.fromhex(b)) for k, (a, b) in case["slo"].items()}
    a3 = np.array([slo[n][0] + 3 * slo[n][1] if n in slo else 0.0 for n in st.svcop_names])
    ok = np.array([n in slo for n in st.svcop_names], np.uint8)
    t0, t1 = case["detect"]["start_ns"], case["detect"]["end_ns"]
    f = tmp_path / "window.bin"
    with open(f, "wb") as fh:
        fh.write(np.array([st.n_spans], np.int64).tobytes())
        fh.write(np.array([st.n_traces, st.n_podops, st.n_svcops, 0], np.int32).tobytes())
        fh.write(np.array([t0, t1], np.int64).tobytes())
        for a, dt in ((st.trace, np.int32), (st.podop, np.int32), (st.svcop, np.int32), (st.span, np.int64),
                      (st.parent, np.int64), (st.duration, np.int64), (st.tstart, np.int64), (st.tend, np.int64),
                      (a3, np.float64), (ok, np.uint8)):
            fh.write(np.ascontiguousarray(a, dtype=dt).tobytes())
    env = dict(os.environ, ASAN_OPTIONS="abort_on_error=0:detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([_san_binary(), str(f)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    lines = r.stdout.split("\n")
    na, nn, n_out, edges = map(int, lines[0].split())
    got = [(int(l.split()[0]), float.fromhex(l.split()[1])) for l in lines[1:1 + n_out]]
    codes, scores, na2, nn2, edges2 = c_oracle.rca_window(st, t0, t1, a3, ok, nthreads=2)
    assert (na, nn, edges) == (na2, nn2, edges2)
    assert [c for c, _ in got] == list(codes)
    assert [s for _, s in got] == list(scores)
    assert [st.podop_names[c] for c, _ in got] == case["spectrum"]["dstar2"]["top"]


@pytest.mark.parametrize("anomaly", [False, True])
def test_c_incidence_pagerank_matches_numpy_oracle(anomaly):
    """oracle_incidence_pagerank (bench.py's C4 CPU baseline: hashed kinds, OpenMP iterations) on
    a power-law incidence graph equals the numpy oracle (1e-12) with the same coverage, on one
    thread and on four."""
    from microrank_amd import synth

    hg = synth.big_graph(300, 30_000, seed=3)
    T, N = hg.T, hg.N
    sr_t = np.repeat(np.arange(T, dtype=np.int64), np.diff(hg.sr_off))
    ss_c = np.repeat(np.arange(N, dtype=np.int64), np.diff(hg.ss_off))
    g = orc.Graph(list(range(N)), list(range(T)), sr_t, hg.sr_ops.astype(np.int64), sr_t,
                  hg.sr_ops.astype(np.int64), hg.len_t, hg.len_o, ss_c, hg.ss_par.astype(np.int64), hg.nchild,
                  np.arange(T), hg.len_t.copy())
    s = orc.power_iteration(g, orc.preference(g, orc.trace_kinds(g), anomaly))
    w_ref, cov_ref = orc.weights(g, s)
    for nt in (1, 4):
        w, cov, tp = c_oracle.incidence_pagerank(hg, anomaly, nthreads=nt)
        np.testing.assert_array_equal(cov, np.array(list(cov_ref.values())))
        np.testing.assert_allclose(w, np.array(list(w_ref.values())), rtol=1e-12, atol=0)
        assert tp[0] > 0 and tp[1] > 0
