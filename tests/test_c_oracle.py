"""The C restatement (oracle/mr_oracle.c, bench.py's cpu_baseline) agrees with the numpy
oracle and with the reference's golden vectors."""
import numpy as np
import pytest

import c_oracle
import oracle as orc
from conftest import load_golden, regen_window, unhex
from microrank_amd.spans import SpanTable


@pytest.mark.parametrize("name", ["c1", "pods_dup_broken", "ops200"])
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
