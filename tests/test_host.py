"""Host-side logic of the drop-in surface (no GPU): the span-table cache key, the detector's
trace lists, the reference's config defaults as keywords."""
import inspect

import numpy as np
import pandas as pd
import pytest

from conftest import load_golden, regen_window


def test_fingerprint_sees_column_replacement_sampled_edits_and_invalidate():
    """The cache key is O(columns): buffer identity (the reference's own mutations replace whole
    columns, preprocess_data.py:27,53,100), a 64-row content sample (first and last rows included)
    and a version bumped by this package's mutating drop-ins / invalidate()."""
    from microrank_amd.preprocess_data import _fingerprint, get_operation_duration_data, invalidate

    case = load_golden("c1.json")
    _, adf = regen_window(case)
    df = adf.copy()
    fp = _fingerprint(df)
    assert _fingerprint(df) == fp                        # stable while nothing changes
    df["operation"] = "x"                               # a column the table does not read
    assert _fingerprint(df) == fp
    df.loc[df.index[0], "duration"] += 1                 # in place, a sampled row
    fp2 = _fingerprint(df)
    assert fp2 != fp
    df.loc[df.index[-1], "spanID"] = "changed"           # in place, last row (sampled)
    fp3 = _fingerprint(df)
    assert fp3 != fp2
    get_operation_duration_data(case["operation_list"], df)   # replaces operationName (+ version)
    fp4 = _fingerprint(df)
    assert fp4 != fp3
    invalidate(df)
    assert _fingerprint(df) != fp4
    assert _fingerprint(df.iloc[:0]) == (0, tuple(c for c in df.columns if c in (
        "traceID", "spanID", "ParentSpanId", "serviceName", "operationName", "podName", "duration", "startTime",
        "endTime")))


def test_trace_list_is_a_plain_list_with_codes():
    from microrank_amd.anormaly_detector import TraceList

    class T:
        trace_names = ["a", "b", "c", "d"]
        meta = {}

    t = T()
    lst = TraceList.of(t, np.array([1, 3]))
    assert lst == ["b", "d"] and isinstance(lst, list)
    assert lst.codes_for(t).tolist() == [1, 3]
    assert lst.codes_for(T()) is None                   # another table
    lst.append("a")
    assert lst.codes_for(t) is None                     # changed by the caller
    assert TraceList(["b"]).codes_for(t) is None


def test_reference_defaults_are_keywords():
    """d = 0.85, alpha = 0.01 (pagerank.py:116), 25 iterations (:117), phi = 0.5
    (:82-84) are keywords of trace_pagerank with the reference's values as defaults."""
    from microrank_amd import pagerank

    sig = inspect.signature(pagerank.trace_pagerank)
    assert [sig.parameters[k].default for k in ("d", "alpha", "iters", "phi")] == [0.85, 0.01, 25, 0.5]
    assert list(sig.parameters)[:5] == ["operation_operation", "operation_trace", "trace_operation", "pr_trace",
                                        "anomaly"]


@pytest.mark.parametrize("phi", [0.5, 0.3])
def test_oracle_phi_keyword(phi):
    """The oracle's preference with phi = 0.5 is the reference's (pinned by the goldens elsewhere);
    another phi changes only the anomaly form."""
    import oracle as orc

    d = load_golden("dict_cases.json")["fig3"]["input"]
    g = orc.graph_from_dicts(d["operation_operation"], d["operation_trace"], d["trace_operation"], d["pr_trace"])
    k = orc.trace_kinds(g)
    base = orc.preference(g, k, True)
    got = orc.preference(g, k, True, phi)
    assert (got == base).all() == (phi == 0.5)
    assert (orc.preference(g, k, False) == orc.preference(g, k, False, phi)).all()
