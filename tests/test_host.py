"""Host-side logic of the drop-in surface (no GPU): the span-table cache key, the detector's
trace lists, the reference's config defaults as keywords."""
import inspect

import numpy as np
import pandas as pd
import pytest

from conftest import load_golden, regen_window


def test_fingerprint_is_exact_for_any_in_place_edit_and_invalidate():
    """The cache key decides "unchanged" exactly: any in-place cell edit of a
    column the span table reads -- at any row, not a sample -- and any column replacement (the
    reference's own mutations, preprocess_data.py:27,53,100) no longer match; columns the table
    does not read do not matter; invalidate() and this package's mutating drop-ins bump the
    version."""
    from microrank_amd.preprocess_data import _fingerprint, get_operation_duration_data, invalidate

    case = load_golden("c1.json")
    _, adf = regen_window(case)
    df = adf.copy()
    n = len(df)
    fp = _fingerprint(df)
    assert fp.matches(df) and fp.matches(df)             # stable while nothing changes
    df["operation"] = "x"                               # a column the table does not read
    assert fp.matches(df)
    mid = df.index[n // 2 + 7]                          # an arbitrary interior row
    for col, val in (("duration", int(df["duration"].iloc[n // 2 + 7]) + 1), ("operationName", "changed-op"),
                     ("spanID", "changed-span"), ("startTime", df["startTime"].iloc[0])):
        fp = _fingerprint(df)
        assert fp.matches(df)
        df.loc[mid, col] = val                          # in place, one cell
        assert not fp.matches(df), col
    # the same value written back: the content is what it was, the key matches again
    fp = _fingerprint(df)
    old = df.loc[mid, "operationName"]
    df.loc[mid, "operationName"] = "tmp"
    df.loc[mid, "operationName"] = old
    assert fp.matches(df)
    fp = _fingerprint(df)
    get_operation_duration_data(case["operation_list"], df)   # replaces operationName (+ version)
    assert not fp.matches(df)
    fp = _fingerprint(df)
    invalidate(df)
    assert not fp.matches(df)
    fp = _fingerprint(df.iloc[:0])
    assert fp.matches(df.iloc[:0]) and not fp.matches(df)


def test_fingerprint_nullable_and_extension_columns():
    """nullable (masked) columns -- an Int64 duration holding pd.NA -- and other
    extension arrays keep an exact, stable key: unchanged frames match on every lookup (no rebuild
    per call), an in-place edit anywhere (value or NA-ness) does not."""
    from microrank_amd.preprocess_data import _fingerprint

    case = load_golden("c1.json")
    _, adf = regen_window(case)
    df = adf.copy()
    n = len(df)
    df["duration"] = df["duration"].astype("Int64")
    df.loc[df.index[3], "duration"] = pd.NA
    df["podName"] = df["podName"].astype("category")     # another extension array
    fp = _fingerprint(df)
    assert fp.matches(df) and fp.matches(df)
    mid = df.index[n // 2 + 5]
    df.loc[mid, "duration"] = int(df["duration"].iloc[n // 2 + 5]) + 1
    assert not fp.matches(df)
    fp = _fingerprint(df)
    df.loc[mid, "duration"] = pd.NA                     # value -> NA
    assert not fp.matches(df)
    fp = _fingerprint(df)
    assert fp.matches(df)
    cats = list(df["podName"].cat.categories)
    df.loc[mid, "podName"] = cats[0] if df.loc[mid, "podName"] != cats[0] else cats[-1]
    assert not fp.matches(df)


def test_fingerprint_arrow_columns_and_cost():
    """Arrow-backed columns (read_traces_csv) match by identity of their immutable arrays (an
    in-place edit replaces the array); a C2-sized frame (2.7M spans) is checked in a few tens
    of ms -- O(rows) like the reference's own per-window filtering."""
    import time

    import pyarrow as pa

    from microrank_amd.preprocess_data import _fingerprint

    n = 50_000
    df = pd.DataFrame({"traceID": pd.array([f"t{i // 20}" for i in range(n)], dtype=pd.ArrowDtype(pa.string())),
                       "duration": np.arange(n, dtype=np.int64)})
    fp = _fingerprint(df)
    assert fp.matches(df)
    df.loc[df.index[n // 3], "traceID"] = "edited"
    assert not fp.matches(df)
    n = 2_740_000
    big = pd.DataFrame({c: np.array([f"s{i % 9973}" for i in range(n)], dtype=object) for c in
                        ("traceID", "spanID", "ParentSpanId", "serviceName", "operationName", "podName")})
    for c in ("duration", "startTime", "endTime"):
        big[c] = np.arange(n, dtype=np.int64)
    fp = _fingerprint(big)
    ts = time.perf_counter()
    for _ in range(5):
        assert fp.matches(big)
    per = (time.perf_counter() - ts) / 5
    assert per < 0.25, per
    big.loc[big.index[n - 12345], "podName"] = "edited"
    assert not fp.matches(big)


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


def test_fingerprint_reads_subset():
    """A call compares only the columns its result depends on: an edit of another column keeps
    the cached table for that call and is caught by the next call that reads the edited column."""
    from microrank_amd.preprocess_data import DETECT_READS, GRAPH_READS, _fingerprint

    n = 70_000
    df = pd.DataFrame({c: np.array([f"{c}{i % 977}" for i in range(n)], dtype=object) for c in
                       ("traceID", "spanID", "ParentSpanId", "serviceName", "operationName", "podName")})
    for c in ("duration", "startTime", "endTime"):
        df[c] = np.arange(n, dtype=np.int64)
    fp = _fingerprint(df)
    assert fp.matches(df, DETECT_READS) and fp.matches(df, GRAPH_READS) and fp.matches(df)
    df.loc[df.index[n // 2], "spanID"] = "edited"
    assert fp.matches(df, DETECT_READS)
    assert not fp.matches(df, GRAPH_READS) and not fp.matches(df)
    df.loc[df.index[7], "duration"] = -1
    assert not fp.matches(df, DETECT_READS)
