"""span ingest on the device (mr_spans_ingest) against the host factorisation
(SpanTable.from_dataframe, pandas), which the golden tests pin to the reference's naming and
ordering rules (preprocess_data.py:26-33, 151-165; T10).  Codes and name lists must be identical;
spanID codes are compared as partitions (only equality matters, T11)."""
import contextlib
import io
import os

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN, load_golden, regen_window

pytestmark = pytest.mark.gpu


def _canon(codes):
    """codes -> first-appearance ranks (equal codes stay equal, -1 stays -1)"""
    out = np.full(codes.shape, -1, np.int64)
    pos = codes >= 0
    _, first, inv = np.unique(codes[pos], return_index=True, return_inverse=True)
    rank = np.empty(first.size, np.int64)
    rank[np.argsort(first, kind="stable")] = np.arange(first.size)
    out[pos] = rank[inv]
    return out


def _check(df):
    from microrank_amd import _lib
    from microrank_amd.preprocess_data import DeviceSpans
    from microrank_amd.spans import SpanTable, arrow_columns

    host = SpanTable.from_dataframe(df)
    arrays = arrow_columns(df)
    assert arrays is not None
    ctx = _lib.default_context()
    dev_t, dev = DeviceSpans.ingest(ctx, df, arrays)
    assert (dev_t.n_spans, dev_t.n_traces, dev_t.n_podops, dev_t.n_svcops) == \
        (host.n_spans, len(host.trace_names), len(host.podop_names), len(host.svcop_names))
    assert list(dev_t.trace_names) == list(host.trace_names)
    assert list(dev_t.podop_names) == list(host.podop_names)
    assert list(dev_t.svcop_names) == list(host.svcop_names)
    assert np.array_equal(dev_t.trace, host.trace)
    assert np.array_equal(dev_t.podop, host.podop)
    assert np.array_equal(dev_t.svcop, host.svcop)
    # spanIDs: the same partition; parents: the same span (or none)
    assert np.array_equal(_canon(dev_t.span), _canon(host.span))
    assert np.array_equal(dev_t.parent < 0, host.parent < 0)
    m = host.parent >= 0
    # a parent code is a span code: map both through each side's canonical span ids
    dmap = dict(zip(dev_t.span.tolist(), _canon(dev_t.span).tolist()))
    hmap = dict(zip(host.span.tolist(), _canon(host.span).tolist()))
    assert [dmap[int(p)] for p in dev_t.parent[m]] == [hmap[int(p)] for p in host.parent[m]]
    return dev_t, dev


@pytest.mark.parametrize("name", ["c1", "pods_dup_broken", "span_times"])
def test_ingest_equals_host_factorisation_golden(name):
    case = load_golden(f"{name}.json")
    ndf, adf = regen_window(case)
    _check(adf)
    _check(ndf)


def test_ingest_edge_names():
    """Names that stress the string rules: '_' joins that collide, ts-ui-dashboard with zero, one
    and several '/', non-ASCII (code-point order = UTF-8 byte order), prefixes, long names,
    duplicated spanIDs, null / unknown parents, traceIDs of different lengths."""
    rows = [
        # traceID, spanID, parent, service, operation, pod
        ("t1", "s1", None, "ts-ui-dashboard", "GET /api/v1/x/123", "ui-pod"),
        ("t1", "s2", "s1", "a_b", "c", "p_q"),             # a_b + _ + c == a + _ + b_c
        ("t1", "s3", "s2", "a", "b_c", "p"),
        ("t10", "s4", None, "ts-ui-dashboard", "noslash", "ui-pod"),
        ("t10", "s5", "s4", "ts-ui-dashboard", "/lead", "ui-pod"),
        ("t10", "s6", "s5", "ts-ui-dashboard", "a/b/c/", "ui-pod"),
        ("t2", "s7", "zzz", "svcü", "opé", "podß"),     # parent that is no span
        ("t2", "s8", "s7", "svcü", "opéx", "pod"),
        ("t中", "s9", None, "svc\U0001F600", "op", "pod\U0001F600"),
        ("t2", "s1", "s9", "svc", "op", "pod"),           # duplicated spanID across traces
        ("t3", "s10", "s1", "svc", "o" * 70, "pod"),      # long names, > 64 bytes
        ("t3", "s11", "s10", "svc", "o" * 71, "pod"),
        ("t3", "s12", "", "svc", "", "pod"),              # empty op, empty parent string
        ("t", "s13", "s12", "svc", "op", "pod"),
        ("", "s14", None, "svc", "op", ""),               # empty traceID and pod
        ("t4", "s15", "s14", "ts-ui-dashboard-2", "GET /keep/1", "p"),   # not the UI service
    ]
    df = pd.DataFrame(rows, columns=["traceID", "spanID", "ParentSpanId", "serviceName", "operationName", "podName"])
    df["duration"] = np.arange(len(df), dtype=np.int64) * 1000 + 5
    t0 = pd.Timestamp("2024-01-01 00:00:00")
    df["startTime"] = t0
    df["endTime"] = t0 + pd.Timedelta(seconds=1)
    dev_t, _ = _check(df)
    assert "ts-ui-dashboard_GET /api/v1/x" in dev_t.svcop_names
    assert "ts-ui-dashboard_a/b/c" in dev_t.svcop_names and "ts-ui-dashboard_" in dev_t.svcop_names
    assert "ts-ui-dashboard-2_GET /keep/1" in dev_t.svcop_names
    assert dev_t.svcop_names.count("a_b_c") == 1   # the colliding joins share one code


def test_ingest_large_random_names():
    """200k spans of random-length random-byte names (UTF-8, incl. multibyte) against pandas."""
    rng = np.random.default_rng(7)
    alphabet = np.array(list("abcXYZ_/-09") + ["é", "中", "\U0001F600"], dtype=object)

    def names(n, lo, hi, k):
        pool = ["".join(rng.choice(alphabet, rng.integers(lo, hi))) for _ in range(k)]
        return np.array(pool, dtype=object)[rng.integers(0, k, n)]

    S = 200_000
    span = np.array([f"{x:x}" for x in rng.permutation(S * 2)[:S]], dtype=object)
    span[rng.integers(0, S, 500)] = span[rng.integers(0, S, 500)]    # duplicates
    parent = span[rng.integers(0, S, S)].copy()
    parent[rng.random(S) < 0.1] = None
    svc = names(S, 1, 20, 300)
    svc[rng.random(S) < 0.05] = "ts-ui-dashboard"
    df = pd.DataFrame({"traceID": names(S, 1, 40, 20_000), "spanID": span, "ParentSpanId": parent,
                       "serviceName": svc, "operationName": names(S, 0, 90, 2_000), "podName": names(S, 1, 30, 500),
                       "duration": rng.integers(1, 10**6, S).astype(np.int64)})
    _check(df)


@pytest.mark.parametrize("name", ["c1", "pods_dup_broken"])
def test_driver_same_on_host_factorisation(name, tmp_path, monkeypatch):
    """The drop-in driver prints the same whether the table came from the device ingest (default)
    or from the host factorisation."""
    from microrank_amd import online_rca, preprocess_data

    case = load_golden(f"{name}.json")
    _, adf = regen_window(case)
    slo = {k: [np.float64(float.fromhex(a)), np.float64(float.fromhex(b))] for k, (a, b) in case["slo"].items()}
    outs = []
    for host in (False, True):
        monkeypatch.setattr(preprocess_data, "_HOST_FACTORIZE", host)
        d = tmp_path / str(host)
        d.mkdir()
        monkeypatch.chdir(d)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            online_rca.online_anomaly_detect_RCA(adf.copy(), slo, case["operation_list"])
        outs.append((buf.getvalue(), (d / "result.csv").read_text()))
    assert outs[0] == outs[1]
    assert outs[0][0].splitlines()[0] == case["driver_stdout"].splitlines()[0]


def test_edges_parquet_ingest():
    df = pd.read_parquet(os.path.join(GOLDEN, "edges_spans.parquet"))
    _check(df)


@pytest.mark.parametrize("name", ["c1", "pods_dup_broken"])
def test_driver_from_otel_csv(name, tmp_path, monkeypatch):
    """f2 end to end: the window written as the OTel export (collect_data.py:35-46), read back with
    read_traces_csv (Arrow-backed strings), ingested on the device and run through the drop-in
    driver: the reference's stdout, rank lines included."""
    from microrank_amd import online_rca
    from microrank_amd.spans import OTEL_RENAME, read_traces_csv

    case = load_golden(f"{name}.json")
    _, adf = regen_window(case)
    inv = {v: k for k, v in OTEL_RENAME.items()}
    p = tmp_path / "traces.csv"
    adf.rename(columns=inv).to_csv(p, index=False)
    df = read_traces_csv(p)
    slo = {k: [np.float64(float.fromhex(a)), np.float64(float.fromhex(b))] for k, (a, b) in case["slo"].items()}
    monkeypatch.chdir(tmp_path)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        online_rca.online_anomaly_detect_RCA(df, slo, case["operation_list"])
    got, exp = buf.getvalue().splitlines(), case["driver_stdout"].splitlines()
    assert len(got) == len(exp)
    for g, x in zip(got, exp):
        if g.startswith("[") and x.startswith("["):
            gs = [float(v.split("(")[-1].rstrip(")]")) for v in g.split("] [", 1)[1].split(", ")]
            xs = [float(v.split("(")[-1].rstrip(")]")) for v in x.split("] [", 1)[1].split(", ")]
            assert g.split("] [", 1)[0] == x.split("] [", 1)[0]
            np.testing.assert_allclose(gs, xs, rtol=1e-10)
        else:
            assert g == x
