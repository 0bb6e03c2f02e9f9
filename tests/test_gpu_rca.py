"""GPU parity of K3 (spectrum), K4 (SLO), K5 (detector) and the whole driver against the
reference's own outputs (tests/golden).  Spectrum scores, SLO values and the detector's
partition are bit-exact; the driver's stdout is identical except the full-precision repr line
(online_rca.py:202) and result.csv, whose scores are compared at 1e-10 relative."""
import contextlib
import io
import math
import os

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN, load_golden, regen_window, unhex

pytestmark = pytest.mark.gpu
SPAN_CASES = ["c1", "pods_dup_broken", "ops200", "span_times"]


def _spectrum_inputs(case):
    a, n = case["pr_anomaly"], case["pr_normal"]
    a_w = {k: np.float64(v) for k, v in zip(a["keys"], unhex(a["weight"]))}
    n_w = {k: np.float64(v) for k, v in zip(n["keys"], unhex(n["weight"]))}
    return (a_w, n_w, len(case["detect"]["normal"]), len(case["detect"]["abnormal"]),
            dict(zip(n["num_keys"], n["num"])), dict(zip(a["num_keys"], a["num"])))


@pytest.mark.parametrize("name", SPAN_CASES)
def test_spectrum_all_methods(name):
    from microrank_amd.online_rca import calculate_spectrum_without_delay_list as spec

    case = load_golden(f"{name}.json")
    a_w, n_w, A, Nn, n_num, a_num = _spectrum_inputs(case)
    for m, exp in case["spectrum"].items():
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            top, score = spec(anomaly_result=a_w, normal_result=n_w, anomaly_list_len=A, normal_list_len=Nn,
                              top_max=5, normal_num_list=n_num, anomaly_num_list=a_num, spectrum_method=m)
        if "error" in exp:
            pytest.fail(f"reference raised {exp['error']} for {m}")
        assert top == exp["top"], m
        assert [float(s).hex() for s in score] == exp["score"], m
        assert buf.getvalue() == exp["stdout"], m
        assert all(isinstance(s, np.float64) for s in score)


def test_spectrum_python_scalar_edges():
    """Python-float inputs: the reference raises ZeroDivisionError where both operands of a
    division are Python scalars; numpy scalars give inf/nan instead."""
    from microrank_amd.online_rca import calculate_spectrum_without_delay_list as spec

    d = load_golden("dict_cases.json")["spectrum_edges"]
    i = d["input"]
    for m, exp in d["out"].items():
        args = dict(anomaly_result=i["a_w"], normal_result=i["n_w"], anomaly_list_len=i["A"], normal_list_len=i["N"],
                    top_max=5, normal_num_list=i["n_n"], anomaly_num_list=i["a_n"], spectrum_method=m)
        buf = io.StringIO()
        if "error" in exp:
            with pytest.raises(ZeroDivisionError), contextlib.redirect_stdout(buf):
                spec(**args)
            continue
        with contextlib.redirect_stdout(buf):
            top, score = spec(**args)
        assert top == exp["top"], m
        assert [float(s).hex() for s in score] == exp["score"], m
        assert buf.getvalue() == exp["stdout"], m


@pytest.mark.parametrize("name", SPAN_CASES)
def test_slo_bit_exact(name):
    from microrank_amd.anormaly_detector import get_slo
    from microrank_amd.preprocess_data import get_operation_slo, get_service_operation_list

    case = load_golden(f"{name}.json")
    ndf, _ = regen_window(case)
    df = ndf.copy()
    ol = get_service_operation_list(df)
    assert ol == case["operation_list"]
    slo = get_operation_slo(ol, df)
    assert list(slo) == list(case["slo"])
    for k, v in slo.items():
        assert [float(v[0]).hex(), float(v[1]).hex()] == case["slo"][k], k
        assert isinstance(v[0], np.float64)
    slo2 = get_slo(ndf.copy())   # T16: the working form of get_slo
    assert {k: [float(x).hex() for x in v] for k, v in slo2.items()} == case["slo"]


def test_slo_large_ops_bit_exact():
    """Ops of 1..131075 spans around numpy's 8192-element reduction buffer (golden from the
    reference's get_operation_slo)."""
    from microrank_amd import synth
    from microrank_amd.preprocess_data import get_operation_slo, get_service_operation_list

    case = load_golden("slo_large.json")
    df = synth.slo_frame(case["seed"], tuple(case["sizes"]))
    assert synth.frame_digest(df) == case["digest"]
    ol = get_service_operation_list(df)
    assert ol == case["operation_list"]
    slo = get_operation_slo(ol, df)
    assert {k: [float(v[0]).hex(), float(v[1]).hex()] for k, v in slo.items()} == case["slo"]
    assert list(slo) == list(case["slo"])


@pytest.mark.parametrize("name", SPAN_CASES)
def test_detector_partition(name):
    from microrank_amd.anormaly_detector import system_anomaly_detect

    case = load_golden(f"{name}.json")
    _, adf = regen_window(case)
    slo = {k: [np.float64(float.fromhex(a)), np.float64(float.fromhex(b))] for k, (a, b) in case["slo"].items()}
    det = case["detect"]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        flag, ab, no = system_anomaly_detect(adf, start_time=pd.Timestamp(det["start_ns"]),
                                             end_time=pd.Timestamp(det["end_ns"]), slo=slo,
                                             operation_list=case["operation_list"])
    tnames = sorted(adf["traceID"].unique())
    assert ab == [tnames[i] for i in det["abnormal"]]
    assert no == [tnames[i] for i in det["normal"]]
    assert flag == det["flag"]
    assert buf.getvalue() == det["stdout"]


def test_edge_spans_slo_and_detector():
    from microrank_amd.anormaly_detector import system_anomaly_detect
    from microrank_amd.preprocess_data import get_operation_slo, get_service_operation_list

    e = load_golden("edges.json")
    df = pd.read_parquet(os.path.join(GOLDEN, "edges_spans.parquet"))
    sdf = df.copy()
    ol = get_service_operation_list(sdf)
    slo = get_operation_slo(ol[:-1], sdf)
    assert {k: [float(v[0]).hex(), float(v[1]).hex()] for k, v in slo.items()} == e["slo"]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        flag, ab, no = system_anomaly_detect(df, start_time=df.startTime.min(),
                                             end_time=df.startTime.min() + pd.Timedelta(minutes=5), slo=slo,
                                             operation_list=ol)
    assert (flag, ab, no) == (e["detect"]["flag"], e["detect"]["abnormal"], e["detect"]["normal"])
    assert buf.getvalue() == e["detect"]["stdout"]


def test_empty_window_returns_false_and_driver_raises():
    from microrank_amd.anormaly_detector import system_anomaly_detect

    df = pd.read_parquet(os.path.join(GOLDEN, "edges_spans.parquet"))
    t = df.startTime.min() - pd.Timedelta(days=1)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        assert system_anomaly_detect(df, t, t + pd.Timedelta(minutes=5), {}, []) is False
    assert buf.getvalue() == "Error: Current span list is empty \n"
    # T2: every trace outlasts the first 5-minute window -> the detector returns False and the
    # driver's 3-way unpacking raises TypeError, as in the reference
    from microrank_amd.online_rca import online_anomaly_detect_RCA

    long = df.copy()
    long["endTime"] = long["startTime"] + pd.Timedelta(minutes=10)
    with pytest.raises(TypeError), contextlib.redirect_stdout(io.StringIO()):
        online_anomaly_detect_RCA(long, {}, [])


def _run_driver(adf, case, sweep=True, monkeypatch=None):
    """stdout and error type of the drop-in driver (the window sweep on the device, or window by
    window with ``sweep=False``)."""
    from microrank_amd import online_rca

    slo = {k: [np.float64(float.fromhex(a)), np.float64(float.fromhex(b))] for k, (a, b) in case["slo"].items()}
    if not sweep:
        monkeypatch.setattr(online_rca, "_sweep_plan", lambda *a, **k: None)
    buf = io.StringIO()
    err = None
    try:
        with contextlib.redirect_stdout(buf):
            online_rca.online_anomaly_detect_RCA(adf.copy(), slo, case["operation_list"])
    except TypeError as e:
        err = type(e).__name__
    return buf.getvalue(), err


@pytest.mark.parametrize("name", ["c1", "pods_dup_broken", "span_times", "stream", "stream_gap"])
def test_driver_matches_reference(name, tmp_path, monkeypatch):
    """The driver's stdout / result.csv / error against the reference's.  c1 and pods_dup_broken,
    stream and stream_gap (multi-window, one ending in the empty-window TypeError) run as one
    device sweep (mr_detect_sweep + mr_windows_batch); span_times (per-span times) window by window."""
    from microrank_amd import synth

    case = load_golden(f"{name}.json")
    if name.startswith("stream"):
        _, adf = synth.stream_dataframes(**case["params"])
        assert synth.frame_digest(adf) == case["input_digest"]["abnormal"]
    else:
        _, adf = regen_window(case)
    monkeypatch.chdir(tmp_path)
    out, err = _run_driver(adf, case)
    assert err == case.get("driver_error")
    got = out.splitlines()
    exp = case["driver_stdout"].splitlines()
    assert len(got) == len(exp)
    for g, x in zip(got, exp):
        if g.startswith("[") and x.startswith("["):    # print(top_list, score_list): full repr
            gl, xl = g.split("] [", 1), x.split("] [", 1)
            assert gl[0] == xl[0]
            gs = [float(v.split("(")[-1].rstrip(")]")) for v in gl[1].split(", ")]
            xs = [float(v.split("(")[-1].rstrip(")]")) for v in xl[1].split(", ")]
            np.testing.assert_allclose(gs, xs, rtol=1e-10)
        else:
            assert g == x
    if case["result_csv"] is None:
        assert not os.path.exists("result.csv")
        return
    got_csv = open("result.csv").read().splitlines()
    exp_csv = case["result_csv"].splitlines()
    assert len(got_csv) == len(exp_csv)
    for g, x in zip(got_csv, exp_csv):
        gp, xp = g.split(","), x.split(",")
        assert gp[:-1] == xp[:-1]
        if gp[-1] != "confidence":
            assert math.isclose(float(gp[-1]), float(xp[-1]), rel_tol=1e-10)


@pytest.mark.parametrize("name", ["stream", "stream_gap"])
def test_driver_sweep_equals_window_loop(name, tmp_path, monkeypatch):
    """f3: the device sweep prints what the window-by-window driver prints (same windows, same
    counts, same rankings and '%.8f' lines), and writes the same result.csv.  The sweep ranks
    through the window batch's layout-order build, the loop through the drop-in per-window graphs
    (get_pagerank_graph + trace_pagerank): a trace's entries are summed in another order, so the
    full-repr scores (online_rca.py:202) and result.csv's agree to 1e-12, not bit for bit."""
    from microrank_amd import synth

    case = load_golden(f"{name}.json")
    _, adf = synth.stream_dataframes(**case["params"])
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    monkeypatch.chdir(tmp_path / "a")
    out_a, err_a = _run_driver(adf, case)
    monkeypatch.chdir(tmp_path / "b")
    out_b, err_b = _run_driver(adf, case, sweep=False, monkeypatch=monkeypatch)
    assert err_a == err_b
    la, lb = out_a.splitlines(), out_b.splitlines()
    assert len(la) == len(lb)
    for a, b in zip(la, lb):
        if a.startswith("[") and b.startswith("["):   # print(top_list, score_list): full repr
            aa, bb = a.split("] [", 1), b.split("] [", 1)
            assert aa[0] == bb[0]
            xa = [float(v.split("(")[-1].rstrip(")]")) for v in aa[1].split(", ")]
            xb = [float(v.split("(")[-1].rstrip(")]")) for v in bb[1].split(", ")]
            np.testing.assert_allclose(xa, xb, rtol=1e-12, atol=0)
        else:
            assert a == b
    csv_a, csv_b = tmp_path / "a" / "result.csv", tmp_path / "b" / "result.csv"
    assert csv_a.exists() == csv_b.exists()
    if csv_a.exists():
        ra, rb = csv_a.read_text().splitlines(), csv_b.read_text().splitlines()
        assert len(ra) == len(rb)
        for a, b in zip(ra, rb):
            pa_, pb_ = a.split(","), b.split(",")
            assert pa_[:-1] == pb_[:-1]
            if pa_[-1] != "confidence":
                assert math.isclose(float(pa_[-1]), float(pb_[-1]), rel_tol=1e-12)


def test_detect_sweep_counts_equal_per_window_detector():
    """mr_detect_sweep: every 1-minute window start's counts and the per-trace partition equal the
    per-window detector (mr_detect) and the numpy oracle, over a 60-minute stream with a gap."""
    import ctypes as C

    import oracle as orc
    from microrank_amd import _lib, synth
    from microrank_amd._lib import ptr
    from microrank_amd.anormaly_detector import detect_states, slo_arrays
    from microrank_amd.preprocess_data import span_table

    case = load_golden("stream_gap.json")
    _, adf = synth.stream_dataframes(**case["params"])
    slo = {k: [np.float64(float.fromhex(a)), np.float64(float.fromhex(b))] for k, (a, b) in case["slo"].items()}
    ctx = _lib.default_context()
    table, dev = span_table(adf, ctx)
    a3, ok = slo_arrays(table, slo)
    grain, width = 60 * 10**9, 5 * 60 * 10**9
    t_begin = int(table.tstart.min())
    M = -(-(int(table.tend.max()) - t_begin) // grain)
    na, nn, rows = np.zeros(M, np.int32), np.zeros(M, np.int32), np.zeros(M, np.int64)
    state = np.zeros(table.n_traces, np.uint8)
    ctx.check(_lib.load().mr_detect_sweep(ctx.h, dev.h, t_begin, grain, width, M, ptr(a3, C.c_double),
                                          ptr(ok, C.c_uint8), ptr(state, C.c_uint8), ptr(na, C.c_int32),
                                          ptr(nn, C.c_int32), ptr(rows, C.c_int64)), "mr_detect_sweep")
    a3d = {c: float(a3[c]) for c in range(len(a3)) if ok[c]}
    n_empty = 0
    for m in range(M):
        t0 = t_begin + m * grain
        inwin = (table.tstart >= t0) & (table.tend <= t0 + width)
        assert rows[m] == int(inwin.sum()), m
        res = detect_states(adf, pd.Timestamp(t0), pd.Timestamp(t0 + width), slo, ctx=ctx)
        ref = orc.detect(table.trace, table.svcop, table.duration, table.tstart, table.tend, t0, t0 + width, a3d)
        if res is None:
            assert rows[m] == 0 and ref is None
            n_empty += 1
            continue
        st, a_, n_, _ = res
        assert (na[m], nn[m]) == (a_, n_) == (len(ref[1]), len(ref[2])), m
        tw = np.zeros(table.n_traces, bool)
        tw[table.trace[inwin]] = True
        assert np.array_equal(np.where(tw, state, 0), st), m   # the window's partition is the global one
    assert n_empty > 0 and (na > 0).any()


@pytest.mark.parametrize("name", ["c1", "pods_dup_broken", "ops200", "span_times"])
def test_rca_window_device_pipeline(name):
    """mr_rca_window (all intermediates in HBM) ranks like the reference driver's window."""
    from microrank_amd.online_rca import rca_window

    case = load_golden(f"{name}.json")
    _, adf = regen_window(case)
    slo = {k: [np.float64(float.fromhex(a)), np.float64(float.fromhex(b))] for k, (a, b) in case["slo"].items()}
    det = case["detect"]
    out = rca_window(adf, pd.Timestamp(det["start_ns"]), pd.Timestamp(det["end_ns"]), slo)
    exp = case["spectrum"]["dstar2"]
    assert out["n_abnormal"] == len(det["abnormal"]) and out["n_normal"] == len(det["normal"])
    assert out["top"] == exp["top"]
    np.testing.assert_allclose(out["score"], unhex(exp["score"]), rtol=1e-10)
    out32 = rca_window(adf, pd.Timestamp(det["start_ns"]), pd.Timestamp(det["end_ns"]), slo, precision="fp32")
    assert out32["top"][:5] == exp["top"][:5]
    np.testing.assert_allclose(out32["score"], unhex(exp["score"]), rtol=1e-4)


def test_slo_bench_scale_matches_oracle():
    """K4 on the bench's normal period (1k ops, ~1.4M spans, hot ops of >8192 spans) against the
    oracle's np.std restatement: bit-exact."""
    import ctypes as C

    import bench
    import oracle as orc
    from microrank_amd import _lib
    from microrank_amd._lib import ptr
    from microrank_amd.preprocess_data import DeviceSpans

    _, normal, _ = bench.make_window(1234, 1000, 100_000)
    ctx = _lib.default_context()
    dev = DeviceSpans(ctx, normal)
    n = normal.n_svcops
    mean, std, cnt = np.empty(n), np.empty(n), np.empty(n, np.int64)
    ctx.check(_lib.load().mr_slo(ctx.h, dev.h, ptr(mean, C.c_double), ptr(std, C.c_double), ptr(cnt, C.c_int64)))
    dev.close()
    assert cnt.max() > 8192
    names = [str(i) for i in range(n)]
    exp = orc.operation_slo(normal.svcop, normal.duration, names, names)
    for code in range(n):
        if cnt[code] == 0:
            assert str(code) not in exp
            continue
        e = exp[str(code)]
        assert (mean[code], std[code]) == (float(e[0]), float(e[1])), code


def test_concurrent_contexts_rank_like_one():
    """bench.py's --streams: four contexts (streams) ranking copies of one window from four host
    threads at once give bitwise the same top list, scores and edge counts as one context alone,
    and the oracle's C restatement ranks the same top list."""
    from concurrent.futures import ThreadPoolExecutor

    import bench
    import c_oracle
    from microrank_amd import _lib
    from microrank_amd.preprocess_data import DeviceSpans

    _, normal, abnormal = bench.make_window(1234, 300, 30_000)
    t0 = int(abnormal.tstart.min())
    t1 = t0 + 5 * 60 * 10**9
    ctxs = [_lib.Context(0) for _ in range(4)]
    wins = []
    for cx in ctxs:
        a3, ok = bench.slo_from_gpu(cx, normal)
        wins.append((cx, DeviceSpans(cx, abnormal), a3, ok))
    ref = bench.run_window(wins[0][0], wins[0][1], t0, t1, wins[0][2], wins[0][3], _lib.MR_FP64)

    def go(w):
        return [bench.run_window(w[0], w[1], t0, t1, w[2], w[3], _lib.MR_FP64) for _ in range(3)]

    with ThreadPoolExecutor(max_workers=4) as ex:
        outs = list(ex.map(go, wins))
    for o in outs:
        for e, top, scores, na, nn in o:
            assert (e, na, nn) == (ref[0], ref[3], ref[4])
            assert list(top) == list(ref[1])
            assert scores.tobytes() == ref[2].tobytes()
    cres = c_oracle.rca_window(abnormal, t0, t1, wins[0][2], wins[0][3], nthreads=4)
    assert list(cres[0]) == list(ref[1])
    for w in wins:
        w[1].close()
    for cx in ctxs:
        cx.close()


def _oracle_rca(st, t0, t1, a3, ok, top_max=5):
    """The driver's window (online_rca.py:164-201) on the numpy oracle: detector (T1 swap), the
    two span graphs (preprocess_data.py:146-171), both PageRanks (pagerank.py:15-112), DStar2."""
    import oracle as orc

    a3map = {i: float(a3[i]) for i in range(len(a3)) if ok[i]}
    _, ab, no = orc.detect(st.trace, st.svcop, st.duration, st.tstart, st.tend, t0, t1, a3map)
    res = {}
    for lst, anomaly in ((ab, False), (no, True)):   # normal_list = the detector's abnormal traces
        sel = np.zeros(st.n_traces, bool)
        sel[lst] = True
        g = orc.span_graph(st.trace, st.podop, st.span, st.parent, sel).as_graph()
        s = orc.power_iteration(g, orc.preference(g, orc.trace_kinds(g), anomaly))
        res[anomaly] = orc.weights(g, s)
    top, score, _ = orc.spectrum(res[True][0], res[False][0], len(no), len(ab), top_max, res[False][1], res[True][1],
                                 "dstar2")
    return top, score, len(ab), len(no)


@pytest.fixture(scope="module")
def c3_window():
    import bench

    _, normal, abnormal = bench.make_window(4242, 500, 20_000)   # BASELINE configs[2]: 500 ops / 20k traces
    t0 = int(abnormal.tstart.min())
    return normal, abnormal, t0, t0 + 5 * 60 * 10**9


def test_c3_window_against_oracle(c3_window):
    """C3-shaped window (500 ops / 20k traces): mr_rca_window's top-11 and DStar2 scores against
    the numpy oracle's whole window at 1e-10 (fp64), the top-5 and 1e-4 in fp32."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.preprocess_data import DeviceSpans

    normal, abnormal, t0, t1 = c3_window
    ctx = _lib.default_context()
    a3, ok = bench.slo_from_gpu(ctx, normal)
    dev = DeviceSpans(ctx, abnormal)
    top, score, na, nn = _oracle_rca(abnormal, t0, t1, a3, ok)
    assert na > 0 and nn > 0 and len(top) == 11
    e, codes, scores, gna, gnn = bench.run_window(ctx, dev, t0, t1, a3, ok, _lib.MR_FP64)
    assert (gna, gnn) == (na, nn)
    assert list(codes) == list(top)
    np.testing.assert_allclose(scores, score, rtol=1e-10, atol=0)
    e32, c32, s32, _, _ = bench.run_window(ctx, dev, t0, t1, a3, ok, _lib.MR_FP32)
    assert list(c32[:5]) == list(top[:5])
    np.testing.assert_allclose(s32, score, rtol=1e-4, atol=0)
    dev.close()


def test_windows_batch_matches_standalone(c3_window):
    """mr_windows_batch: four C3-shaped windows (three distinct span tables, one of them twice)
    plus an empty window in one call -- every window's top list equals its standalone
    mr_rca_window run, scores within 1e-12 (the batch shares the PageRank launches: only the
    fixed-point scale of a block may differ), the empty window flagged MR_ERR_VALUE."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    ctx = _lib.default_context()
    wins = []
    normal, abnormal, t0, t1 = c3_window
    a3, ok = bench.slo_from_gpu(ctx, normal)
    dev0 = DeviceSpans(ctx, abnormal)
    wins.append((dev0, t0, t1, a3, ok))
    devs = [dev0]
    for seed in (77, 78):
        _, nrm, ab = bench.make_window(seed, 500, 20_000)
        s3, sok = bench.slo_from_gpu(ctx, nrm)
        d = DeviceSpans(ctx, ab)
        devs.append(d)
        u0 = int(ab.tstart.min())
        wins.append((d, u0, u0 + 5 * 60 * 10**9, s3, sok))
    wins.append(wins[0])
    wins.append((dev0, 0, 1, a3, ok))   # no trace in [0, 1] ns: empty window
    got = rank_windows(ctx, wins)
    for w, (codes, scores, na, nn, edges, status) in zip(wins[:4], got[:4]):
        assert status == 0
        e, c1, s1, na1, nn1 = bench.run_window(ctx, w[0], w[1], w[2], w[3], w[4], _lib.MR_FP64)
        assert (na, nn, edges) == (na1, nn1, e)
        assert list(codes) == list(c1)
        np.testing.assert_allclose(scores, s1, rtol=1e-12, atol=0)
    assert got[0][0].tolist() == got[3][0].tolist() and got[0][1].tobytes() == got[3][1].tobytes()
    assert got[4][5] == _lib.MR_ERR_VALUE
    for d in devs:
        d.close()


def test_window_spectrum_one_block_equals_general_path(monkeypatch):
    """k_win_spectrum (the window's union, scores, bitonic sort -- lane-exchange stages below
    stride 64 -- and top k in one block) against the general multi-launch spectrum path
    (MR_NO_WIN_SPECTRUM_SMALL), on windows of 40 to 2500 ops (unions from a few nodes to > 2048:
    one to four elements per thread) with top lists of 256: codes and scores bitwise equal."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    ctx = _lib.default_context()
    wins, devs = [], []
    for seed, ops in ((501, 40), (502, 300), (503, 700), (504, 1500), (505, 2500)):
        _, nrm, ab = bench.make_window(seed, ops, 12_000)
        s3, sok = bench.slo_from_gpu(ctx, nrm)
        d = DeviceSpans(ctx, ab)
        devs.append(d)
        u0 = int(ab.tstart.min())
        wins.append((d, u0, u0 + 5 * 60 * 10**9, s3, sok))
    runs = {}
    for mode in ("one_block", "general"):
        monkeypatch.delenv("MR_NO_WIN_SPECTRUM_SMALL", raising=False)
        if mode == "general":
            monkeypatch.setenv("MR_NO_WIN_SPECTRUM_SMALL", "1")
        runs[mode] = rank_windows(ctx, wins, top_max=250)
    lens = []
    for a, b in zip(runs["one_block"], runs["general"]):
        assert a[5] == b[5] == 0
        assert list(a[0]) == list(b[0]) and a[1].tobytes() == b[1].tobytes()
        lens.append(len(a[0]))
    assert max(lens) == 256 and min(lens) < 256   # (a window with fewer nodes than k)
    for d in devs:
        d.close()


def test_windows_batch_fx_ops_per_block_bitwise(c3_window, monkeypatch):
    """k_fx_b's ops per block (16 for few graphs, 64 for batches of many: MR_FB_OPS forces either)
    only regroups the integer limb sums and the per-op call-graph terms: a 4-window batch ranks
    bitwise the same with 16, 32 and 64."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    ctx = _lib.default_context()
    normal, abnormal, t0, t1 = c3_window
    a3, ok = bench.slo_from_gpu(ctx, normal)
    devs = [DeviceSpans(ctx, abnormal)]
    wins = [(devs[0], t0, t1, a3, ok)]
    for seed in (71, 72, 73):
        _, nrm, ab = bench.make_window(seed, 500, 20_000)
        s3, sok = bench.slo_from_gpu(ctx, nrm)
        d = DeviceSpans(ctx, ab)
        devs.append(d)
        u0 = int(ab.tstart.min())
        wins.append((d, u0, u0 + 5 * 60 * 10**9, s3, sok))
    runs = {}
    monkeypatch.setenv("MR_TR_LASTFIN", "0")   # (k_fx_b for every graph: the path under test)
    for v in ("16", "32", "64"):
        monkeypatch.setenv("MR_FB_OPS", v)
        runs[v] = rank_windows(ctx, wins, top_max=60)
    for v in ("32", "64"):
        for a, b in zip(runs["16"], runs[v]):
            assert a[5] == b[5] == 0
            assert a[2:] == b[2:] and list(a[0]) == list(b[0]) and a[1].tobytes() == b[1].tobytes(), v
    for d in devs:
        d.close()


def test_windows_batch_last_block_finish_bitwise(c3_window, monkeypatch):
    """k_tr_a's last block of a graph finishing the iteration itself (window graphs: one launch per
    iteration, MR_TR_LASTFIN) against the k_tr_a + k_fx_b pair: the same integer limb sums and
    call-graph terms, so a 4-window batch ranks bitwise the same; one window alone too."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    ctx = _lib.default_context()
    normal, abnormal, t0, t1 = c3_window
    a3, ok = bench.slo_from_gpu(ctx, normal)
    devs = [DeviceSpans(ctx, abnormal)]
    wins = [(devs[0], t0, t1, a3, ok)]
    for seed in (81, 82, 83):
        _, nrm, ab = bench.make_window(seed, 500, 20_000)
        s3, sok = bench.slo_from_gpu(ctx, nrm)
        d = DeviceSpans(ctx, ab)
        devs.append(d)
        u0 = int(ab.tstart.min())
        wins.append((d, u0, u0 + 5 * 60 * 10**9, s3, sok))
    runs = {}
    for v in ("0", "1"):
        monkeypatch.setenv("MR_TR_LASTFIN", v)
        runs[v] = (rank_windows(ctx, wins, top_max=60), rank_windows(ctx, wins[:1], top_max=60))
    for many_a, many_b in zip(runs["0"], runs["1"]):
        for a, b in zip(many_a, many_b):
            assert a[5] == b[5] == 0
            assert a[2:] == b[2:] and list(a[0]) == list(b[0]) and a[1].tobytes() == b[1].tobytes()
    for d in devs:
        d.close()


def test_windows_batch_fast_paths_equal_general_paths(c3_window, monkeypatch):
    """The window batch's fast paths -- the detector fused into the index pass's first launch
    (k_ix_detect_scan2), both graphs built in one index pass (mr_ix_launch2) with dense edge ids,
    windows built in chunks and prepared together (mr_graph_prepare_batch), set up in batched
    launches over the group (pagerank_setup_batch) or over the chunk (mr_pagerank_presetup_n) --
    give the same rankings as the one-graph-at-a-time paths (MR_NO_IX2 / MR_EDGE_HASH /
    MR_NO_PREP_BATCH / MR_NO_SETUP_BATCH): top lists identical, scores within 1e-12, counts and
    edges equal; the separate detector launch (MR_NO_DET_FUSE) and one-window chunks
    (MR_WIN_CHUNK=1) give bitwise the same results."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    ctx = _lib.default_context()
    normal, abnormal, t0, t1 = c3_window
    a3, ok = bench.slo_from_gpu(ctx, normal)
    devs = [DeviceSpans(ctx, abnormal)]
    wins = [(devs[0], t0, t1, a3, ok)]
    for seed in (91, 92, 93):
        _, nrm, ab = bench.make_window(seed, 500, 20_000)
        s3, sok = bench.slo_from_gpu(ctx, nrm)
        d = DeviceSpans(ctx, ab)
        devs.append(d)
        u0 = int(ab.tstart.min())
        wins.append((d, u0, u0 + 5 * 60 * 10**9, s3, sok))
    runs = {}
    knobs = ("MR_NO_IX2", "MR_EDGE_HASH", "MR_NO_PREP_BATCH", "MR_NO_SETUP_BATCH", "MR_WIN_SETUP_SPLIT",
             "MR_NO_DET_FUSE", "MR_WIN_CHUNK")
    for mode in ("fast", "split0", "general", "nofuse_chunk1"):
        for k in knobs:
            monkeypatch.delenv(k, raising=False)
        if mode == "split0":   # every chunk sets its graphs up on its own stream (presetup_n)
            monkeypatch.setenv("MR_WIN_SETUP_SPLIT", "0")
        if mode == "nofuse_chunk1":
            monkeypatch.setenv("MR_NO_DET_FUSE", "1")
            monkeypatch.setenv("MR_WIN_CHUNK", "1")
        if mode == "general":
            for k in ("MR_NO_IX2", "MR_EDGE_HASH", "MR_NO_PREP_BATCH", "MR_NO_SETUP_BATCH"):
                monkeypatch.setenv(k, "1")
        runs[mode] = rank_windows(ctx, wins)
    for mode in ("split0", "general"):
        for a, b in zip(runs["fast"], runs[mode]):
            assert a[5] == b[5] == 0
            assert (a[2], a[3], a[4]) == (b[2], b[3], b[4]), mode
            assert list(a[0]) == list(b[0]), mode
            np.testing.assert_allclose(a[1], b[1], rtol=1e-12, atol=0)
    for a, b in zip(runs["fast"], runs["nofuse_chunk1"]):
        assert a[2:] == b[2:] and list(a[0]) == list(b[0]) and a[1].tobytes() == b[1].tobytes()
    for d in devs:
        d.close()


@pytest.mark.parametrize("name,minutes,device_append", [("stream", 7, True), ("stream", 3, True),
                                                         ("stream_gap", 7, True), ("stream", 7, False),
                                                         ("stream_gap", 3, False)])
def test_rca_stream_matches_offline_driver(name, minutes, device_append, tmp_path, monkeypatch):
    """f3 online (RCAStream): the reference-captured 60-minute streams pushed in trace-aligned
    chunks of a few minutes print what the reference's offline driver printed over the whole frame
    (and write its result.csv, and raise its empty-window TypeError) -- with the resident table grown
    on the device (mr_spans_append) and with the host concat + re-ingest."""
    from microrank_amd import synth
    from microrank_amd.online_rca import RCAStream

    case = load_golden(f"{name}.json")
    _, adf = synth.stream_dataframes(**case["params"])
    slo = {k: [np.float64(float.fromhex(a)), np.float64(float.fromhex(b))] for k, (a, b) in case["slo"].items()}
    monkeypatch.chdir(tmp_path)
    t0 = adf["startTime"].min()
    bucket = ((adf["startTime"] - t0) // pd.Timedelta(minutes=minutes)).to_numpy()
    assert (np.diff(bucket) >= 0).all()   # rows in trace-start order: chunks keep the frame's order
    buf = io.StringIO()
    err = None
    try:
        with contextlib.redirect_stdout(buf):
            s = RCAStream(slo, case["operation_list"], device_append=device_append)
            for b in np.unique(bucket):
                s.push(adf[bucket == b].copy())
            s.close()
    except TypeError as e:
        err = type(e).__name__
    assert err == case["driver_error"]
    got, exp = buf.getvalue().splitlines(), case["driver_stdout"].splitlines()
    assert len(got) == len(exp)
    for g, x in zip(got, exp):
        if g.startswith("[") and x.startswith("["):
            gl, xl = g.split("] [", 1), x.split("] [", 1)
            assert gl[0] == xl[0]
            gs = [float(v.split("(")[-1].rstrip(")]")) for v in gl[1].split(", ")]
            xs = [float(v.split("(")[-1].rstrip(")]")) for v in xl[1].split(", ")]
            np.testing.assert_allclose(gs, xs, rtol=1e-10)
        else:
            assert g == x
    if case["result_csv"] is not None:
        got_csv = open("result.csv").read().splitlines()
        assert [r.split(",")[:-1] for r in got_csv] == [r.split(",")[:-1] for r in case["result_csv"].splitlines()]


def test_span_append_equals_ingest_of_concatenation():
    """mr_spans_append: the table grown chunk by chunk (with resident rows retired by trace start)
    is the table mr_spans_ingest builds from the concatenated, filtered frame -- same size,
    dictionaries (names in code order), code columns bit for bit, and the same detector / graph
    results; prev stays usable; a foreign prev is refused."""
    from microrank_amd import _lib, synth
    from microrank_amd.preprocess_data import SpanStream, span_table

    _, adf = synth.stream_dataframes(24, 1200, 5, minutes=30.0)
    ctx = _lib.default_context()
    t0 = adf["startTime"].min()
    bucket = ((adf["startTime"] - t0) // pd.Timedelta(minutes=4)).to_numpy()
    st = SpanStream(ctx)
    resident = None
    cuts = [t0 + pd.Timedelta(minutes=m) for m in (0, 0, 3, 9, 9, 15, 22, 22)]
    for i, b in enumerate(np.unique(bucket)):
        chunk = adf[bucket == b].copy()
        cut = cuts[min(i, len(cuts) - 1)]
        prev_dev = st.dev
        table, dev = st.append(chunk, int(cut.value))
        if resident is not None:
            resident = resident[resident["startTime"] >= cut]
        resident = chunk if resident is None else pd.concat([resident, chunk], ignore_index=True)
        resident = resident.reset_index(drop=True)
        ref_table, _ = span_table(resident.copy(), ctx)
        assert (table.n_spans, table.n_traces, table.n_podops, table.n_svcops) == \
            (ref_table.n_spans, ref_table.n_traces, ref_table.n_podops, ref_table.n_svcops)
        assert table.trace_names == ref_table.trace_names
        assert table.podop_names == ref_table.podop_names
        assert table.svcop_names == ref_table.svcop_names
        for a, b_ in zip(table._code_cols(), ref_table._code_cols()):
            assert np.array_equal(a, b_)
        assert prev_dev is None or prev_dev.h is None   # the previous handle was released
    # a table that was not appended cannot be the previous one
    ref_table, ref_dev = span_table(adf.copy(), ctx)
    from microrank_amd.preprocess_data import span_strings
    from microrank_amd.spans import arrow_columns
    import ctypes as C
    ss, _keep, *_ = span_strings(adf, arrow_columns(adf))
    h = _lib.P()
    rc = _lib.load().mr_spans_append(ctx.h, ref_dev.h, 0, C.byref(ss), C.byref(h))
    assert rc == _lib.MR_ERR_STATE
    st.close()


def test_c3_window_matches_reference_golden():
    """One C3-sized window (BASELINE configs[2]: 500 ops / 20k traces, 471k spans) against the
    REFERENCE's own outputs (tests/golden/c3_window.json, make_golden.py c3_window: 835 s of
    reference trace_pagerank): SLO bit-exact, the detector's lists identical, both swapped graphs'
    node order and weights (1e-10) and coverage, the DStar2 top-11 identical with scores at 1e-10 --
    through the drop-in functions the unchanged driver calls (online_rca.py:167-201), and the
    device window pipeline (mr_rca_window) giving the same top list."""
    from microrank_amd import synth
    from microrank_amd.anormaly_detector import system_anomaly_detect
    from microrank_amd.online_rca import calculate_spectrum_without_delay_list, rca_window
    from microrank_amd.pagerank import trace_pagerank
    from microrank_amd.preprocess_data import (get_operation_slo, get_pagerank_graph,
                                               get_service_operation_list)

    case = load_golden("c3_window.json")
    p = dict(case["params"])
    ndf, adf = synth.window_dataframes(p.pop("n_ops"), p.pop("n_traces"), p.pop("seed"), **p)
    assert synth.frame_digest(ndf) == case["input_digest"]["normal"]
    assert synth.frame_digest(adf) == case["input_digest"]["abnormal"]
    span_df = ndf.copy()
    op_list = get_service_operation_list(span_df)
    assert op_list == case["operation_list"]
    slo = get_operation_slo(op_list, span_df)
    assert {k: [v[0].hex(), v[1].hex()] for k, v in slo.items()} == case["slo"]
    det = case["detect"]
    start, end = pd.Timestamp(det["start_ns"]), pd.Timestamp(det["end_ns"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        flag, abn, nor = system_anomaly_detect(adf, start_time=start, end_time=end, slo=slo, operation_list=op_list)
    assert buf.getvalue() == det["stdout"] and flag == det["flag"]
    tn = sorted(adf["traceID"].unique())
    assert abn == [tn[i] for i in det["abnormal"]] and nor == [tn[i] for i in det["normal"]]
    w_n, c_n = trace_pagerank(*get_pagerank_graph(abn, adf), False)   # T1: the driver's swap
    w_a, c_a = trace_pagerank(*get_pagerank_graph(nor, adf), True)
    for got_w, got_c, key, nodes in ((w_n, c_n, "pr_normal", "nodes_normal"), (w_a, c_a, "pr_anomaly", "nodes_anomaly")):
        exp = case[key]
        assert list(got_w) == exp["keys"] == case[nodes] and list(got_c) == exp["num_keys"]
        assert [int(v) for v in got_c.values()] == exp["num"]
        np.testing.assert_allclose(np.array(list(got_w.values())), unhex(exp["weight"]), rtol=1e-10, atol=0)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        top, score = calculate_spectrum_without_delay_list(
            anomaly_result=w_a, normal_result=w_n, anomaly_list_len=len(nor), normal_list_len=len(abn), top_max=5,
            normal_num_list=c_n, anomaly_num_list=c_a, spectrum_method="dstar2")
    sp = case["spectrum_dstar2"]
    assert list(top) == sp["top"]
    np.testing.assert_allclose(np.array(score, dtype=np.float64), unhex(sp["score"]), rtol=1e-10, atol=0)
    got_lines, exp_lines = buf.getvalue().splitlines(), sp["stdout"].splitlines()
    assert [ln.split(":")[0] for ln in got_lines] == [ln.split(":")[0] for ln in exp_lines]
    res = rca_window(adf, start, end, slo)
    assert res["top"] == sp["top"] and (res["n_abnormal"], res["n_normal"]) == (len(abn), len(nor))
    np.testing.assert_allclose(np.array(res["score"], dtype=np.float64), unhex(sp["score"]), rtol=1e-10, atol=0)


def test_windows_batch_reaper_and_context_destroy(c3_window, monkeypatch):
    """large windows' graphs are held by the context and released by its NEXT
    mr_windows_batch call (MR_WIN_REAP): two calls on one context with the reaper forced on give
    bitwise the results of calls with it off; a context destroyed while it still holds such graphs
    frees them, and a stale handle freed afterwards is a no-op."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    normal, abnormal, t0, t1 = c3_window
    runs = {}
    for reap in ("0", "1"):
        monkeypatch.setenv("MR_WIN_REAP", reap)
        cx = _lib.Context(0)
        a3, ok = bench.slo_from_gpu(cx, normal)
        dev = DeviceSpans(cx, abnormal)
        wins = [(dev, t0, t1, a3, ok)] * 3
        first = rank_windows(cx, wins)
        second = rank_windows(cx, wins)    # reap=1: releases the first call's graphs meanwhile
        runs[reap] = (first, second)
        h = dev.h
        cx.close()                         # reap=1: the second call's graphs are still held
        assert _lib.load().mr_spans_free(h) == 0
        dev.close()
    for a, b in zip(runs["0"][0] + runs["0"][1], runs["1"][0] + runs["1"][1]):
        assert a[2:] == b[2:] and list(a[0]) == list(b[0]) and a[1].tobytes() == b[1].tobytes()


# ---------------------------------------------------------------- the headline's own shape (C2 windows)
C2_WINDOWS = 8


@pytest.fixture(scope="module")
def c2_batch():
    """BASELINE configs[1] windows exactly as bench.py's default line builds them: 8 distinct
    1k-op / 200k-trace windows of one system (own seed and span table each) and the SLO of its
    normal period, resident on the device."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.preprocess_data import DeviceSpans

    normal, tabs = bench.c2_windows(C2_WINDOWS, 1000, 200_000, rank=3)
    ctx = _lib.default_context()
    a3, ok = bench.slo_from_gpu(ctx, normal)
    wins, devs = [], []
    for st in tabs:
        d = DeviceSpans(ctx, st)
        devs.append(d)
        t0 = int(st.tstart.min())
        wins.append((d, t0, t0 + 5 * 60 * 10**9, a3, ok))
    yield ctx, tabs, wins
    for d in devs:
        d.close()


def test_c2_windows_batch_against_oracle(c2_batch, monkeypatch):
    """bench.py's default line (online_rca.py:164-201 per window) at its own size: 8 distinct C2
    windows (1k ops / 200k traces, ~2.3M index entries each) through ONE mr_windows_batch call with
    the default grouping -- one PageRank group of all 8 windows (256 graphs per launch in the bench:
    the same grouped k_tr_a / k_fx_b launches), chunks of 4 windows (> 65536 traces per window), the
    batched stats pass at 64 entries per thread (>= 1M index entries) and the separate detector
    launch (tables above the 65536-trace fuse limit).  Every window's top-11, DStar2 scores and
    (abnormal, normal, edges) against the C restatement (oracle/mr_oracle.c, pinned to the
    reference's goldens) at 1e-10 in fp64; top-5 at 1e-4 in fp32."""
    import c_oracle
    from microrank_amd.online_rca import rank_windows

    for k in ("MR_WIN_GROUP", "MR_WIN_CHUNK", "MR_IX_EPT", "MR_DET_FUSE_MAX", "MR_NO_DET_FUSE"):
        monkeypatch.delenv(k, raising=False)
    ctx, tabs, wins = c2_batch
    for st in tabs:   # the branches under test are the ones this shape selects
        assert st.n_traces > 65536
        pairs = np.unique(st.trace.astype(np.int64) * st.n_podops + st.podop).size
        assert pairs >= 1 << 20
    got = rank_windows(ctx, wins)
    got32 = rank_windows(ctx, wins, precision="fp32")
    for i, (st, w) in enumerate(zip(tabs, wins)):
        codes, scores, na, nn, edges, status = got[i]
        assert status == 0, i
        ref = c_oracle.rca_window(st, w[1], w[2], w[3], w[4], nthreads=0)
        rc, rs, rna, rnn, redges = ref
        assert (na, nn) == (rna, rnn), i
        assert na > 0 and nn > 0 and len(rc) == 11
        assert edges == redges, i
        assert list(codes) == list(rc), i
        np.testing.assert_allclose(scores, rs, rtol=1e-10, atol=0, err_msg=f"window {i}")
        c32, s32, _, _, e32, st32 = got32[i]
        assert st32 == 0 and e32 == edges
        assert list(c32[:5]) == list(rc[:5]), i
        np.testing.assert_allclose(s32, rs, rtol=1e-4, atol=0, err_msg=f"window {i} fp32")


def test_c2_windows_batch_groupings_agree(c2_batch, monkeypatch):
    """The same 8 C2 windows under other batch shapes: chunks of 1 and 2 windows, the stats pass
    at 16 entries per thread and the detector fused into the index pass (MR_DET_FUSE_MAX above the
    table) rank bitwise as the default -- build-side choices, the PageRank launches untouched; and
    PageRank groups of 4 and 2 windows (MR_WIN_GROUP) rank bitwise too: a group's block budget
    changes how a graph's tiles are cut into blocks, but the fixed-point scale of X_t is one
    cut-independent constant (tr_scfix), so the exact limb sums -- and a window's scores -- do not depend on the batch.
    k_fx_b every iteration (MR_TR_PF=0) instead of the next k_tr_a launch finishing the iteration in
    its prologue ranks bitwise as the default: the same limb sums and expressions.  The run-merged walk (MR_TR_MERGE=1: a run of
    identical traces shares one id rotation and its head walks for it with X times the run length;
    the bench's side leg, never the headline) ranks bitwise as every lane walking its own trace in
    the same run rotations (MR_TR_MERGE=2): the merge is exact; against the default (a rotation per
    trace: each trace's sum in another order) the scores agree to 1e-12."""
    from microrank_amd.online_rca import rank_windows

    knobs = ("MR_WIN_GROUP", "MR_WIN_CHUNK", "MR_IX_EPT", "MR_DET_FUSE_MAX", "MR_NO_DET_FUSE", "MR_TR_MERGE", "MR_TR_PF")
    ctx, _, wins = c2_batch
    variants = {"default": {}, "chunk1_ept16": {"MR_WIN_CHUNK": "1", "MR_IX_EPT": "16"},
                "chunk2_fused": {"MR_WIN_CHUNK": "2", "MR_DET_FUSE_MAX": "100000000"},
                "merge": {"MR_TR_MERGE": "1"}, "runrot": {"MR_TR_MERGE": "2"}, "nopf": {"MR_TR_PF": "0"},
                "group4_chunk4": {"MR_WIN_GROUP": "4", "MR_WIN_CHUNK": "4"}, "group2": {"MR_WIN_GROUP": "2"}}
    runs = {}
    for name, env in variants.items():
        for k in knobs:
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        runs[name] = rank_windows(ctx, wins)
    base = runs["default"]
    for name, got in runs.items():
        for i, (a, b) in enumerate(zip(base, got)):
            assert a[5] == b[5] == 0, (name, i)
            assert a[2:] == b[2:] and list(a[0]) == list(b[0]), (name, i)
            if name in ("merge", "runrot"):
                np.testing.assert_allclose(b[1], a[1], rtol=1e-12, atol=0, err_msg=f"{name} window {i}")
            else:
                assert a[1].tobytes() == b[1].tobytes(), (name, i)
    for i, (a, b) in enumerate(zip(runs["merge"], runs["runrot"])):
        assert a[1].tobytes() == b[1].tobytes() and list(a[0]) == list(b[0]), ("merge == runrot", i)


def test_windows_batch_layout_order_equals_general_build(c3_window, monkeypatch):
    """The layout-order window build (tables indexed with their trace layout and exact kind
    classes: k_lo_sel_b, k_lo_fill_b, ...) against the general per-window build (MR_NO_LO_WIN):
    four C3-shaped windows of three tables and an empty window -- statuses, abnormal / normal
    counts and edges equal, top lists identical, DStar2 scores within 1e-12 (a tile's traces sum in
    another rotation); and one-window chunks (the layout-order launches with n = 1) bitwise equal
    to the default chunks of eight."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    ctx = _lib.default_context()
    normal, abnormal, t0, t1 = c3_window
    a3, ok = bench.slo_from_gpu(ctx, normal)
    devs = [DeviceSpans(ctx, abnormal)]
    wins = [(devs[0], t0, t1, a3, ok)]
    for seed in (61, 62):
        _, nrm, ab = bench.make_window(seed, 500, 20_000)
        s3, sok = bench.slo_from_gpu(ctx, nrm)
        d = DeviceSpans(ctx, ab)
        devs.append(d)
        u0 = int(ab.tstart.min())
        wins.append((d, u0, u0 + 5 * 60 * 10**9, s3, sok))
    wins.append((devs[0], 0, 1, a3, ok))   # empty window
    runs = {}
    for mode in ("lo", "general", "lo_chunk1"):
        for k in ("MR_NO_LO_WIN", "MR_WIN_CHUNK"):
            monkeypatch.delenv(k, raising=False)
        if mode == "general":
            monkeypatch.setenv("MR_NO_LO_WIN", "1")
        if mode == "lo_chunk1":
            monkeypatch.setenv("MR_WIN_CHUNK", "1")
        runs[mode] = rank_windows(ctx, wins)
    for a, b in zip(runs["lo"], runs["general"]):
        assert a[5] == b[5]
        assert a[2:] == b[2:] and list(a[0]) == list(b[0])
        np.testing.assert_allclose(a[1], b[1], rtol=1e-12, atol=0)
    assert runs["lo"][3][5] == _lib.MR_ERR_VALUE
    for a, b in zip(runs["lo"], runs["lo_chunk1"]):
        assert a[2:] == b[2:] and list(a[0]) == list(b[0]) and a[1].tobytes() == b[1].tobytes()
    for d in devs:
        d.close()


def test_layout_index_failure_keeps_general_path(c3_window, monkeypatch):
    """The layout order is a best-effort fast path of the span index: a failure inside it
    (MR_LO_TEST_FAIL: an error after an allocation, read per table) leaves the upload successful,
    the context's error text clear, and the table on the general window build -- the window ranks
    as on a table indexed with its layout (top list, counts and edges equal, scores 1e-12)."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    ctx = _lib.default_context()
    normal, abnormal, t0, t1 = c3_window
    a3, ok = bench.slo_from_gpu(ctx, normal)
    good = DeviceSpans(ctx, abnormal)
    monkeypatch.setenv("MR_LO_TEST_FAIL", "1")
    bad = DeviceSpans(ctx, abnormal)
    monkeypatch.delenv("MR_LO_TEST_FAIL")
    assert (_lib.load().mr_last_error(ctx.h) or b"") == b""
    a, b = rank_windows(ctx, [(good, t0, t1, a3, ok), (bad, t0, t1, a3, ok)])
    assert a[5] == b[5] == 0
    assert a[2:] == b[2:] and list(a[0]) == list(b[0])
    np.testing.assert_allclose(b[1], a[1], rtol=1e-12, atol=0)
    good.close()
    bad.close()


def test_windows_batch_layout_order_rerun_sets_up_again(c3_window, monkeypatch):
    """A PageRank group that mixes layout-order graphs with general-build ones (a table uploaded
    without its layout: MR_NO_LO) and whose kind hashing collides (MR_KIND_TEST_COLLIDE) reruns
    the whole group: the layout-order graphs' set-up runs again from their kept class sizes and
    span counts (lo_setup_one), and every window ranks bitwise as without the collision; the
    same window on either table ranks alike (1e-12)."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    ctx = _lib.default_context()
    normal, abnormal, t0, t1 = c3_window
    a3, ok = bench.slo_from_gpu(ctx, normal)
    d_lo = DeviceSpans(ctx, abnormal)
    monkeypatch.setenv("MR_NO_LO", "1")
    d_gen = DeviceSpans(ctx, abnormal)
    monkeypatch.delenv("MR_NO_LO")
    wins = [(d_lo, t0, t1, a3, ok), (d_gen, t0, t1, a3, ok)] * 2
    monkeypatch.setenv("MR_WIN_CHUNK", "1")
    monkeypatch.setenv("MR_WIN_GROUP", "4")
    base = rank_windows(ctx, wins)
    monkeypatch.setenv("MR_KIND_TEST_COLLIDE", "1")
    coll = rank_windows(ctx, wins)
    for a, b in zip(base, coll):
        assert a[5] == b[5] == 0
        assert a[2:] == b[2:] and list(a[0]) == list(b[0]) and a[1].tobytes() == b[1].tobytes()
    assert base[0][2:] == base[1][2:] and list(base[0][0]) == list(base[1][0])
    np.testing.assert_allclose(base[0][1], base[1][1], rtol=1e-12, atol=0)
    d_lo.close()
    d_gen.close()


def test_single_window_early_spectrum_and_rerun(c3_window, monkeypatch):
    """A call of one window runs inline and queues its spectrum behind its PageRanks before their
    error words are read; a kind-hash collision (MR_KIND_TEST_COLLIDE, general build) reruns the
    PageRanks and queues the spectrum again.  Every variant ranks bitwise as the spectrum queued
    after the words (MR_WIN_SPEC_EARLY=0), on both table layouts."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    ctx = _lib.default_context()
    normal, abnormal, t0, t1 = c3_window
    a3, ok = bench.slo_from_gpu(ctx, normal)
    d_lo = DeviceSpans(ctx, abnormal)
    monkeypatch.setenv("MR_NO_LO", "1")
    d_gen = DeviceSpans(ctx, abnormal)
    monkeypatch.delenv("MR_NO_LO")
    for d in (d_lo, d_gen):
        one = [(d, t0, t1, a3, ok)]
        monkeypatch.setenv("MR_WIN_SPEC_EARLY", "0")
        base = rank_windows(ctx, one)[0]
        monkeypatch.delenv("MR_WIN_SPEC_EARLY")
        early = rank_windows(ctx, one)[0]
        monkeypatch.setenv("MR_KIND_TEST_COLLIDE", "1")
        coll = rank_windows(ctx, one)[0]
        monkeypatch.delenv("MR_KIND_TEST_COLLIDE")
        assert base[5] == 0 and len(base[0]) > 0
        for r in (early, coll):
            assert r[2:] == base[2:] and list(r[0]) == list(base[0]) and r[1].tobytes() == base[1].tobytes()
    d_lo.close()
    d_gen.close()


def test_last_block_call_graph_terms_bitwise(c3_window, monkeypatch):
    """Last-block graphs (one launch per iteration: C3-sized window graphs) take the call-graph
    terms alpha (P_ss s_k)[o] / M_s(k) from every block's write-through share (tr_ssv_share) instead
    of the last block's own ss_off -> ss_par -> pw chain: the same arithmetic, so a batch of four
    windows and a window alone rank bitwise as with the chain (MR_TR_LFSSV=0)."""
    import bench
    from microrank_amd import _lib
    from microrank_amd.online_rca import rank_windows
    from microrank_amd.preprocess_data import DeviceSpans

    ctx = _lib.default_context()
    normal, abnormal, t0, t1 = c3_window
    a3, ok = bench.slo_from_gpu(ctx, normal)
    d = DeviceSpans(ctx, abnormal)
    span = (t1 - t0) // 4
    wins = [(d, t0 + k * span // 8, t1 - k * span // 8, a3, ok) for k in range(4)]
    for batch in (wins, wins[:1]):
        monkeypatch.setenv("MR_TR_LFSSV", "0")
        base = rank_windows(ctx, batch)
        monkeypatch.delenv("MR_TR_LFSSV")
        got = rank_windows(ctx, batch)
        for a, b in zip(base, got):
            assert a[5] == 0 and len(a[0]) > 0
            assert a[2:] == b[2:] and list(a[0]) == list(b[0]) and a[1].tobytes() == b[1].tobytes()
    d.close()
