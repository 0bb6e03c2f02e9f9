"""CPU checks of the C-ABI boundary: the HIP library loads here (no GPU needed), exports every
symbol include/microrank_hip.h declares, and the Python surface mirrors the reference's."""
import inspect
import os
import re

import pytest

from conftest import REPO


def _header_symbols():
    text = open(os.path.join(REPO, "include", "microrank_hip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(mr_[a-z0-9_]+)\s*\(", text))


def test_library_exports_every_declared_symbol():
    from microrank_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libmicrorank_hip.so not built (run __graft_entry__.build())")
    declared = _header_symbols()
    assert declared, "no declarations parsed"
    import ctypes

    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = sorted(s for s in declared if not hasattr(lib, s))
    assert not missing, f"declared but not exported: {missing}"
    # and the ctypes table covers exactly the header
    assert declared == set(_lib.SIGNATURES), (declared ^ set(_lib.SIGNATURES))


def test_no_gpu_fails_loudly():
    """Without a GPU the product raises instead of computing anything on the host."""
    from microrank_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    n = _lib.C.c_int(0)
    _lib.load().mr_device_count(_lib.C.byref(n))
    if n.value:
        pytest.skip("a GPU is visible")
    from microrank_amd.pagerank import trace_pagerank

    with pytest.raises(_lib.MRError):
        trace_pagerank({"a": []}, {"t": ["a"]}, {"a": ["t"]}, {"t": ["a"]}, False)


def test_python_surface_matches_reference_signatures():
    """Argument names of the drop-in functions are the reference's (the driver passes several
    by keyword: online_rca.py:167-201)."""
    from microrank_amd import anormaly_detector, online_rca, pagerank, preprocess_data

    def names(fn):
        return [p.name for p in inspect.signature(fn).parameters.values() if p.kind != p.KEYWORD_ONLY]

    assert names(pagerank.trace_pagerank) == ["operation_operation", "operation_trace", "trace_operation",
                                             "pr_trace", "anomaly"]
    assert names(online_rca.calculate_spectrum_without_delay_list) == [
        "anomaly_result", "normal_result", "anomaly_list_len", "normal_list_len", "top_max", "normal_num_list",
        "anomaly_num_list", "spectrum_method"]
    assert names(online_rca.online_anomaly_detect_RCA) == ["data", "slo", "operation_list"]
    assert names(anormaly_detector.system_anomaly_detect) == ["data", "start_time", "end_time", "slo",
                                                              "operation_list"]
    assert names(preprocess_data.get_pagerank_graph) == ["trace_list", "span_df"]
    assert names(preprocess_data.get_operation_slo) == ["service_operation_list", "span_df"]
    assert names(preprocess_data.get_service_operation_list) == ["span_df"]
    assert names(preprocess_data.get_span) == ["df", "start", "end"]


def test_product_does_not_import_oracle():
    import ast

    pkg = os.path.join(REPO, "microrank_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if not f.endswith(".py"):
                continue
            tree = ast.parse(open(os.path.join(root, f)).read())
            for node in ast.walk(tree):
                if isinstance(node, (ast.Import, ast.ImportFrom)):
                    mods = [a.name for a in node.names] if isinstance(node, ast.Import) else [node.module or ""]
                    assert not any(m.split(".")[0] in ("oracle", "c_oracle") for m in mods), f"{f} imports the oracle"


def test_span_table_ingest_codes_follow_string_order():
    import pandas as pd

    from microrank_amd.spans import SpanTable

    df = pd.DataFrame({"traceID": ["t2", "t10", "t1"], "spanID": ["a", "b", "c"], "ParentSpanId": [None, "a", "zz"],
                       "serviceName": ["ts-ui-dashboard", "s", "s"],
                       "operationName": ["GET /x/9", "op", "op"], "podName": ["p", "q", "q"],
                       "duration": [3, 2, 1]})
    st = SpanTable.from_dataframe(df)
    assert st.trace_names == ["t1", "t10", "t2"]        # code-point order (T10)
    assert list(st.trace) == [2, 1, 0]
    assert st.svcop_names == ["s_op", "ts-ui-dashboard_GET /x"]   # rsplit rule for the UI service
    assert list(st.parent) == [-1, 0, -1]               # orphan parent id -> -1 (T11)
