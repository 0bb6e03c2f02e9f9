"""ORACLE -- TEST INFRASTRUCTURE ONLY: ctypes binding of the C restatement (mr_oracle.c)."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libmr_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            import subprocess

            subprocess.run(["make"], cwd=HERE, check=True)
        _lib = C.CDLL(LIB)
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def rca_window(st, t0, t1, a3, a3v, method=0, top_max=5, nthreads=0):
    """One window on the CPU (oracle_rca_window).  Returns (codes, scores, n_abn, n_nor, edges)."""
    k = top_max + 6
    codes = np.zeros(k, np.int32)
    scores = np.zeros(k, np.float64)
    n_out, edges, na, nn = C.c_int32(), C.c_int64(), C.c_int32(), C.c_int32()
    cols = [np.ascontiguousarray(x) for x in (st.trace.astype(np.int32), st.podop.astype(np.int32),
                                               st.svcop.astype(np.int32), st.span.astype(np.int64),
                                               st.parent.astype(np.int64), st.duration.astype(np.int64),
                                               st.tstart.astype(np.int64), st.tend.astype(np.int64))]
    a3 = np.ascontiguousarray(a3, np.float64)
    a3v = np.ascontiguousarray(a3v, np.uint8)
    rc = lib().oracle_rca_window(
        C.c_int64(st.n_spans), _p(cols[0], C.c_int32), _p(cols[1], C.c_int32), _p(cols[2], C.c_int32),
        _p(cols[3], C.c_int64), _p(cols[4], C.c_int64), _p(cols[5], C.c_int64), _p(cols[6], C.c_int64),
        _p(cols[7], C.c_int64), C.c_int32(st.n_traces), C.c_int32(st.n_podops), C.c_int32(st.n_svcops),
        C.c_int64(t0), C.c_int64(t1), _p(a3, C.c_double), _p(a3v, C.c_uint8), C.c_int(method), C.c_int32(top_max),
        _p(codes, C.c_int32), _p(scores, C.c_double), C.byref(n_out), C.byref(edges), C.byref(na), C.byref(nn),
        C.c_int(nthreads))
    if rc == -2:
        return None
    m = n_out.value
    return codes[:m], scores[:m], na.value, nn.value, edges.value


def graph_pagerank(st, mask, anomaly):
    """(node podop codes, weights, coverage, nnz) for one graph (oracle_graph_pagerank)."""
    NP = st.n_podops
    node = np.zeros(NP, np.int32)
    w = np.zeros(NP, np.float64)
    cov = np.zeros(NP, np.int32)
    nn, nnz = C.c_int32(), C.c_int64()
    cols = [np.ascontiguousarray(x) for x in (st.trace.astype(np.int32), st.podop.astype(np.int32),
                                               st.span.astype(np.int64), st.parent.astype(np.int64))]
    m = np.ascontiguousarray(mask, np.uint8)
    rc = lib().oracle_graph_pagerank(C.c_int64(st.n_spans), _p(cols[0], C.c_int32), _p(cols[1], C.c_int32),
                                     _p(cols[2], C.c_int64), _p(cols[3], C.c_int64), C.c_int32(st.n_traces),
                                     C.c_int32(NP), _p(m, C.c_uint8), C.c_int(int(anomaly)), _p(node, C.c_int32),
                                     _p(w, C.c_double), _p(cov, C.c_int32), C.byref(nn), C.byref(nnz))
    if rc != 0:
        raise ValueError("zero-size array to reduction operation maximum which has no identity")
    n = nn.value
    return node[:n], w[:n], cov[:n], nnz.value


def incidence_pagerank(hg, anomaly, iters=25, nthreads=0):
    """trace_pagerank of a graph given as incidence lists (graph.HostGraph), on the CPU
    (oracle_incidence_pagerank).  Returns (weights, coverage, [s kinds + preference, s iterations])."""
    N, T = int(hg.N), int(hg.T)
    arrs = [np.ascontiguousarray(hg.sr_off, np.int64), np.ascontiguousarray(hg.sr_ops, np.int32),
            np.ascontiguousarray(hg.len_t, np.int32), np.ascontiguousarray(hg.len_o, np.int32),
            np.ascontiguousarray(hg.ss_off, np.int64), np.ascontiguousarray(hg.ss_par, np.int32),
            np.ascontiguousarray(hg.nchild, np.int32)]
    w = np.zeros(N, np.float64)
    cov = np.zeros(N, np.int32)
    tp = np.zeros(2, np.float64)
    rc = lib().oracle_incidence_pagerank(
        C.c_int32(N), C.c_int32(T), _p(arrs[0], C.c_int64), _p(arrs[1], C.c_int32), _p(arrs[2], C.c_int32),
        _p(arrs[3], C.c_int32), _p(arrs[4], C.c_int64), _p(arrs[5], C.c_int32), _p(arrs[6], C.c_int32),
        C.c_int(int(anomaly)), C.c_int(iters), C.c_int(nthreads), _p(w, C.c_double), _p(cov, C.c_int32),
        _p(tp, C.c_double))
    if rc != 0:
        raise ValueError("zero-size array to reduction operation maximum which has no identity")
    return w, cov, tp
