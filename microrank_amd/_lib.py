"""ctypes binding of libmicrorank_hip.so (include/microrank_hip.h).

There is no CPU fallback: if the library or a GPU is missing every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import sys
import os
import threading
from typing import Optional

import numpy as np

# MR_LIB_PATH: an alternative build of the same library (timing experiments)
LIB_PATH = os.environ.get("MR_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmicrorank_hip.so")

MR_OK, MR_ERR_ARG, MR_ERR_HIP, MR_ERR_VALUE, MR_ERR_ZERODIV, MR_ERR_OOM, MR_ERR_COMM, MR_ERR_STATE = range(8)
MR_FP64, MR_FP32 = 0, 1
MR_PR_EXACT_SUMS = 1
MR_PR_KIND_COMPRESS = 2   # mr_pagerank: iterate over one representative per trace kind (§8(f) f4)

SPECTRUM_METHODS = ("dstar2", "ochiai", "jaccard", "sorensendice", "m1", "m2", "goodman", "tarantula",
                    "russellrao", "hamann", "dice", "simplematcing", "rogers")

P = C.c_void_p
i32p = C.POINTER(C.c_int32)
i64p = C.POINTER(C.c_int64)
f64p = C.POINTER(C.c_double)
f32p = C.POINTER(C.c_float)
u8p = C.POINTER(C.c_uint8)


class GraphDesc(C.Structure):
    _fields_ = [("n_nodes", C.c_int32), ("n_traces", C.c_int32), ("nnz_sr", C.c_int64),
                ("sr_off", i64p), ("sr_ops", i32p), ("nnz_rs", C.c_int64), ("rs_off", i64p),
                ("rs_ops", i32p), ("len_t", i32p), ("len_o", i32p), ("n_edges", C.c_int64),
                ("ss_off", i64p), ("ss_par", i32p), ("nchild", i32p), ("n_pr", C.c_int32),
                ("pr_trace", i32p), ("pr_len", i32p)]


class SpanCols(C.Structure):
    _fields_ = [("n_spans", C.c_int64), ("n_traces", C.c_int32), ("n_podops", C.c_int32),
                ("n_svcops", C.c_int32), ("trace", i32p), ("podop", i32p), ("svcop", i32p),
                ("span", i64p), ("parent", i64p), ("duration", i64p), ("tstart", i64p), ("tend", i64p),
                ("row", i32p)]


class StrCol(C.Structure):
    _fields_ = [("offsets", i64p), ("bytes", C.c_void_p), ("valid", C.c_void_p)]


class SpanStrings(C.Structure):
    _fields_ = [("n_spans", C.c_int64), ("trace_id", StrCol), ("span_id", StrCol), ("parent_id", StrCol),
                ("service", StrCol), ("operation", StrCol), ("pod", StrCol), ("duration", i64p),
                ("tstart", i64p), ("tend", i64p)]


# name -> (restype, argtypes); every symbol here must be exported (tests check it)
SIGNATURES = {
    "mr_version": (C.c_int, []),
    "mr_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "mr_ctx_create": (C.c_int, [C.c_int, C.c_uint32, C.POINTER(P)]),
    "mr_ctx_destroy": (None, [P]),
    "mr_last_error": (C.c_char_p, [P]),
    "mr_ctx_sync": (C.c_int, [P]),
    "mr_ctx_stream": (P, [P]),
    "mr_ctx_profile": (C.c_int, [P, C.c_int]),
    "mr_ctx_prof_read": (C.c_int, [P, i64p, f64p, f64p]),
    "mr_copy_peak": (C.c_int, [P, C.c_int64, C.c_int, f64p]),
    "mr_graph_upload": (C.c_int, [P, C.POINTER(GraphDesc), C.POINTER(P)]),
    "mr_graph_free": (C.c_int, [P]),
    "mr_graph_info": (C.c_int, [P, i32p, i32p, i64p, i64p]),
    "mr_pagerank": (C.c_int, [P, P, C.c_int, C.c_double, C.c_double, C.c_int, C.c_int, C.c_uint32]),
    "mr_comm_peer_enable": (C.c_int, [P, C.c_int]),
    "mr_comm_peer_active": (C.c_int, [P, i32p]),
    "mr_pagerank_ex": (C.c_int, [P, P, C.c_int, C.c_double, C.c_double, C.c_int, C.c_double, C.c_int, C.c_uint32]),
    "mr_pagerank_batch": (C.c_int, [P, C.POINTER(P), C.POINTER(C.c_int), C.c_int, C.c_double, C.c_double, C.c_int,
                                    C.c_int, C.c_uint32]),
    "mr_graph_fetch": (C.c_int, [P, f64p, i32p, f64p, f32p]),
    "mr_spans_upload": (C.c_int, [P, C.POINTER(SpanCols), C.POINTER(P)]),
    "mr_graph_build_sharded": (C.c_int, [P, P, C.POINTER(C.c_uint8), C.POINTER(P)]),
    "mr_spans_free": (C.c_int, [P]),
    "mr_spans_ingest": (C.c_int, [P, C.POINTER(SpanStrings), C.POINTER(P)]),
    "mr_spans_info": (C.c_int, [P, i64p, i32p, i32p, i32p]),
    "mr_spans_dict_rows": (C.c_int, [P, C.c_int, i32p]),
    "mr_spans_append": (C.c_int, [P, P, C.c_int64, C.POINTER(SpanStrings), C.POINTER(P)]),
    "mr_spans_dict_sources": (C.c_int, [P, C.c_int, i64p]),
    "mr_spans_codes": (C.c_int, [P, i32p, i32p, i32p, i64p, i64p]),
    "mr_graph_build": (C.c_int, [P, P, u8p, C.POINTER(P)]),
    "mr_graph_nodes": (C.c_int, [P, i32p, i32p]),
    "mr_graph_export": (C.c_int, [P, i64p, i32p, i32p, i32p, i64p, i32p, i32p]),
    "mr_spectrum": (C.c_int, [P, C.c_int32, u8p, f64p, i64p, u8p, f64p, i64p, C.c_int64, C.c_int64,
                              C.c_int, C.c_int32, i32p, f64p, i32p, i32p]),
    "mr_slo": (C.c_int, [P, P, f64p, f64p, i64p]),
    "mr_detect": (C.c_int, [P, P, C.c_int64, C.c_int64, f64p, u8p, u8p, i32p, i32p, i64p]),
    "mr_detect_sweep": (C.c_int, [P, P, C.c_int64, C.c_int64, C.c_int64, C.c_int32, f64p, u8p, u8p, i32p, i32p,
                                  i64p]),
    "mr_windows_batch": (C.c_int, [P, C.c_int32, C.POINTER(P), i64p, i64p, C.POINTER(C.c_void_p),
                                   C.POINTER(C.c_void_p), C.c_int, C.c_int32, C.c_int, i32p, f64p, i32p, i64p, i32p,
                                   i32p, i32p]),
    "mr_rca_window": (C.c_int, [P, P, C.c_int64, C.c_int64, f64p, u8p, C.c_int, C.c_int32, C.c_int,
                                i32p, f64p, i32p, i64p, i32p, i32p]),
    "mr_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "mr_comm_init": (C.c_int, [P, C.c_int, C.c_int, C.POINTER(C.c_uint8)]),
    "mr_comm_allreduce_f64": (C.c_int, [P, P, C.c_int64, C.c_int]),
    "mr_comm_set_host": (C.c_int, [P, C.c_void_p, C.c_void_p, C.c_int, C.c_int]),
    "mr_pagerank_sharded": (C.c_int, [P, P, C.c_int, C.c_double, C.c_double, C.c_int, C.c_int, C.c_uint32]),
}

_lib = None
_lock = threading.Lock()


def load(path: str = LIB_PATH):
    """Load the shared library (raises if absent: there is no CPU fallback)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise RuntimeError(f"microrank_amd: HIP library not built ({path}); run __graft_entry__.build()")
        lib = C.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def exported_symbols(path: str = LIB_PATH):
    lib = C.CDLL(path)
    return {name for name in SIGNATURES if hasattr(lib, name)}


def ptr(a: Optional[np.ndarray], ctype):
    if a is None:
        return C.cast(None, C.POINTER(ctype))
    assert a.flags.c_contiguous, "arrays passed to the C-ABI must be contiguous"
    return a.ctypes.data_as(C.POINTER(ctype))


class MRError(RuntimeError):
    pass


def check(rc: int, ctx_handle=None, what: str = ""):
    if rc == MR_OK:
        return
    msg = ""
    if ctx_handle is not None:
        m = load().mr_last_error(ctx_handle)
        msg = m.decode(errors="replace") if m else ""
    text = f"{what}: {msg}" if what and not msg.startswith(what) else (msg or what)
    if rc == MR_ERR_VALUE:
        raise ValueError(msg or what)
    if rc == MR_ERR_ZERODIV:
        raise ZeroDivisionError(msg or "float division by zero")
    if rc == MR_ERR_ARG:
        raise ValueError(text)
    raise MRError(f"[{rc}] {text}")


class Context:
    """One HIP device + stream (mr_ctx).  Not re-entrant; use one per thread."""

    def __init__(self, device: int = 0, flags: int = 0):
        lib = load()
        h = P()
        rc = lib.mr_ctx_create(device, flags, C.byref(h))
        if rc != MR_OK:
            n = C.c_int(0)
            lib.mr_device_count(C.byref(n))
            raise MRError(f"mr_ctx_create(device={device}) failed with status {rc} "
                          f"({n.value} HIP devices visible)")
        self.h = h
        self.device = device

    def check(self, rc, what=""):
        check(rc, self.h, what)

    def sync(self):
        self.check(load().mr_ctx_sync(self.h), "mr_ctx_sync")

    def close(self):
        if getattr(self, "h", None):
            load().mr_ctx_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - interpreter teardown order
        if sys.is_finalizing():   # device handles may already be gone; the process exit frees all
            return
        try:
            self.close()
        except Exception:
            pass


_default = {}


def default_context() -> Context:
    """Per-process context on the device named by MICRORANK_DEVICE (else LOCAL_RANK, else 0)."""
    dev = int(os.environ.get("MICRORANK_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    ctx = _default.get(dev)
    if ctx is None:
        ctx = _default[dev] = Context(dev)
    return ctx
