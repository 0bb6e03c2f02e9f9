/*
 * microrank_hip.h -- C-ABI of libmicrorank_hip.so, the MI355X (gfx950) implementation of
 * MicroRank's ranking hot path.  Plain pointers and sizes only; every entry point returns
 * an MR_* status (0 = ok) and mr_last_error(ctx) describes the failure.
 *
 * Each entry point names the reference interface it replaces (file:line in
 * CUHK-SE-Group/MicroRank @ 2025-02-14).  The Python drop-in modules in
 * microrank_amd/ (pagerank.py, preprocess_data.py, anormaly_detector.py, online_rca.py)
 * bind these with ctypes; INTEGRATION.md shows the binding a maintainer would add.
 *
 * Conventions
 *   - "host" pointers are caller-owned CPU memory, copied in/out inside the call.
 *   - "device" handles (mr_graph, mr_spans) own HBM; they belong to one mr_ctx.
 *   - Node order, trace order and every tie-break follow the reference.
 *   - Calls on distinct contexts are thread-safe; one context is not re-entrant.
 */
#ifndef MICRORANK_HIP_H
#define MICRORANK_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (the Python layer maps them onto the reference's exception types) ---- */
enum {
    MR_OK = 0,
    MR_ERR_ARG = 1,       /* bad argument / shape                        -> ValueError/TypeError */
    MR_ERR_HIP = 2,       /* HIP runtime failure                          -> RuntimeError */
    MR_ERR_VALUE = 3,     /* reference raises ValueError (empty graph, list.index miss) */
    MR_ERR_ZERODIV = 4,   /* reference raises ZeroDivisionError (1.0/len of an empty pr list) */
    MR_ERR_OOM = 5,       /* device allocation failed */
    MR_ERR_COMM = 6,      /* RCCL failure */
    MR_ERR_STATE = 7      /* handle used with the wrong context / before setup */
};

enum { MR_FP64 = 0, MR_FP32 = 1 };      /* precision of the rank vectors */

/* mr_pagerank flags */
enum {
    MR_PR_EXACT_SUMS = 1u,  /* sequential fp64 sums in reference order for the one-time scalars
                               (pagerank.py:71-78, 95-96; T7) instead of a fixed-order tree */
    MR_PR_KIND_COMPRESS = 2u /* mr_pagerank only: iterate over one
                               representative trace per kind with its multiplicity -- traces of
                               one kind (pagerank.py:54-66) have identical r; same weights
                               within fp64 rounding, work proportional to the kinds */
};

typedef struct mr_ctx mr_ctx;
typedef struct mr_graph mr_graph;
typedef struct mr_spans mr_spans;

/* ------------------------------------------------------------------ context */
int         mr_version(void);
int         mr_device_count(int* n);
int         mr_ctx_create(int device, uint32_t flags, mr_ctx** out);
void        mr_ctx_destroy(mr_ctx* ctx);
const char* mr_last_error(const mr_ctx* ctx);
int         mr_ctx_sync(mr_ctx* ctx);
/* stream the context launches on (a hipStream_t), for callers that time with HIP events */
void*       mr_ctx_stream(mr_ctx* ctx);
/* live timing of the power-iteration kernel: while enabled every launch is bracketed by HIP
 * events on the context stream; mr_ctx_prof_read syncs, returns the number of ITERATIONS the
 * recorded launches covered (one per launch pair; all of a call's for a persistent k_pr_cluster
 * launch), the summed kernel time and the summed algorithmic bytes (SURVEY §8(d) B_iter), and
 * clears the record */
int         mr_ctx_profile(mr_ctx* ctx, int enable);
int         mr_ctx_prof_read(mr_ctx* ctx, int64_t* launches, double* total_ms, double* total_bytes);
/* the device's measured copy peak (the HBM roofline is also reported against a
 * measured STREAM-copy rate beside the 8 TB/s spec): 16-B-per-lane copy kernels (grid-stride
 * and block-tile shapes, plain and non-temporal) over two buffers of `bytes` each on the context
 * stream, per shape one warm-up and `reps` timed launches; *gbs = the best launch's (read +
 * written) bytes / time in GB/s.  No reference counterpart (measurement) */
int         mr_copy_peak(mr_ctx* ctx, int64_t bytes, int reps, double* gbs);

/* ------------------------------------------------------------------ graph from index arrays
 * Replaces the dense matrix fill of pagerank.trace_pagerank (pagerank.py:16-52): the four
 * dicts become incidence lists.  Node ids follow the operation_operation key order, trace
 * ids the operation_trace key order.
 */
typedef struct mr_graph_desc {
    int32_t n_nodes;          /* N = len(operation_operation)                        */
    int32_t n_traces;         /* T = len(operation_trace)                            */
    int64_t nnz_sr;           /* distinct (trace, op) pairs of P_sr                  */
    const int64_t* sr_off;    /* [T+1] trace-major P_sr incidence (op in operation_trace[t]) */
    const int32_t* sr_ops;    /* [nnz_sr] node ids, ascending within a trace          */
    int64_t nnz_rs;           /* distinct pairs of P_rs; 0 with rs_* NULL = same as sr */
    const int64_t* rs_off;    /* [T+1] trace-major P_rs incidence (t in trace_operation[o]) */
    const int32_t* rs_ops;
    const int32_t* len_t;     /* [T] len(operation_trace[t])  -> P_sr value fp32(1/len_t) */
    const int32_t* len_o;     /* [N] len(trace_operation[o])  -> P_rs value fp32(1/len_o) */
    int64_t n_edges;          /* distinct (child, parent) pairs of P_ss               */
    const int64_t* ss_off;    /* [N+1] by child                                       */
    const int32_t* ss_par;    /* [n_edges] parent node ids, ascending within a child   */
    const int32_t* nchild;    /* [N] len(operation_operation[p]) -> P_ss value fp32(1/nchild) */
    int32_t n_pr;             /* len(pr_trace)                                        */
    const int32_t* pr_trace;  /* [n_pr] trace id of each pr_trace key, in pr_trace order */
    const int32_t* pr_len;    /* [n_pr] len(pr_trace[key])                            */
} mr_graph_desc;

int mr_graph_upload(mr_ctx* ctx, const mr_graph_desc* desc, mr_graph** out);
int mr_graph_free(mr_graph* g);
int mr_graph_info(const mr_graph* g, int32_t* n_nodes, int32_t* n_traces, int64_t* nnz,
                  int64_t* n_edges);

/* ------------------------------------------------------------------ K2: personalised PageRank
 * pagerank.trace_pagerank (pagerank.py:15-112) + pageRank (pagerank.py:116-130):
 * kinds (:54-66), preference vector (:68-85), `iters` Jacobi power iterations with max
 * normalisation (:121-129), weight = s*sum(s)/N and trace coverage (:93-107).
 * Results stay on the device; mr_graph_fetch copies them out.
 */
int mr_pagerank(mr_ctx* ctx, mr_graph* g, int anomaly, double d, double alpha, int iters,
                int precision, uint32_t flags);
/* mr_pagerank with the anomaly preference's weight phi exposed (the 0.5 at both places of
 * pagerank.py:82-84; SURVEY §5 config defaults: d = 0.85, alpha = 0.01 at :116, iters = 25 at
 * :117, phi = 0.5).  mr_pagerank is mr_pagerank_ex with phi = 0.5. */
int mr_pagerank_ex(mr_ctx* ctx, mr_graph* g, int anomaly, double d, double alpha, int iters, double phi,
                   int precision, uint32_t flags);
/* several independent graphs (e.g. the normal and anomaly graphs of a window, or many windows)
 * ranked together: one launch per Jacobi iteration covers every graph */
int mr_pagerank_batch(mr_ctx* ctx, mr_graph* const* graphs, const int* anomaly, int n_graphs, double d,
                      double alpha, int iters, int precision, uint32_t flags);
int mr_graph_fetch(mr_graph* g, double* weight /*[N] host*/, int32_t* coverage /*[N] host*/,
                   double* kind /*[T] host or NULL*/, float* pref /*[T] host or NULL*/);

/* ------------------------------------------------------------------ spans (int-coded columns)
 * The DataFrame of online_rca.py:221-248 after factorisation (microrank_amd/spans.py).
 */
typedef struct mr_span_cols {
    int64_t n_spans;
    int32_t n_traces, n_podops, n_svcops;
    const int32_t* trace;     /* trace code (rank of traceID in sorted order)       */
    const int32_t* podop;     /* podName_op code (sorted name order)                */
    const int32_t* svcop;     /* serviceName_op code (sorted name order)            */
    const int64_t* span;      /* spanID code                                        */
    const int64_t* parent;    /* ParentSpanId as a spanID code, -1 if absent        */
    const int64_t* duration;  /* span duration (reference units)                   */
    const int64_t* tstart;    /* trace-level start, ns (NULL if absent)             */
    const int64_t* tend;      /* trace-level end, ns                                */
    const int32_t* row;       /* global row index (NULL: the rows are the whole table) --
                                 a shard of a table split over ranks keeps the table's
                                 row order here for first appearance (T10)           */
} mr_span_cols;

int mr_spans_upload(mr_ctx* ctx, const mr_span_cols* cols, mr_spans** out);
int mr_spans_free(mr_spans* s);

/* SURVEY §8(f) f2 -- span ingest on the device from the string columns of the OTel export
 * (collect_data.py:35-46, renamed at online_rca.py:221-244).  A string column is Arrow-style:
 * value i = bytes[offsets[i] .. offsets[i+1]); valid is an Arrow validity bitmap (bit i of byte
 * i/8, 1 = present) or NULL (no nulls) -- only ParentSpanId may have nulls (a root span).
 * Produces the same table mr_spans_upload would get from SpanTable.from_dataframe: traceID,
 * podName_op and serviceName_op codes in sorted (code-point) name order, op = operationName with
 * ts-ui-dashboard's last '/segment' dropped (preprocess_data.py:26-33, 151-155), ParentSpanId
 * resolved to the equal spanID's code or -1.  Replaces the per-function string work of
 * preprocess_data.py (:26-33, 53-57, 100-104, 151-165). */
typedef struct mr_str_col {
    const int64_t* offsets;   /* [n_spans + 1] */
    const uint8_t* bytes;
    const uint8_t* valid;     /* Arrow bitmap or NULL */
} mr_str_col;
typedef struct mr_span_strings {
    int64_t n_spans;
    mr_str_col trace_id, span_id, parent_id, service, operation, pod;
    const int64_t* duration;  /* [n_spans] */
    const int64_t* tstart;    /* [n_spans] trace-level start, ns (NULL if absent) */
    const int64_t* tend;
} mr_span_strings;
int mr_spans_ingest(mr_ctx* ctx, const mr_span_strings* cols, mr_spans** out);
int mr_spans_info(const mr_spans* s, int64_t* n_spans, int32_t* n_traces, int32_t* n_podops, int32_t* n_svcops);
/* first row of each code in code order, which 0 trace / 1 pod-op / 2 service-op (ingested tables):
 * name of code k = that row's traceID / podName_op / serviceName_op */
int mr_spans_dict_rows(const mr_spans* s, int which, int32_t* rows);
/* SURVEY 8(f) f3, streaming: a new table = the rows of `prev` whose trace-level start is >=
 * keep_from (ns), in their order, then the chunk's rows -- the same table mr_spans_ingest builds
 * from those rows' strings.  The string columns stay on the device, so only the chunk crosses
 * PCIe (the resident rows are gathered device to device and re-coded there).  prev: NULL (the
 * first chunk) or a table this function returned on the same context; it stays valid (free it
 * with mr_spans_free).  The chunk needs tstart / tend.  Replaces the reference's per-window
 * re-read of the whole span frame (online_rca.py:161-216 over preprocess_data.get_span, :10-14). */
int mr_spans_append(mr_ctx* ctx, const mr_spans* prev, int64_t keep_from, const mr_span_strings* chunk,
                    mr_spans** out);
/* tables from mr_spans_append: the stream row number (position in the concatenation of every
 * chunk appended so far) of each code's first row, in code order -- mr_spans_dict_rows in stream
 * terms, so the host can read names from the chunk that holds the row */
int mr_spans_dict_sources(const mr_spans* s, int which, int64_t* src);
/* the code columns of a table (any pointer may be NULL), [n_spans] each */
int mr_spans_codes(const mr_spans* s, int32_t* trace, int32_t* podop, int32_t* svcop, int64_t* span,
                   int64_t* parent);

/* K1: preprocess_data.get_pagerank_graph (preprocess_data.py:146-171) on the device.
 * trace_mask[n_traces] (host, 0/1) selects the trace_list.  Node order = sorted parent ops,
 * then never-parent ops in first-appearance row order (T10).  The parent join ignores
 * traceID (T11). */
int mr_graph_build(mr_ctx* ctx, const mr_spans* s, const uint8_t* trace_mask, mr_graph** out);
/* K1 over a trace-sharded span table (one process per GPU, every span of a trace on one
 * rank, span / pod-op / trace codes global, cols.row set): this rank's graph over the GLOBAL
 * node order -- pod-op counts, first appearances and parent flags reduced over the ranks
 * (preprocess_data.py:159-163, T10), and the ParentSpanId == spanID join resolved across ranks
 * too (:157-158, T11: a child's parent rows may lie in traces of another rank).  len_o, nchild
 * and the call edges stay this rank's parts: mr_pagerank_sharded combines them.  Collectives
 * over the context's backend (mr_comm_init / mr_comm_set_host); replaces the per-rank
 * get_pagerank_graph(trace_list, span_df) of a sharded deployment. */
int mr_graph_build_sharded(mr_ctx* ctx, const mr_spans* s, const uint8_t* trace_mask, mr_graph** out);
/* node order (podop codes) and trace codes of a built graph */
int mr_graph_nodes(const mr_graph* g, int32_t* node_podop /*[N]*/, int32_t* trace_code /*[T]*/);
/* structure export for parity tests: any pointer may be NULL */
int mr_graph_export(const mr_graph* g, int64_t* sr_off /*[T+1]*/, int32_t* sr_ops /*[nnz]*/,
                    int32_t* len_t /*[T]*/, int32_t* len_o /*[N]*/, int64_t* ss_off /*[N+1]*/,
                    int32_t* ss_par /*[E]*/, int32_t* nchild /*[N]*/);

/* ------------------------------------------------------------------ K3: spectrum + top-k
 * online_rca.calculate_spectrum_without_delay_list (online_rca.py:33-152).  Inputs are in the
 * reference's iteration order: the anomaly_result nodes first, then normal-only nodes.
 * has_a/has_n mark membership; method is an index into
 * {dstar2, ochiai, jaccard, sorensendice, m1, m2, goodman, tarantula, russellrao, hamann,
 *  dice, simplematcing, rogers}.  Output: the first min(n, top) indices of the stable
 * descending sort and their scores.  A division by zero sets *zerodiv (the reference
 * raises ZeroDivisionError). */
int mr_spectrum(mr_ctx* ctx, int32_t n, const uint8_t* has_a, const double* a_w, const int64_t* a_num,
                const uint8_t* has_n, const double* n_w, const int64_t* n_num, int64_t a_len,
                int64_t n_len, int method, int32_t top, int32_t* out_idx, double* out_score,
                int32_t* n_out, int32_t* zerodiv);

/* ------------------------------------------------------------------ K4: SLO
 * preprocess_data.get_operation_slo (preprocess_data.py:50-78), the semantic body of the
 * broken anormaly_detector.get_slo (anormaly_detector.py:22-27, T16): per svcop code,
 * round(mean/1000, 4) and round(std/1000, 4) (population std, numpy pairwise order, T13).
 * count[o] = 0 marks an op with no spans. */
int mr_slo(mr_ctx* ctx, const mr_spans* s, double* mean /*[n_svcops]*/, double* std_ /*[n_svcops]*/,
           int64_t* count /*[n_svcops]*/);

/* ------------------------------------------------------------------ K5: detector
 * anormaly_detector.system_anomaly_detect (anormaly_detector.py:44-84) with
 * get_operation_duration_data (preprocess_data.py:97-122): window [t0, t1] on trace-level
 * times (inclusive), real = max duration/1000, expect = sum over ops (sorted order) of
 * count*a3[op] with a3 = mean+3*std, ops without SLO (a3_valid=0) contribute 0.
 * state[n_traces] (host): 0 not in window / dropped, 1 normal, 2 abnormal.
 * Returns MR_ERR_VALUE with *n_spans_in_window = 0 for an empty window (the reference
 * returns False, T2). */
int mr_detect(mr_ctx* ctx, const mr_spans* s, int64_t t0, int64_t t1, const double* a3,
              const uint8_t* a3_valid, uint8_t* state, int32_t* n_abnormal, int32_t* n_normal,
              int64_t* n_spans_in_window);

/* SURVEY §8(f) f3 -- the driver's whole window sweep (online_rca.py:161-216) detected at once:
 * for window m in [0, n_win) = [t_begin + m*grain, t_begin + m*grain + window] the counts of
 * mr_detect (abnormal / normal traces, in-window rows; n_rows[m] = 0 is the reference's empty
 * window, T2).  Needs trace-level times constant within each trace (the renamed TraceStart /
 * TraceEnd columns, online_rca.py:229-230): then a trace's partition does not depend on the window
 * and is computed once; state[n_traces] (host, optional) receives it (0 dropped, 1 normal,
 * 2 abnormal), so window m's lists are the traces of that state inside the window.
 * MR_ERR_STATE when times vary within a trace (run mr_detect per window instead). */
int mr_detect_sweep(mr_ctx* ctx, const mr_spans* s, int64_t t_begin, int64_t grain, int64_t window,
                    int32_t n_win, const double* a3, const uint8_t* a3_valid, uint8_t* state,
                    int32_t* n_abnormal, int32_t* n_normal, int64_t* n_rows);

/* ------------------------------------------------------------------ whole RCA window on device
 * online_rca.online_anomaly_detect_RCA body for one window (online_rca.py:164-215):
 * detect -> (swapped, T1) two graph builds -> two PageRanks -> spectrum -> top list, with
 * all intermediates resident in HBM.  out_idx are podop codes. */
int mr_rca_window(mr_ctx* ctx, const mr_spans* s, int64_t t0, int64_t t1, const double* a3,
                  const uint8_t* a3_valid, int method, int32_t top_max, int precision,
                  int32_t* out_podop, double* out_score, int32_t* n_out, int64_t* edges_traversed,
                  int32_t* n_abnormal, int32_t* n_normal);

/* C3: rank n_windows RCA windows in one call -- each as mr_rca_window.  Window i:
 * spans[i] (a span table of this context; windows may share one), [t0[i], t1[i]], the SLO
 * a3[i] / a3_valid[i] (n_svcops of spans[i]).  The windows' detectors and graph builds run
 * concurrently on auxiliary streams of this context, the PageRanks of all their graphs share
 * each power iteration's launches, then the spectra run concurrently.  Per window i:
 * out_podop / out_score[i * (top_max + 6) ..], n_out[i], edges_traversed[i], n_abnormal[i],
 * n_normal[i], status[i] (MR_OK, or MR_ERR_VALUE for an empty window -- the reference's
 * unpack of False, T2).  Replaces a loop of online_anomaly_detect_RCA windows
 * (online_rca.py:161-216) over independent windows.  Device memory: the graphs of large windows
 * (>= 64k traces on average) stay in the context's pools until the next call on it (released
 * there beside the new builds) or mr_ctx_destroy. */
int mr_windows_batch(mr_ctx* ctx, int32_t n_windows, const mr_spans* const* spans, const int64_t* t0,
                     const int64_t* t1, const double* const* a3, const uint8_t* const* a3_valid, int method,
                     int32_t top_max, int precision, int32_t* out_podop, double* out_score, int32_t* n_out,
                     int64_t* edges_traversed, int32_t* n_abnormal, int32_t* n_normal, int32_t* status);

/* ------------------------------------------------------------------ multi-GPU (RCCL over xGMI)
 * One process per GPU.  The unique id (128 bytes) is produced by rank 0 and broadcast by the
 * caller (torch.distributed / any host channel).  Used by the trace-sharded PageRank. */
int mr_comm_unique_id(uint8_t id[128]);
int mr_comm_init(mr_ctx* ctx, int nranks, int rank, const uint8_t id[128]);
int mr_comm_allreduce_f64(mr_ctx* ctx, double* dev_buf, int64_t n, int op /*0 sum, 1 max*/);

/* Host-staged collectives instead of RCCL (ranks sharing one GPU, CPU-side transports, tests):
 * the library copies the operand to host memory, calls fn, and copies the result back.
 *   coll 0 allreduce: buf[n] in/out, op 0 sum / 1 max
 *   coll 1 allgather: buf[nranks * n]; this rank's n elements are at rank * n on entry
 * dtype: 0 float64, 1 int32, 2 uint64, 3 int64.  fn returns 0 on success. */
typedef int (*mr_host_coll_fn)(void* user, int coll, void* buf, int64_t n, int dtype, int op);
int mr_comm_set_host(mr_ctx* ctx, mr_host_coll_fn fn, void* user, int nranks, int rank);

/* One-shot peer all-reduce for the per-iteration exchange of mr_pagerank_sharded (collective:
 * every rank of the context's backend calls it).  enable != 0: each rank exports a receive region
 * (uncached device memory) by IPC and maps every other rank's; an iteration's P_sr r limbs are then
 * written straight into every rank's region (xGMI stores between GPUs, one hop) and summed locally
 * in rank order, instead of an RCCL ring all-reduce (2 (R - 1) dependent steps).  The handles are
 * exchanged over the context's collectives on first use; enable = 0 unmaps them. */
int mr_comm_peer_enable(mr_ctx* ctx, int enable);
/* *active: 1 while the peer path carries this context's all-reduces (enabled and its regions
 * mapped on every rank), 0 otherwise -- e.g. after the ranks agreed that a mapping failed and fell
 * back to the RCCL / host collective, or after a peer timeout reset the regions.  Not collective. */
int mr_comm_peer_active(mr_ctx* ctx, int* active);

/* Trace-sharded PageRank: g holds THIS rank's traces (every span of
 * a trace on one rank) over the GLOBAL node index space, with this rank's partial len_o and
 * nchild and its local call edges.  Once per graph the library sums len_o / nchild / coverage,
 * unites the call edges, merges the trace-kind classes and the preference sums over the ranks;
 * per iteration it takes the max of r' and sums the P_sr r partials: exact fixed-point uint64
 * limbs on the fused iteration (N <= 16384), fp64 per-op sums on the tile path (larger N, C5).
 * Afterwards every rank holds the same weight and coverage vectors (mr_graph_fetch).
 * Requires a collective backend (mr_comm_init or mr_comm_set_host). */
int mr_pagerank_sharded(mr_ctx* ctx, mr_graph* g, int anomaly, double d, double alpha, int iters,
                        int precision, uint32_t flags);

#ifdef __cplusplus
}
#endif
#endif /* MICRORANK_HIP_H */
