// K5: anormaly_detector.system_anomaly_detect (anormaly_detector.py:44-84) with
// preprocess_data.get_operation_duration_data (preprocess_data.py:97-122), and the whole
// RCA window of online_rca.online_anomaly_detect_RCA (online_rca.py:164-215) on the device.
//
// Detector: spans whose trace-level [start, end] lies in [t0, t1] (inclusive, T15) are sorted
// by (trace, service-op); per trace, expect = sum over its ops in name order of
// count * (mean + 3 std), ops without an SLO adding nothing (the reference's bare except),
// real = max duration / 1000, abnormal iff real > expect (strict), traces with max <= 0
// dropped (preprocess_data.py:117).  The sum is sequential per trace with separate multiply and add (T14), so
// the partition is bit-exact.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <utility>
#include <vector>
#include <climits>
#include <cstring>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <tuple>
#include <mutex>
#include <string>
#include <thread>

#include "mr_detect_dev.h"
#include "mr_prim.h"
#include "mr_sort.h"

int mr_graph_build_dev(mr_ctx* ctx, const mr_spans* sp, const uint8_t* d_mask, mr_graph** out, const int64_t* win);
int mr_detect_indexed(mr_ctx* ctx, const mr_spans* s, int64_t t0, int64_t t1, const double* d_a3, const uint8_t* d_a3v,
                      uint8_t* d_state, int32_t* n_abn, int32_t* n_nor, int64_t* n_in);
int mr_spectrum_dev(mr_ctx* ctx, int32_t n, const uint8_t* flags, const double* a_w, const int64_t* a_num,
                    const double* n_w, const int64_t* n_num, int64_t A, int64_t Nl, int method, int32_t top,
                    int32_t* d_out_idx, double* d_out_score, uint8_t* d_out_np, int32_t* d_zflag);

namespace {
__global__ void k_win_flags(const int64_t* ts, const int64_t* te, int64_t S, int64_t t0, int64_t t1, int32_t* flag) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < S) flag[i] = (ts[i] >= t0 && te[i] <= t1) ? 1 : 0;
}
// Spans of a trace are mostly adjacent in DataFrame order, so a per-span atomicMax on
// tmax[trace] serialises lanes on one address.  A segmented max over the wave (combine with
// lane-off when it belongs to the same trace; max is idempotent, so non-adjacent runs of one
// trace merging is harmless) leaves the run maximum in the run's last lane, which alone issues
// the atomic.
__global__ void k_win_keys(const int32_t* flag, const int64_t* pos, int64_t S, const int32_t* trace, const int32_t* svcop,
                           const int64_t* dur, int nb, uint64_t* keys, long long* tmax) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = i < S && flag[i];
    const int32_t t = in ? trace[i] : -1;
    long long v = in ? (long long)dur[i] : LLONG_MIN;
    if (in) keys[pos[i]] = ((uint64_t)(uint32_t)t << nb) | (uint32_t)svcop[i];
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int32_t to = __shfl_up(t, off, 64);
        const long long vo = __shfl_up(v, off, 64);
        if (lane >= off && to == t && vo > v) v = vo;
    }
    const int32_t tn = __shfl_down(t, 1, 64);
    if (in && (lane == 63 || tn != t)) atomicMax(&tmax[t], v);
}
__global__ void k_win_runs(const uint64_t* keys, int64_t n, int32_t* head) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) head[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}
// runs -> (key, count); first run of each trace
__global__ void k_win_run_out(const uint64_t* keys, const int32_t* head, const int64_t* hpos, int64_t n, int nb,
                              uint64_t* rkey, int64_t* rstart, int64_t* tfirst) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !head[i]) return;
    const int64_t r = hpos[i];
    rkey[r] = keys[i];
    rstart[r] = i;
    const uint64_t t = keys[i] >> nb;
    if (i == 0 || (keys[i - 1] >> nb) != t) tfirst[t] = r;
}
__global__ void k_win_traces(const uint64_t* rkey, const int64_t* rstart, int64_t nruns, int64_t nspan, int nb,
                             const int64_t* tfirst, const long long* tmax, const double* a3, const uint8_t* a3v,
                             int32_t n_traces, uint8_t* state, int32_t* counts) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    int st = 0;
    if (t < n_traces) {
        const int64_t r0 = tfirst[t];
        const long long mx = r0 < 0 ? 0 : tmax[t];
        if (r0 >= 0 && mx > 0) {   // grouped[grouped['duration'] > 0] (preprocess_data.py:117)
            double expect = 0.0;
            const uint64_t mask = (1ull << nb) - 1ull;
            for (int64_t r = r0; r < nruns && (rkey[r] >> nb) == (uint64_t)t; ++r) {
                const int32_t op = (int32_t)(rkey[r] & mask);
                const int64_t end = r + 1 < nruns ? rstart[r + 1] : nspan;
                const int64_t cnt = end - rstart[r];
                if (a3v[op]) expect += (double)cnt * a3[op];   // anormaly_detector.py:64-65
            }
            const double real = (double)mx / 1000.0;           // :58
            st = real > expect ? 2 : 1;                        // :69
        }
        state[t] = (uint8_t)st;
    }
    // one counter update per wave (200k same-address atomics cost ~2 ms)
    const uint64_t ab = __ballot(st == 2), nr = __ballot(st == 1);
    if ((threadIdx.x & 63) == 0) {
        if (ab) atomicAdd(&counts[0], (int32_t)__popcll(ab));
        if (nr) atomicAdd(&counts[1], (int32_t)__popcll(nr));
    }
}
__global__ void k_fill_i64(int64_t* p, int64_t n, int64_t v) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

__global__ void k_union_init(int32_t* pos_of_code, int32_t NP, int64_t* ua_num, int64_t* un_num, uint8_t* fl,
                             double* ua_w, double* un_w, int32_t U, int32_t* zf) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < NP) pos_of_code[i] = -1;
    if (i < U) {
        ua_num[i] = 0;
        un_num[i] = 0;
        fl[i] = 0;
        ua_w[i] = 0.0;
        un_w[i] = 0.0;
    }
    if (i == 0) zf[0] = 0;
}
// union of the two graphs' nodes in the reference's spectrum order (online_rca.py:45-69)
__global__ void k_union_a(const int32_t* a_podop, int32_t Na, const double* a_w, const int32_t* a_cov, int32_t* pos_of_code,
                          uint8_t* flags, double* ua_w, int64_t* ua_num, int32_t* uc) {
    int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= Na) return;
    pos_of_code[a_podop[i]] = i;
    flags[i] = 1 | 4 | 8;   // in anomaly_result; np.float64 weights on both sides
    ua_w[i] = a_w[i];
    ua_num[i] = a_cov[i];
    uc[i] = a_podop[i];
}
__global__ void k_union_n_flags(const int32_t* n_podop, int32_t Nn, const int32_t* pos_of_code, int32_t* only) {
    int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < Nn) only[j] = pos_of_code[n_podop[j]] < 0 ? 1 : 0;
}
__global__ void k_union_n(const int32_t* n_podop, int32_t Nn, const double* n_w, const int32_t* n_cov,
                          const int32_t* pos_of_code, const int32_t* only, const int64_t* opos, int32_t Na,
                          uint8_t* flags, double* ua_w, int64_t* ua_num, double* un_w, int64_t* un_num, int32_t* uc) {
    int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= Nn) return;
    const int32_t c = n_podop[j];
    int32_t p;
    if (only[j]) {
        p = Na + (int32_t)opos[j];
        flags[p] = 2 | 8;
        ua_w[p] = 0.0;
        ua_num[p] = 0;
        uc[p] = c;
    } else {
        p = pos_of_code[c];
        flags[p] = 1 | 2 | 4 | 8;
    }
    un_w[p] = n_w[j];
    un_num[p] = n_cov[j];
}
}  // namespace

// Detector on the device; d_state[n_traces] receives 0/1/2.  Returns MR_ERR_VALUE for an empty window.
static int detect_dev(mr_ctx* ctx, const mr_spans* s, int64_t t0, int64_t t1, const double* d_a3, const uint8_t* d_a3v,
                      uint8_t* d_state, int32_t* n_abn, int32_t* n_nor, int64_t* n_in) {
    hipStream_t st = ctx->stream;
    const int64_t S = s->S;
    const int32_t NT = s->n_traces, NO = s->n_svcops;
    if (!s->has_times) return mr_fail(ctx, MR_ERR_ARG, "spans have no startTime/endTime columns");
    static const bool no_index = getenv("MR_NO_INDEX") != nullptr;   // A/B knob: force the row-level path
    if (s->indexed && s->uniform_times && !no_index)   // the window selects whole traces: per-trace pass
        return mr_detect_indexed(ctx, s, t0, t1, d_a3, d_a3v, d_state, n_abn, n_nor, n_in);
    DBuf<int32_t> flag;
    DBuf<int64_t> pos, tmp;
    MR_TRY(flag.alloc(ctx, S));
    MR_TRY(pos.alloc(ctx, S + 1));
    MR_TRY(tmp.alloc(ctx, std::max<int64_t>(scan_tmp_elems(S), 1)));
    if (S) hipLaunchKernelGGL(k_win_flags, dim3(cdiv(S, 256)), dim3(256), 0, st, s->tstart.p, s->tend.p, S, t0, t1, flag.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, flag.p, pos.p, S, tmp.p));
    int64_t W = 0;
    MR_TRY_HIP(ctx, hipMemcpyAsync(&W, pos.p + S, sizeof W, hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    *n_in = W;
    if (W == 0) return mr_fail(ctx, MR_ERR_VALUE, "Current span list is empty");
    const int nb = std::max(1, bits_for((uint64_t)std::max(NO - 1, 0)));
    DBuf<uint64_t> keys;
    DBuf<long long> tmax;
    MR_TRY(keys.alloc(ctx, W));
    MR_TRY(tmax.alloc(ctx, NT));
    MR_TRY_HIP(ctx, hipMemsetAsync(tmax.p, 0x80, NT * sizeof(long long), st));   // very negative
    hipLaunchKernelGGL(k_win_keys, dim3(cdiv(S, 256)), dim3(256), 0, st, flag.p, pos.p, S, s->trace.p, s->svcop.p,
                       s->duration.p, nb, keys.p, tmax.p);
    SortScratch ws;
    MR_TRY(mr_radix_sort(ctx, keys.p, nullptr, W, nb + bits_for((uint64_t)std::max(NT - 1, 0)), ws));
    DBuf<int32_t> head;
    DBuf<int64_t> hpos;
    MR_TRY(head.alloc(ctx, W));
    MR_TRY(hpos.alloc(ctx, W + 1));
    hipLaunchKernelGGL(k_win_runs, dim3(cdiv(W, 256)), dim3(256), 0, st, keys.p, W, head.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, head.p, hpos.p, W, tmp.p));
    int64_t R = 0;
    MR_TRY_HIP(ctx, hipMemcpyAsync(&R, hpos.p + W, sizeof R, hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    DBuf<uint64_t> rkey;
    DBuf<int64_t> rstart, tfirst;
    DBuf<int32_t> counts;
    MR_TRY(rkey.alloc(ctx, R));
    MR_TRY(rstart.alloc(ctx, R));
    MR_TRY(tfirst.alloc(ctx, NT));
    MR_TRY(counts.zero(ctx, 2));
    hipLaunchKernelGGL(k_fill_i64, dim3(cdiv(NT, 256)), dim3(256), 0, st, tfirst.p, (int64_t)NT, (int64_t)-1);
    hipLaunchKernelGGL(k_win_run_out, dim3(cdiv(W, 256)), dim3(256), 0, st, keys.p, head.p, hpos.p, W, nb, rkey.p,
                       rstart.p, tfirst.p);
    hipLaunchKernelGGL(k_win_traces, dim3(cdiv(NT, 256)), dim3(256), 0, st, rkey.p, rstart.p, R, W, nb, tfirst.p, tmax.p,
                       d_a3, d_a3v, NT, d_state, counts.p);
    MR_TRY_HIP(ctx, hipGetLastError());
    int32_t hc[2];
    MR_TRY(counts.download(ctx, hc, 2));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    *n_abn = hc[0];
    *n_nor = hc[1];
    return MR_OK;
}

extern "C" int mr_detect(mr_ctx* ctx, const mr_spans* s, int64_t t0, int64_t t1, const double* a3, const uint8_t* a3_valid,
                         uint8_t* state, int32_t* n_abnormal, int32_t* n_normal, int64_t* n_spans_in_window) {
    if (!ctx || !s || s->ctx != ctx || !a3 || !a3_valid || !state || !n_abnormal || !n_normal || !n_spans_in_window)
        return mr_fail(ctx, MR_ERR_ARG, "mr_detect: bad arguments");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    DBuf<double> da3;
    DBuf<uint8_t> dv, dst;
    MR_TRY(da3.upload(ctx, a3, s->n_svcops));
    MR_TRY(dv.upload(ctx, a3_valid, s->n_svcops));
    MR_TRY(dst.zero(ctx, s->n_traces));
    *n_abnormal = *n_normal = 0;
    MR_TRY(detect_dev(ctx, s, t0, t1, da3.p, dv.p, dst.p, n_abnormal, n_normal, n_spans_in_window));
    MR_TRY(dst.download(ctx, state, s->n_traces));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return MR_OK;
}

// f3: every window start of the driver's sweep (online_rca.py:161-216) detected in
// one pass -- each trace classified once, window counts from difference arrays (k_ix_sweep).
extern "C" int mr_detect_sweep(mr_ctx* ctx, const mr_spans* s, int64_t t_begin, int64_t grain, int64_t window,
                               int32_t n_win, const double* a3, const uint8_t* a3_valid, uint8_t* state,
                               int32_t* n_abnormal, int32_t* n_normal, int64_t* n_rows) {
    if (!ctx || !s || s->ctx != ctx || !a3 || !a3_valid || grain <= 0 || window < 0 || n_win < 0 ||
        (n_win && (!n_abnormal || !n_normal || !n_rows)))
        return mr_fail(ctx, MR_ERR_ARG, "mr_detect_sweep: bad arguments");
    if (!s->has_times) return mr_fail(ctx, MR_ERR_ARG, "spans have no startTime/endTime columns");
    if (!s->indexed || !s->uniform_times)
        return mr_fail(ctx, MR_ERR_STATE, "mr_detect_sweep: trace-level times differ within a trace (use mr_detect per window)");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    const int32_t NT = s->n_traces;
    DBuf<double> da3;
    DBuf<uint8_t> dv, dst;
    DBuf<unsigned long long> diff;
    MR_TRY(da3.upload(ctx, a3, (size_t)std::max(s->n_svcops, 1)));
    MR_TRY(dv.upload(ctx, a3_valid, (size_t)std::max(s->n_svcops, 1)));
    MR_TRY(dst.alloc(ctx, (size_t)std::max(NT, 1)));
    MR_TRY(diff.zero(ctx, (size_t)3 * (n_win + 1)));
    MR_TRY(mr_detect_sweep_launch(ctx, s, t_begin, grain, window, n_win, da3.p, dv.p, dst.p, diff.p));
    std::vector<unsigned long long> h((size_t)3 * (n_win + 1));
    MR_TRY(diff.download(ctx, h.data(), h.size()));
    if (state && NT) MR_TRY(dst.download(ctx, state, (size_t)NT));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    unsigned long long run[3] = {0, 0, 0};   // prefix sums mod 2^64 of exact integer differences
    for (int32_t m = 0; m < n_win; ++m) {
        for (int k = 0; k < 3; ++k) run[k] += h[(size_t)k * (n_win + 1) + m];
        n_abnormal[m] = (int32_t)run[0];
        n_normal[m] = (int32_t)run[1];
        n_rows[m] = (int64_t)run[2];
    }
    return MR_OK;
}

namespace {
__global__ void k_masks(const uint8_t* state, int32_t n, uint8_t* m_abn, uint8_t* m_nor) {
    int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    m_abn[t] = state[t] == 2;
    m_nor[t] = state[t] == 1;
}
__global__ void k_top_codes(const int32_t* idx, const int32_t* uc, int32_t k, int32_t* out) {
    int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) out[i] = uc[idx[i]];
}
}  // namespace

// One RCA window (online_rca.py:164-215) with every intermediate in HBM, in three phases so a
// batch of windows can overlap them: detect + both graph builds (any context), the two
// PageRanks (batched with other windows' graphs), the spectrum over the union.
struct WinRun {
    int rc = MR_OK;
    int32_t na = 0, nn = 0;
    int64_t nin = 0;
    mr_graph *gn = nullptr, *ga = nullptr;   // "normal" graph (detector's abnormal traces), "anomaly" graph
    bool slot = false;                       // batch: its spectrum went to the device result slot
    ~WinRun() {
        delete gn;
        delete ga;
    }
};

// MR_WIN_TIMING: wall time of each phase (a stream sync at each mark; diagnostics only)
struct WinMarks {
    hipStream_t st;
    bool on;
    std::vector<std::pair<const char*, std::chrono::steady_clock::time_point>> m;
    explicit WinMarks(hipStream_t s) : st(s), on(getenv("MR_WIN_TIMING") != nullptr) {}
    void mark(const char* name) {
        if (!on) return;
        (void)hipStreamSynchronize(st);
        m.emplace_back(name, std::chrono::steady_clock::now());
    }
    ~WinMarks() {
        if (m.size() < 2) return;
        fprintf(stderr, "[window]");
        for (size_t i = 1; i < m.size(); ++i)
            fprintf(stderr, " %s %.1f", m[i].first, std::chrono::duration<double, std::micro>(m[i].second - m[i - 1].second).count());
        fprintf(stderr, " us\n");
    }
};

static int win_detect_build(mr_ctx* ctx, const mr_spans* s, int64_t t0, int64_t t1, const double* a3,
                            const uint8_t* a3_valid, WinRun& w, WinMarks* mk, int precision = -1) {
    hipStream_t st = ctx->stream;
    const int32_t NT = s->n_traces;
    DBuf<double> da3;
    DBuf<uint8_t> dv, dst, m_abn, m_nor;
    MR_TRY(da3.upload(ctx, a3, s->n_svcops));
    MR_TRY(dv.upload(ctx, a3_valid, s->n_svcops));
    MR_TRY(dst.zero(ctx, NT));
    MR_TRY(detect_dev(ctx, s, t0, t1, da3.p, dv.p, dst.p, &w.na, &w.nn, &w.nin));
    if (mk) mk->mark("detect");
    // T1: the driver unpacks (flag, normal_list, abnormal_list) from (flag, abnormal, normal)
    if (w.na == 0 || w.nn == 0) return MR_OK;   // no anomaly, or one list empty: nothing is ranked
    MR_TRY(m_abn.alloc(ctx, NT));
    MR_TRY(m_nor.alloc(ctx, NT));
    hipLaunchKernelGGL(k_masks, dim3(cdiv(NT, 256)), dim3(256), 0, st, dst.p, NT, m_abn.p, m_nor.p);
    // the graphs take EVERY row of the selected traces: the driver passes the whole DataFrame,
    // get_pagerank_graph(normal_list, data) (online_rca.py:180,185), which filters by traceID
    // only (preprocess_data.py:148) -- not the detector's window rows
    MR_TRY(mr_graph_build_dev(ctx, s, m_abn.p, &w.gn, nullptr));   // "normal" graph = detector's abnormal traces
    if (mk) mk->mark("build_n");
    MR_TRY(mr_graph_build_dev(ctx, s, m_nor.p, &w.ga, nullptr));
    if (mk) mk->mark("build_a");
    if (precision >= 0) {   // batch: kinds / preference / iteration state on this stream too
        MR_TRY(mr_pagerank_presetup(ctx, w.gn, 0, 0.85, precision, 0));
        MR_TRY(mr_pagerank_presetup(ctx, w.ga, 1, 0.85, precision, 0));
    }
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    return MR_OK;
}

// Batch form of win_detect_build for a CHUNK of windows over indexed spans with trace-level times,
// all on this context's stream: every window's detector and both graph builds are enqueued first,
// their counters / sizes come back in ONE host round trip, and the chunk's graphs are prepared
// (and, when large, set up for PageRank) together -- five + six launches for all of them
// (mr_graph_prepare_batch, mr_pagerank_presetup_n).  A window costs its own seven build
// launches, the chunk one read-back; `ev` marks the chunk's graphs ready on this stream, and the
// caller's PageRank waits on it instead of on the host.  Per-window outcome in w->rc (MR_ERR_VALUE:
// empty window); a non-OK return fails the whole chunk.
// MR_WIN_PHASES=1 (read per call): host time per phase of mr_windows_batch, summed over the
// threads, printed to stderr at the end of a call (diagnostic)
struct WinPhases {
    std::atomic<long long> ns[10];
    WinPhases() {
        for (auto& x : ns) x = 0;
    }
};
static WinPhases* g_phases = nullptr;
static inline long long win_now() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
struct WinPhase {   // adds the scope's duration to phase i when timing is on
    int i;
    long long t;
    explicit WinPhase(int i_) : i(i_), t(g_phases ? win_now() : 0) {}
    ~WinPhase() {
        if (g_phases) g_phases->ns[i] += win_now() - t;
    }
};
static const char* const WIN_PHASE_NAME[10] = {"chunk launch", "chunk read-back wait", "chunk finish+prepare",
                                               "spectrum task", "worker idle", "main: wait builds",
                                               "main: pagerank batch", "main: tail", "main: call setup",
                                               "main: release graphs"};

struct WinIn {
    const mr_spans* s;
    int64_t t0, t1;
    const double* a3;      // (device)
    const uint8_t* a3v;    // (device)
    WinRun* w;
};
struct WinChunk {
    hipEvent_t ev = nullptr;
    std::vector<unsigned char> keep, keep2;   // host descriptors of the batched prepare / set-up
    ~WinChunk() {
        if (ev) (void)hipEventDestroy(ev);
    }
};
static int win_chunk_build_async(mr_ctx* ctx, const WinIn* in, int n, int precision, WinChunk& c) {
    hipStream_t st = ctx->stream;
    constexpr size_t CW = 3 * MR_DETECT_SHARDS;   // per window: detector counter shards, then 8 + 8 size words
    constexpr size_t WW = CW + 16;
    DBuf<int64_t> wb;
    auto ph0 = std::make_unique<WinPhase>(0);
    MR_TRY(wb.zero(ctx, (size_t)n * WW));
    std::vector<DBuf<uint8_t>> dst((size_t)n);   // (DBufs return to the pool stream-ordered: the
    std::vector<IxBuild> bx(2 * (size_t)n);      //  kernels enqueued on them run first)
    // the detector inside the index pass's first launch for tables up to MR_DET_FUSE_MAX traces
    // (default 65536; measured: C3's 20k traces +2%, C2's 200k -3% -- the fused launch's tiles
    // are the detector's 256 traces, 8x k_ix_sel_scan2's, and its look-back chains 8x longer).
    // MR_NO_DET_FUSE: never.  (Both read per call.)
    const char* fm = getenv("MR_DET_FUSE_MAX");
    const bool no_fuse = getenv("MR_NO_DET_FUSE") != nullptr;
    const int64_t fuse_max = fm ? (int64_t)atoll(fm) : 65536;
    std::vector<DetIn> dis((size_t)n);
    std::vector<char> fz((size_t)n);
    for (int k = 0; k < n; ++k) {
        const mr_spans* s = in[k].s;
        WinRun& w = *in[k].w;
        const int32_t NT = s->n_traces;
        int64_t* wk = wb.p + (size_t)k * WW;
        MR_TRY(dst[(size_t)k].alloc(ctx, std::max(NT, 1)));
        dis[(size_t)k] = mr_detect_in(s, in[k].t0, in[k].t1, in[k].a3, in[k].a3v, dst[(size_t)k].p, (unsigned long long*)wk);
        fz[(size_t)k] = !no_fuse && (int64_t)NT <= fuse_max;
        w.gn = new mr_graph();
        w.gn->ctx = ctx;
        w.ga = new mr_graph();
        w.ga->ctx = ctx;
    }
    // the whole chunk's index pass in one launch per stage when every window allows it (and the
    // windows agree on the detector fusion), else window by window.  Tables with a layout order
    // (mr_spans.lo_ok): the layout-order build (mr_lo_launch_batch), its kind histograms in one
    // zeroed buffer
    bool batched = false, lo = false;
    DBuf<uint32_t> zw;
    {
        bool ok = getenv("MR_NO_LO_WIN") == nullptr;   // (A/B and tests, read per call)
        int64_t nzw = 0;
        for (int k = 0; k < n && ok; ++k) {
            ok = in[k].s->lo_ok && mr_lo_fits(in[k].s);
            if (ok) nzw += mr_lo_zero_words(in[k].s);
        }
        if (ok) {
            MR_TRY(zw.zero(ctx, (size_t)nzw));
            std::vector<const mr_spans*> sps((size_t)n);
            std::vector<mr_graph*> g0((size_t)n), g1((size_t)n);
            std::vector<IxBuild*> b0((size_t)n), b1((size_t)n);
            std::vector<int64_t*> outs((size_t)n);
            std::vector<uint32_t*> zs((size_t)n);
            int64_t zo = 0;
            for (int k = 0; k < n; ++k) {
                sps[(size_t)k] = in[k].s;
                g0[(size_t)k] = in[k].w->gn;
                g1[(size_t)k] = in[k].w->ga;
                b0[(size_t)k] = &bx[2 * (size_t)k];
                b1[(size_t)k] = &bx[2 * (size_t)k + 1];
                outs[(size_t)k] = wb.p + (size_t)k * WW + CW;
                zs[(size_t)k] = zw.p + zo;
                zo += mr_lo_zero_words(in[k].s);
            }
            const int rcl = mr_lo_launch_batch(ctx, n, sps.data(), g0.data(), g1.data(), b0.data(), b1.data(), outs.data(),
                                               dis.data(), zs.data());
            if (rcl != MR_ERR_STATE) MR_TRY(rcl);
            batched = lo = rcl == MR_OK;
        }
    }
    if (n >= 2 && !batched) {
        bool same = true;
        for (int k = 1; k < n; ++k) same = same && fz[(size_t)k] == fz[0];
        if (same) {
            std::vector<const mr_spans*> sps((size_t)n);
            std::vector<uint8_t*> sts((size_t)n);
            std::vector<mr_graph*> g0((size_t)n), g1((size_t)n);
            std::vector<IxBuild*> b0((size_t)n), b1((size_t)n);
            std::vector<int64_t*> outs((size_t)n);
            for (int k = 0; k < n; ++k) {
                sps[(size_t)k] = in[k].s;
                sts[(size_t)k] = dst[(size_t)k].p;
                g0[(size_t)k] = in[k].w->gn;
                g1[(size_t)k] = in[k].w->ga;
                b0[(size_t)k] = &bx[2 * (size_t)k];
                b1[(size_t)k] = &bx[2 * (size_t)k + 1];
                outs[(size_t)k] = wb.p + (size_t)k * WW + CW;
            }
            const int rcb = mr_ix_launch2_batch(ctx, n, sps.data(), sts.data(), g0.data(), g1.data(), b0.data(), b1.data(),
                                                outs.data(), dis.data(), fz[0] != 0);
            if (rcb != MR_ERR_STATE) MR_TRY(rcb);
            batched = rcb == MR_OK;
        }
    }
    for (int k = 0; k < n && !batched; ++k) {
        const mr_spans* s = in[k].s;
        WinRun& w = *in[k].w;
        const int32_t NT = s->n_traces;
        int64_t* wk = wb.p + (size_t)k * WW;
        const DetIn& di = dis[(size_t)k];
        IxBuild &bn = bx[2 * (size_t)k], &ba = bx[2 * (size_t)k + 1];
        // (the graphs take EVERY row of the selected traces: get_pagerank_graph(list, data),
        // online_rca.py:180,185 / preprocess_data.py:148).  Both from the states in one pass over
        // the index when the table allows it, else one build per mask.
        const bool fuse = fz[(size_t)k] != 0;
        if (!fuse) MR_TRY(mr_detect_indexed_launch(ctx, s, in[k].t0, in[k].t1, in[k].a3, in[k].a3v, dst[(size_t)k].p,
                                                   (unsigned long long*)wk));
        const int rc2 = mr_ix_launch2(ctx, s, dst[(size_t)k].p, w.gn, w.ga, bn, ba, wk + CW, fuse ? &di : nullptr);
        if (rc2 == MR_ERR_STATE) {
            if (fuse) MR_TRY(mr_detect_indexed_launch(ctx, s, in[k].t0, in[k].t1, in[k].a3, in[k].a3v, dst[(size_t)k].p,
                                                      (unsigned long long*)wk));
            DBuf<uint8_t> m_abn, m_nor;
            MR_TRY(m_abn.alloc(ctx, std::max(NT, 1)));
            MR_TRY(m_nor.alloc(ctx, std::max(NT, 1)));
            if (NT) hipLaunchKernelGGL(k_masks, dim3(cdiv(NT, 256)), dim3(256), 0, st, dst[(size_t)k].p, NT, m_abn.p, m_nor.p);
            MR_TRY(mr_ix_launch(ctx, s, m_abn.p, w.gn, bn, wk + CW));   // "normal" graph = detector's abnormal traces
            MR_TRY(mr_ix_launch(ctx, s, m_nor.p, w.ga, ba, wk + CW + 8));
        } else {
            MR_TRY(rc2);
        }
    }
    ph0.reset();
    std::vector<int64_t> h((size_t)n * WW);
    {
        WinPhase ph(1);
        unsigned char* hp = nullptr;
        MR_TRY(mr_read_bytes(ctx, wb.p, h.size() * sizeof(int64_t), &hp));
        memcpy(h.data(), hp, h.size() * sizeof(int64_t));
    }
    WinPhase ph2(2);
    // MR_WIN_SETUP_SPLIT: traces of a window from which it sets up here (default 65536): small
    // windows (C3: 20k traces) leave it to the PageRank stream, which sets up the whole group's
    // graphs at once; large ones (C2: 200k traces) set up here, overlapping other work
    const char* se = getenv("MR_WIN_SETUP_SPLIT");   // (read per call: tests flip it)
    const int64_t split = se ? (int64_t)atoll(se) : (int64_t)65536;
    std::vector<mr_graph*> gs, pre;
    std::vector<int> pre_an;
    std::vector<const mr_spans*> gsp;   // (layout-order builds: each graph's table and build)
    std::vector<IxBuild*> gbx;
    for (int k = 0; k < n; ++k) {
        WinRun& w = *in[k].w;
        const int64_t* hk = h.data() + (size_t)k * WW;
        mr_detect_sum((const unsigned long long*)hk, &w.na, &w.nn, &w.nin);
        if (w.nin == 0 || w.na == 0 || w.nn == 0) {   // empty window, or a list empty: nothing is ranked (T1)
            delete w.gn;
            delete w.ga;
            w.gn = w.ga = nullptr;
            if (w.nin == 0) w.rc = MR_ERR_VALUE;   // "Current span list is empty"
            continue;
        }
        IxBuild &bn = bx[2 * (size_t)k], &ba = bx[2 * (size_t)k + 1];
        if (lo && (hk[CW + 2] || hk[CW + 8 + 2]))   // (mr_lo_fits bounds the edges: cannot happen)
            return mr_fail(ctx, MR_ERR_STATE, "mr_windows_batch: layout-order build past the node pass's edge limit");
        MR_TRY(mr_ix_finish_unprepared(ctx, in[k].s, w.gn, bn, bn.small ? hk + CW : nullptr));
        MR_TRY(mr_ix_finish_unprepared(ctx, in[k].s, w.ga, ba, ba.small ? hk + CW + 8 : nullptr));
        gs.push_back(w.gn);
        gs.push_back(w.ga);
        gsp.push_back(in[k].s);
        gsp.push_back(in[k].s);
        gbx.push_back(&bn);
        gbx.push_back(&ba);
        if (lo) continue;
        if ((int64_t)w.gn->T + w.ga->T >= split) {
            pre.push_back(w.gn);
            pre.push_back(w.ga);
            pre_an.push_back(0);
            pre_an.push_back(1);
        }
    }
    if (lo) {   // layout-order graphs: tiles, ids, kinds, preference and iteration state (pre_ok)
        std::vector<int> an(gs.size());
        for (size_t j = 0; j < gs.size(); ++j) an[j] = (int)(j & 1);   // (gn "normal", ga "anomaly": T1)
        if (!gs.empty()) MR_TRY(mr_lo_prepare_batch(ctx, gs.data(), gsp.data(), gbx.data(), an.data(), (int)gs.size(), 0.85,
                                                    precision, c.keep));
    } else if (!gs.empty()) {
        MR_TRY(mr_graph_prepare_batch(ctx, gs.data(), (int)gs.size(), c.keep));
    }
    if (!pre.empty()) MR_TRY(mr_pagerank_presetup_n(ctx, pre.data(), pre_an.data(), (int)pre.size(), 0.85, precision, c.keep2));
    if (!c.ev) MR_TRY_HIP(ctx, hipEventCreateWithFlags(&c.ev, hipEventDisableTiming));
    MR_TRY_HIP(ctx, hipEventRecord(c.ev, st));
    return MR_OK;
}

// spectrum over the union (anomaly nodes, then normal-only nodes) -> top codes / scores (host)
static int win_spectrum(mr_ctx* ctx, const mr_spans* s, const WinRun& w, int method, int32_t top_max,
                        int32_t* out_podop, double* out_score, int32_t* n_out) {
    hipStream_t st = ctx->stream;
    const int32_t NP = s->n_podops;
    const mr_graph *gn = w.gn, *ga = w.ga;
    const int32_t Na = ga->N, Nn = gn->N;
    const bool no_small = getenv("MR_NO_WIN_SPECTRUM_SMALL") != nullptr;   // general path (read per call: tests)
    if (!no_small) {   // one block, one read-back (k_win_spectrum) when the window fits it
        const int rc = mr_win_spectrum_small(ctx, Na, ga->node_podop.p, ga->weight.p, ga->cov.p, Nn, gn->node_podop.p,
                                             gn->weight.p, gn->cov.p, NP, w.nn, w.na, method,
                                             std::max(0, top_max + 6), out_podop, out_score, n_out);
        if (rc != MR_ERR_STATE) return rc;
    }
    DBuf<int32_t> pos_of_code, only, uc, idx, zf;
    DBuf<int64_t> opos, tmp, ua_num, un_num;
    DBuf<uint8_t> fl;
    DBuf<double> ua_w, un_w, sc;
    const int32_t U = Na + Nn;   // upper bound
    MR_TRY(pos_of_code.alloc(ctx, NP));
    MR_TRY(only.alloc(ctx, Nn));
    MR_TRY(uc.alloc(ctx, U));
    MR_TRY(opos.alloc(ctx, Nn + 1));
    MR_TRY(tmp.alloc(ctx, scan_tmp_elems(Nn)));
    MR_TRY(ua_num.alloc(ctx, U));
    MR_TRY(un_num.alloc(ctx, U));
    MR_TRY(fl.alloc(ctx, U));
    MR_TRY(ua_w.alloc(ctx, U));
    MR_TRY(un_w.alloc(ctx, U));
    MR_TRY(zf.alloc(ctx, 1));
    // one launch clears the union's arrays (was seven memsets per window)
    hipLaunchKernelGGL(k_union_init, dim3(cdiv(std::max<int64_t>({(int64_t)NP, (int64_t)U, 1}), 256)), dim3(256), 0, st,
                       pos_of_code.p, NP, ua_num.p, un_num.p, fl.p, ua_w.p, un_w.p, U, zf.p);
    hipLaunchKernelGGL(k_union_a, dim3(cdiv(Na, 256)), dim3(256), 0, st, ga->node_podop.p, Na, ga->weight.p, ga->cov.p,
                       pos_of_code.p, fl.p, ua_w.p, ua_num.p, uc.p);
    hipLaunchKernelGGL(k_union_n_flags, dim3(cdiv(Nn, 256)), dim3(256), 0, st, gn->node_podop.p, Nn, pos_of_code.p, only.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, only.p, opos.p, Nn, tmp.p));
    int64_t nonly = 0;
    MR_TRY_HIP(ctx, hipMemcpyAsync(&nonly, opos.p + Nn, sizeof nonly, hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    hipLaunchKernelGGL(k_union_n, dim3(cdiv(Nn, 256)), dim3(256), 0, st, gn->node_podop.p, Nn, gn->weight.p, gn->cov.p,
                       pos_of_code.p, only.p, opos.p, Na, fl.p, ua_w.p, ua_num.p, un_w.p, un_num.p, uc.p);
    const int32_t n = Na + (int32_t)nonly;
    const int32_t k = std::min(n, std::max(0, top_max + 6));   // online_rca.py:148
    MR_TRY(idx.alloc(ctx, std::max(k, 1)));
    MR_TRY(sc.alloc(ctx, std::max(k, 1)));
    // A = len(abnormal_list) = detector normal count, N = len(normal_list) = detector abnormal count
    MR_TRY(mr_spectrum_dev(ctx, n, fl.p, ua_w.p, ua_num.p, un_w.p, un_num.p, w.nn, w.na, method, k, idx.p, sc.p, nullptr,
                           zf.p));
    DBuf<int32_t> codes;
    MR_TRY(codes.alloc(ctx, std::max(k, 1)));
    if (k) hipLaunchKernelGGL(k_top_codes, dim3(cdiv(k, 256)), dim3(256), 0, st, idx.p, uc.p, k, codes.p);
    if (k && out_podop) MR_TRY(codes.download(ctx, out_podop, k));
    if (k && out_score) MR_TRY(sc.download(ctx, out_score, k));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    *n_out = k;
    return MR_OK;
}

static int64_t win_edges(const WinRun& w) {
    return w.gn ? 25 * (2 * (w.gn->nnz_sr + w.ga->nnz_sr) + w.gn->E + w.ga->E) : 0;
}

extern "C" int mr_rca_window(mr_ctx* ctx, const mr_spans* s, int64_t t0, int64_t t1, const double* a3,
                             const uint8_t* a3_valid, int method, int32_t top_max, int precision, int32_t* out_podop,
                             double* out_score, int32_t* n_out, int64_t* edges_traversed, int32_t* n_abnormal,
                             int32_t* n_normal) {
    if (!ctx || !s || s->ctx != ctx || !a3 || !a3_valid || !n_out) return mr_fail(ctx, MR_ERR_ARG, "mr_rca_window: bad arguments");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    *n_out = 0;
    if (edges_traversed) *edges_traversed = 0;
    // tables with a layout order: the window batch's build (one window), so a window ranks the
    // same whether it comes alone or in a batch (the driver's window loop and its sweep, f3)
    if (s->indexed && s->uniform_times && s->has_times && s->lo_ok && mr_lo_fits(s) && !getenv("MR_NO_LO_WIN") &&
        !getenv("MR_NO_INDEX")) {
        int32_t stw = MR_OK, na = 0, nn = 0;
        int64_t ew = 0;
        MR_TRY(mr_windows_batch(ctx, 1, &s, &t0, &t1, &a3, &a3_valid, method, top_max, precision, out_podop, out_score,
                                n_out, &ew, &na, &nn, &stw));
        if (stw == MR_ERR_VALUE) return mr_fail(ctx, MR_ERR_VALUE, "Current span list is empty");
        if (stw != MR_OK) return stw;
        if (edges_traversed) *edges_traversed = ew;
        if (n_abnormal) *n_abnormal = na;
        if (n_normal) *n_normal = nn;
        return MR_OK;
    }
    WinMarks mk(ctx->stream);
    mk.mark("start");
    WinRun w;
    MR_TRY(win_detect_build(ctx, s, t0, t1, a3, a3_valid, w, &mk));
    if (n_abnormal) *n_abnormal = w.na;
    if (n_normal) *n_normal = w.nn;
    if (!w.gn) return MR_OK;
    mr_graph* both[2] = {w.gn, w.ga};   // both PageRanks in one batched launch per iteration
    const int anom[2] = {0, 1};
    MR_TRY(mr_pagerank_batch(ctx, both, anom, 2, 0.85, 0.01, 25, precision, 0));
    mk.mark("pagerank");
    if (edges_traversed) *edges_traversed = win_edges(w);
    MR_TRY(win_spectrum(ctx, s, w, method, top_max, out_podop, out_score, n_out));
    mk.mark("spectrum");
    return MR_OK;
}

// C3: many windows per call, pipelined over GROUPS of windows.  Auxiliary
// contexts (own stream and pool each) driven by host threads run the windows' detector + graph
// builds and, later, their spectra; this context runs the PageRanks of one group's graphs at a
// time (all of the group's graphs share each iteration's k_tr_a + k_fx_b launches) while the
// auxiliary streams already build the next group's graphs.
static int win_aux(mr_ctx* ctx, int n) {
    while ((int)ctx->aux.size() < n) {
        mr_ctx* a = nullptr;
        const int rc = mr_ctx_create(ctx->device, ctx->flags, &a);
        if (rc != MR_OK) return mr_fail(ctx, rc, "mr_windows_batch: auxiliary context creation failed");
        // (the build streams at the PageRank stream's priority: a high-priority PageRank stream
        // measured C2 -4 % in round 4, low-priority build streams within the spread in round 6,
        // profiles/r06/r06h_serial_priority_ab.txt)
#ifdef MR_AB_CUMASK   // (A/B builds: the build streams on the CUs with i % 4 < MR_AB_CUMASK only)
        {
            int ncu = 0;
            if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device) == hipSuccess && ncu > 0) {
                std::vector<uint32_t> m((size_t)(ncu + 31) / 32, 0u);
                for (int i = 0; i < ncu; ++i)
                    if (i % 4 < MR_AB_CUMASK) m[(size_t)i / 32] |= 1u << (i % 32);
                hipStream_t s2 = nullptr;
                if (hipExtStreamCreateWithCUMask(&s2, (uint32_t)m.size(), m.data()) == hipSuccess) {
                    (void)hipStreamDestroy(a->stream);
                    a->stream = s2;
                }
            }
        }
#endif
        ctx->aux.push_back(a);
    }
    return MR_OK;
}

extern "C" int mr_windows_batch(mr_ctx* ctx, int32_t n_windows, const mr_spans* const* spans, const int64_t* t0,
                                const int64_t* t1, const double* const* a3, const uint8_t* const* a3_valid, int method,
                                int32_t top_max, int precision, int32_t* out_podop, double* out_score, int32_t* n_out,
                                int64_t* edges_traversed, int32_t* n_abnormal, int32_t* n_normal, int32_t* status) {
    if (!ctx || n_windows < 0 || (n_windows && (!spans || !t0 || !t1 || !a3 || !a3_valid || !n_out || !status)))
        return mr_fail(ctx, MR_ERR_ARG, "mr_windows_batch: bad arguments");
    for (int32_t i = 0; i < n_windows; ++i)
        if (!spans[i] || spans[i]->ctx != ctx || !a3[i] || !a3_valid[i])
            return mr_fail(ctx, MR_ERR_ARG, "mr_windows_batch: bad window %d", i);
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    if (n_windows == 0) return MR_OK;
    // (diagnostic phase timers: one call at a time sets them)
    static WinPhases phases_store;
    const bool timing = getenv("MR_WIN_PHASES") != nullptr;
    if (timing) {
        for (auto& x : phases_store.ns) x = 0;
        g_phases = &phases_store;
    }
    const long long t_call = timing ? win_now() : 0;
    const int32_t K = std::max(0, top_max + 6);
    // auxiliary streams (and host threads) of a batch: 4 measured best (C2 2908 / C3 4850
    // windows/s vs 2705 / 4247 at 16): the windows' launches come from the host threads and more
    // threads only contend for the runtime (the box runs 4 hardware queues per process)
    constexpr int max_streams = 4;
    // Windows whose PageRanks share launches (a group): at most WIN_GROUP_TRACES traces per group,
    // 16..128 windows.  The iteration pair of a small-window group is latency-bound, so its cost per
    // window falls with the group (C3, 20k-trace windows, on one box: group 16 / 32 / 64 / 128 ->
    // 9.4k / 12.1k / 14.8k / 15.4k windows/s with chunks of 8 at 128; C2, 200k-trace windows in
    // calls of 64: group 16 / 32 -> 4578 / 4773 windows/s, iteration frac 0.355 / 0.51, two
    // repeats each on one box; round 4, calls of 128: group 32 / 64 -> 5351-5363 / 5402-5433
    // windows/s, in-pipeline iteration frac 0.39 / 0.46, `profiles/r04s/`; calls of 256: group
    // 64 / 128 -> 5780-5868 / 5795-5838 windows/s, frac 0.47 / 0.54, `profiles/r04ac/`).  A window's trace count
    // is bounded by its table's (a window of a long shared table gets the small group: the round-2
    // behaviour).  Chunks of 8 windows for small windows (C3), 4 for large (C2: 4 measured better).
    // MR_WIN_GROUP / MR_WIN_CHUNK: fixed group / chunk sizes (read per call)
    constexpr int64_t WIN_GROUP_TRACES = (int64_t)32 << 20;
    int64_t tsum_tab = 0;
    for (int32_t i = 0; i < n_windows; ++i) tsum_tab += std::max<int32_t>(spans[i]->n_traces, 1);
    const int64_t tper = std::max<int64_t>(1, tsum_tab / n_windows);
    int group_size = 16;
    while (group_size < 128 && (int64_t)group_size * 2 * tper <= WIN_GROUP_TRACES) group_size *= 2;
    // at least two groups per call: the next group's builds overlap this one's PageRanks (round 5,
    // C2 calls of 128 windows: group 128 / 64 -> 652-674 / 748-807 GTEPS; calls of 256: group 128
    // and 64 within the spread, 981-1002 / 904-1000 GTEPS, `profiles/r05/r05f_groups_ab.txt`)
    while (group_size > 16 && 2 * group_size > n_windows) group_size /= 2;
    if (const char* e = getenv("MR_WIN_GROUP")) group_size = std::max(1, atoi(e));
    const char* ce = getenv("MR_WIN_CHUNK");   // windows built together on one stream
    const int chunk_size = ce ? std::max(1, atoi(ce)) : group_size >= 64 && tper <= 65536 ? 8 : 4;
    const int gsz = std::min<int>(n_windows, group_size);
    // group g: windows [gbeg[g], gbeg[g + 1])
    std::vector<int32_t> gbeg(1, 0);
    while (gbeg.back() < n_windows) gbeg.push_back(std::min<int32_t>(n_windows, gbeg.back() + gsz));
    const int ngroups = (int)gbeg.size() - 1;
    std::vector<int32_t> group_of((size_t)n_windows);
    for (int g = 0; g < ngroups; ++g)
        for (int32_t i = gbeg[(size_t)g]; i < gbeg[(size_t)g + 1]; ++i) group_of[(size_t)i] = g;
    // build chunks: consecutive windows of one group
    std::vector<std::pair<int32_t, int32_t>> chunks;
    for (int g = 0; g < ngroups; ++g)
        for (int32_t i = gbeg[(size_t)g], e = gbeg[(size_t)g + 1]; i < e; i += chunk_size)
            chunks.emplace_back(i, std::min<int32_t>(e, i + chunk_size));
    // a call of one chunk (one window: the single-window latency) runs inline: its build, PageRanks
    // and spectrum on this context's stream from the calling thread -- no worker thread to start,
    // no hand-offs between threads or streams
    const bool inl = chunks.size() == 1;
    const int nthr = inl ? 0 : std::min<int>((int)chunks.size(), max_streams);
    // (every group's PageRanks on this context's stream: a second PageRank stream for odd groups
    // measured within the spread, profiles/r04al/, and was removed)
    if (nthr) MR_TRY(win_aux(ctx, nthr));
    auto pr_ctx = [&](int) -> mr_ctx* { return ctx; };
    // the SLO vectors once per distinct (a3, a3_valid, length) of the batch (windows usually share
    // one pair), resident before any window's detector runs
    std::unique_ptr<WinPhase> ph_setup(new WinPhase(8));
    std::map<std::tuple<const double*, const uint8_t*, int32_t>, size_t> slo_ix;
    std::vector<std::unique_ptr<DBuf<double>>> d_a3;
    std::vector<std::unique_ptr<DBuf<uint8_t>>> d_a3v;
    std::vector<size_t> slo_of((size_t)n_windows);
    std::vector<int32_t> slo_win;   // the first window of each distinct vector pair
    size_t slo_bytes = 0;
    for (int32_t i = 0; i < n_windows; ++i) {
        const auto key = std::make_tuple(a3[i], a3_valid[i], spans[i]->n_svcops);
        auto it = slo_ix.find(key);
        if (it == slo_ix.end()) {
            it = slo_ix.emplace(key, slo_win.size()).first;
            slo_win.push_back(i);
            slo_bytes += (size_t)std::max(spans[i]->n_svcops, 1) * 9 + 16;
        }
        slo_of[(size_t)i] = it->second;
    }
    // staged through the context's pinned buffer when they fit: the copies go out asynchronously
    // (a pageable copy blocks this thread while the runtime stages it)
    if (slo_bytes <= MR_PIN_BYTES && !ctx->pin &&
        hipHostMalloc((void**)&ctx->pin, MR_PIN_BYTES, hipHostMallocDefault) != hipSuccess)
        ctx->pin = nullptr;
    unsigned char* stage = slo_bytes <= MR_PIN_BYTES ? (unsigned char*)ctx->pin : nullptr;
    for (int32_t i : slo_win) {
        const size_t ns = (size_t)std::max(spans[i]->n_svcops, 1);
        d_a3.emplace_back(new DBuf<double>());
        d_a3v.emplace_back(new DBuf<uint8_t>());
        if (!stage) {
            MR_TRY(d_a3.back()->upload(ctx, a3[i], ns));
            MR_TRY(d_a3v.back()->upload(ctx, a3_valid[i], ns));
            continue;
        }
        MR_TRY(d_a3.back()->alloc(ctx, ns));
        MR_TRY(d_a3v.back()->alloc(ctx, ns));
        const size_t n_in = (size_t)spans[i]->n_svcops;   // (0: the buffers stay unread)
        memcpy(stage, a3[i], n_in * sizeof(double));
        memcpy(stage + n_in * sizeof(double), a3_valid[i], n_in);
        if (n_in) {
            MR_TRY_HIP(ctx, hipMemcpyAsync(d_a3.back()->p, stage, n_in * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
            MR_TRY_HIP(ctx, hipMemcpyAsync(d_a3v.back()->p, stage + n_in * sizeof(double), n_in, hipMemcpyHostToDevice,
                                           ctx->stream));
        }
        stage += (n_in * 9 + 15) / 16 * 16;
    }
    // the windows' spectrum results land in device slots, read back once at the end
    DBuf<unsigned char> slots;
    MR_TRY(slots.alloc(ctx, (size_t)n_windows * MR_WS_SLOT));
    if (!inl) MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));   // uploads done before other streams read them
    static const bool no_index = getenv("MR_NO_INDEX") != nullptr;
    const bool spec_general = getenv("MR_NO_WIN_SPECTRUM_SMALL") != nullptr;   // (read per call: tests)
    constexpr int spec_batch = MR_WS_BATCH;   // windows per spectrum launch
    ph_setup.reset();
    std::vector<WinRun> w((size_t)n_windows);
    std::vector<WinChunk> cw(chunks.size());
    std::vector<hipEvent_t> gev((size_t)ngroups, nullptr);   // a group's PageRanks are done
    std::vector<std::string> err((size_t)std::max(nthr, 1));
    // task queue: phase-1 tasks (chunk c -> c) first, phase-3 tasks (the spectra of spec[i] -> ~i)
    // appended per group
    std::mutex mu;
    std::condition_variable cv_task, cv_done;
    std::deque<int32_t> q;
    std::vector<std::vector<int32_t>> spec((size_t)n_windows);   // a spectrum task's windows (by its first)
    bool closed = false;
    std::vector<int> built((size_t)ngroups, 0);
    for (int32_t c = 0; c < (int32_t)chunks.size(); ++c) q.push_back(c);
    // a task: chunk c (c >= 0: its detectors + graph builds) or the spectra of spec[~c], on context a
    auto do_task = [&](int32_t task, mr_ctx* a, int k) {
        if (task >= 0) {   // a chunk's detectors + graph builds
            const int32_t i0 = chunks[(size_t)task].first, i1 = chunks[(size_t)task].second;
            std::vector<WinIn> fast;
            for (int32_t i = i0; i < i1; ++i) {
                WinRun& r = w[(size_t)i];
                const mr_spans* sp = spans[i];
                if (sp->indexed && sp->uniform_times && sp->has_times && !no_index) {
                    fast.push_back(WinIn{sp, t0[i], t1[i], d_a3[slo_of[(size_t)i]]->p, d_a3v[slo_of[(size_t)i]]->p, &r});
                } else {   // (synchronised at its end: no event needed)
                    r.rc = win_detect_build(a, sp, t0[i], t1[i], a3[i], a3_valid[i], r, nullptr, precision);
                    if (r.rc != MR_OK && r.rc != MR_ERR_VALUE) err[(size_t)k] = a->err;
                }
            }
            if (!fast.empty()) {
                const int rc = win_chunk_build_async(a, fast.data(), (int)fast.size(), precision, cw[(size_t)task]);
                if (rc != MR_OK) {
                    err[(size_t)k] = a->err;
                    for (WinIn& f : fast) f.w->rc = rc;
                }
            }
            std::lock_guard<std::mutex> lk(mu);
            built[(size_t)group_of[(size_t)i0]] += i1 - i0;
            cv_done.notify_all();
        } else {           // spectra of up to MR_WS_BATCH windows, after their group's PageRanks
            WinPhase ph(3);   // (an event, not a host wait; one launch, a block per window)
            const std::vector<int32_t>& ids = spec[(size_t)~task];
            if (a != pr_ctx(group_of[(size_t)ids[0]]))   // (the PageRanks' own stream: in order already)
                (void)hipStreamWaitEvent(a->stream, gev[(size_t)group_of[(size_t)ids[0]]], 0);
            MrWsWin ws[MR_WS_BATCH];
            int nb = 0;
            std::vector<int32_t> general;
            for (int32_t i : ids) {
                const WinRun& r = w[(size_t)i];
                if (spec_general || !mr_win_spectrum_fits(r.ga->N, r.gn->N, spans[i]->n_podops, K)) {
                    general.push_back(i);
                    continue;
                }
                ws[nb++] = MrWsWin{r.ga->node_podop.p, r.ga->cov.p, r.gn->node_podop.p, r.gn->cov.p, r.ga->weight.p,
                                   r.gn->weight.p, slots.p + (size_t)i * MR_WS_SLOT, r.nn, r.na, r.ga->N,
                                   r.gn->N, spans[i]->n_podops};
            }
            if (nb) {
                const int rc = mr_win_spectrum_launch_n(a, ws, nb, method, K);
                for (int32_t i : ids)
                    if (std::find(general.begin(), general.end(), i) == general.end()) {
                        w[(size_t)i].rc = rc;
                        w[(size_t)i].slot = rc == MR_OK;
                    }
                if (rc != MR_OK) err[(size_t)k] = a->err;
            }
            for (int32_t i : general) {   // past the one-block limits: the general path (synchronous)
                WinRun& r = w[(size_t)i];
                r.rc = win_spectrum(a, spans[i], r, method, top_max,
                                    out_podop ? out_podop + (size_t)i * K : nullptr,
                                    out_score ? out_score + (size_t)i * K : nullptr, &n_out[i]);
                if (r.rc != MR_OK) err[(size_t)k] = a->err;
            }
        }
    };
    std::vector<std::thread> th;
    for (int k = 0; k < nthr; ++k)
        th.emplace_back([&, k] {
            mr_ctx* a = ctx->aux[(size_t)k];
            (void)hipSetDevice(a->device);
            for (;;) {
                int32_t task;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    WinPhase ph(4);
                    cv_task.wait(lk, [&] { return closed || !q.empty(); });
                    if (q.empty()) return;
                    task = q.front();
                    q.pop_front();
                }
                do_task(task, a, k);
            }
        });
    if (inl) {   // the one chunk, here
        {
            std::lock_guard<std::mutex> lk(mu);
            q.clear();
        }
        do_task(0, ctx, 0);
    }
    int rc = MR_OK;
    // the previous call's graphs go back to their pools on a thread of their own (their streams
    // finished with them before that call returned; ~8 us of pool bookkeeping per graph had been
    // ~1 ms at the end of every 64-window call)
    std::vector<mr_graph*> dead;
    dead.swap(ctx->graveyard);
    std::thread reaper;
    // (a few graphs: here, on the calling thread.  The inline chunk's build is already enqueued
    // above, so this runs after it was issued, not before; it is safe because the previous call
    // drained these graphs' streams before it returned, and the blocks go back to stream-ordered
    // pools)
    if (inl && dead.size() <= 64) {
        for (mr_graph* g : dead) delete g;
        dead.clear();
    } else {
        reaper = std::thread([&dead] {
            for (mr_graph* g : dead) delete g;
        });
    }
    // Each group's PageRanks are enqueued without their closing read-back (mr_pagerank_batch_async),
    // so the next group's go in behind them while they run: the PageRank stream no longer idles
    // while this thread waits for a group and then enqueues the next (measured: this thread had
    // spent 12 of a C2 call's 14.5 ms inside the synchronous batch).  A group's error words are
    // read one group later; only then are its spectra queued (a kind-hash collision reruns the
    // group synchronously first).
    {
        const size_t need = (size_t)8 * n_windows;   // 4 words per graph, 2 graphs per window
        if (ctx->pin_flags_n < need) {
            if (ctx->pin_flags) (void)hipHostFree(ctx->pin_flags);
            ctx->pin_flags = nullptr;
            ctx->pin_flags_n = 0;
            if (hipHostMalloc((void**)&ctx->pin_flags, need * sizeof(int32_t), hipHostMallocDefault) != hipSuccess)
                rc = mr_fail(ctx, MR_ERR_OOM, "mr_windows_batch: pinned error words");
            else
                ctx->pin_flags_n = need;
        }
    }
    std::vector<PrAsync*> pend((size_t)ngroups, nullptr);
    std::vector<std::vector<mr_graph*>> ggs((size_t)ngroups);
    std::vector<std::vector<int>> gan((size_t)ngroups);
    auto record = [&](int g) -> int {
        if (!gev[(size_t)g] && hipEventCreateWithFlags(&gev[(size_t)g], hipEventDisableTiming) != hipSuccess) return MR_ERR_HIP;
        return hipEventRecord(gev[(size_t)g], pr_ctx(g)->stream) == hipSuccess ? MR_OK : MR_ERR_HIP;
    };
    // (early spectra: their slots' read-back is queued behind them too, before the words are read;
    // a rerun's spectra clear this and the read-back is queued again at the end)
    const size_t slot_bytes = (size_t)n_windows * MR_WS_SLOT;
    bool slots_queued = false;
    // spectrum tasks of up to MR_WS_BATCH ranked windows of group g: task ~i = list spec[i]
    auto queue_spectra = [&](int g) {   // (under mu)
        const int32_t i0 = gbeg[(size_t)g], i1 = gbeg[(size_t)g + 1];
        int32_t head = -1;
        for (int32_t i = i0; i < i1; ++i) {
            spec[(size_t)i].clear();
            if (w[(size_t)i].rc != MR_OK || !w[(size_t)i].gn) continue;
            if (head < 0 || (int)spec[(size_t)head].size() == spec_batch) {
                if (head >= 0) q.push_back(~head);
                head = i;
            }
            spec[(size_t)head].push_back(i);
        }
        if (head >= 0) q.push_back(~head);
    };
    // group g's results are final: check its words (rerun on a collision) and queue its spectra
    // (early: they went in behind the PageRanks already, again only after a rerun)
    auto settle = [&](int g, bool early) -> int {
        int r = MR_OK;
        bool reran = false;
        if (pend[(size_t)g]) {
            mr_ctx* pc = pr_ctx(g);
            bool rerun = false;
            r = mr_pagerank_async_finish(pc, pend[(size_t)g], &rerun);
            mr_pagerank_async_free(pend[(size_t)g]);
            pend[(size_t)g] = nullptr;
            if (r == MR_OK && rerun) {
                r = mr_pagerank_batch(pc, ggs[(size_t)g].data(), gan[(size_t)g].data(), (int)ggs[(size_t)g].size(), 0.85,
                                      0.01, 25, precision, 0);
                if (r == MR_OK) r = record(g);
                reran = true;
            }
            if (r != MR_OK && pc != ctx) ctx->err = pc->err;
        }
        std::lock_guard<std::mutex> lk(mu);
        if (r == MR_OK && (!early || reran)) queue_spectra(g);
        if (reran) slots_queued = false;
        cv_task.notify_all();
        return r;
    };
    // a call of one chunk (inline, one group): its spectra go in behind its PageRanks before their
    // words are read, so the host's wait for the words no longer sits between the two on the GPU
    // (C2 one window: a ~20 us idle gap plus the spectrum's launch).  A collision rerun overwrites
    // the slots with a second round of spectra.  MR_WIN_SPEC_EARLY=0: after the words (read per call)
    const char* see = getenv("MR_WIN_SPEC_EARLY");
    const bool spec_early = inl && !(see && atoi(see) == 0);
    int settled = 0;   // groups whose spectra are queued
    // (the next group's builds run beside a group's iterations: the iterations run ~20 % slower
    // than alone, but a call that builds every window before the first iterations ranked 3.5 %
    // fewer windows per second, profiles/r06/r06h_serial_priority_ab.txt)
    for (int g = 0; g < ngroups && rc == MR_OK; ++g) {
        const int32_t i0 = gbeg[(size_t)g], i1 = gbeg[(size_t)g + 1];
        {
            std::unique_lock<std::mutex> lk(mu);
            WinPhase ph(5);
            cv_done.wait(lk, [&] { return built[(size_t)g] == i1 - i0; });
        }
        mr_ctx* pc = pr_ctx(g);
        for (size_t c = 0; c < chunks.size(); ++c)   // the group's chunks' graphs are ready
            if (chunks[c].first >= i0 && chunks[c].first < i1 && cw[c].ev &&
                hipStreamWaitEvent(pc->stream, cw[c].ev, 0) != hipSuccess)
                rc = mr_fail(ctx, MR_ERR_HIP, "mr_windows_batch: hipStreamWaitEvent failed");   // (threads joined below)
        if (rc != MR_OK) break;
        std::vector<mr_graph*>& gs = ggs[(size_t)g];
        std::vector<int>& anom = gan[(size_t)g];
        for (int32_t i = i0; i < i1; ++i) {
            WinRun& r = w[(size_t)i];
            n_out[i] = 0;
            if (r.rc == MR_OK && r.gn) {
                r.gn->ctx = r.ga->ctx = pc;   // (built on an auxiliary context)
                gs.push_back(r.gn);
                gs.push_back(r.ga);
                anom.push_back(0);
                anom.push_back(1);
            }
        }
        if (!gs.empty()) {
            WinPhase ph(6);
            rc = mr_pagerank_batch_async(pc, gs.data(), anom.data(), (int)gs.size(), 0.85, 0.01, 25, precision,
                                         ctx->pin_flags + (size_t)8 * i0, &pend[(size_t)g], spec_early);
            if (rc != MR_OK && pc != ctx) ctx->err = pc->err;
        }
        // (early spectra: they follow on this stream, so no event between them and the iterations;
        // the error words' copy and its event go in behind them)
        if (rc == MR_OK && !spec_early) rc = record(g);
        if (rc == MR_OK && spec_early) {
            {
                std::lock_guard<std::mutex> lk(mu);
                queue_spectra(g);
            }
            for (;;) {   // (inline: this thread is the only worker)
                int32_t task;
                {
                    std::lock_guard<std::mutex> lk(mu);
                    if (q.empty()) break;
                    task = q.front();
                    q.pop_front();
                }
                do_task(task, ctx, 0);
            }
            if (pend[(size_t)g]) rc = mr_pagerank_async_commit(pc, pend[(size_t)g]);
            if (rc == MR_OK && slot_bytes <= MR_PIN_BYTES) {
                if (!ctx->pin && hipHostMalloc((void**)&ctx->pin, MR_PIN_BYTES, hipHostMallocDefault) != hipSuccess)
                    ctx->pin = nullptr;
                slots_queued = ctx->pin && hipMemcpyAsync(ctx->pin, slots.p, slot_bytes, hipMemcpyDeviceToHost,
                                                          ctx->stream) == hipSuccess;
            }
        }
        // the previous group's words are in by now, or nearly: settle it (this one stays in flight)
        for (; rc == MR_OK && settled < g; ++settled) rc = settle(settled, spec_early);
    }
    for (; rc == MR_OK && settled < ngroups; ++settled) rc = settle(settled, spec_early);
    while (inl && rc == MR_OK) {   // the spectra settle queued, here
        int32_t task;
        {
            std::lock_guard<std::mutex> lk(mu);
            if (q.empty()) break;
            task = q.front();
            q.pop_front();
        }
        do_task(task, ctx, 0);
    }
    if (rc != MR_OK) {   // (an error left groups in flight)
        (void)hipStreamSynchronize(ctx->stream);
    }
    for (PrAsync* a : pend)
        if (a) mr_pagerank_async_free(a);
    {
        std::lock_guard<std::mutex> lk(mu);
        closed = true;
        cv_task.notify_all();
    }
    std::unique_ptr<WinPhase> ph_tail(new WinPhase(7));
    for (auto& t : th) t.join();
    if (reaper.joinable()) reaper.join();
    for (int k = 0; k < nthr; ++k) (void)hipStreamSynchronize(ctx->aux[(size_t)k]->stream);
    // every device-slot spectrum in one read-back: queued on this stream into the pinned buffer
    // when it fits (one window: ~30 us less than a synchronous pageable copy after the drain)
    bool slots_pinned = slots_queued && rc == MR_OK;
    if (rc == MR_OK && !slots_pinned && slot_bytes <= MR_PIN_BYTES) {
        if (!ctx->pin && hipHostMalloc((void**)&ctx->pin, MR_PIN_BYTES, hipHostMallocDefault) != hipSuccess) ctx->pin = nullptr;
        slots_pinned = ctx->pin && hipMemcpyAsync(ctx->pin, slots.p, slot_bytes, hipMemcpyDeviceToHost, ctx->stream) == hipSuccess;
    }
    // (an error may leave PageRank work queued on the main stream that still reads window graphs
    // whose blocks return to the worker pools below: drain it first)
    (void)hipStreamSynchronize(ctx->stream);
    for (hipEvent_t e : gev)
        if (e) (void)hipEventDestroy(e);
    MR_TRY(rc);
    for (auto& e : err)
        if (!e.empty()) return mr_fail(ctx, MR_ERR_HIP, "mr_windows_batch: %s", e.c_str());
    {
        std::vector<unsigned char> hv;
        const unsigned char* hs = (const unsigned char*)ctx->pin;
        if (!slots_pinned) {
            hv.resize(slot_bytes);
            MR_TRY_HIP(ctx, hipMemcpy(hv.data(), slots.p, slot_bytes, hipMemcpyDeviceToHost));
            hs = hv.data();
        }
        for (int32_t i = 0; i < n_windows; ++i)
            if (w[(size_t)i].slot)
                mr_win_spectrum_unpack(hs + (size_t)i * MR_WS_SLOT, out_podop ? out_podop + (size_t)i * K : nullptr,
                                       out_score ? out_score + (size_t)i * K : nullptr, &n_out[i]);
    }
    for (int32_t i = 0; i < n_windows; ++i) {
        const WinRun& r = w[(size_t)i];
        status[i] = r.rc;
        if (edges_traversed) edges_traversed[i] = r.rc == MR_OK ? win_edges(r) : 0;
        if (n_abnormal) n_abnormal[i] = r.na;
        if (n_normal) n_normal[i] = r.nn;
    }
    // large windows' graphs (>= 64k traces per window on average: C2) are released during the next
    // call (C2 +8 %); small windows' (C3: many graphs, many small blocks) here, on the call's exit --
    // the reaper's pool traffic beside the next call's builds measured -17 % there.
    // MR_WIN_REAP=0 / 1: never / always (read per call)
    const char* ke = getenv("MR_WIN_REAP");
    int64_t tsum = 0, nw = 0;
    for (const WinRun& r : w)
        if (r.gn) {
            tsum += (int64_t)r.gn->T + r.ga->T;
            ++nw;
        }
    const bool reap = ke ? strcmp(ke, "0") != 0 : nw > 0 && tsum >= (int64_t)65536 * nw;
    if (reap)
        for (WinRun& r : w) {   // (every stream is idle here: released during the next call)
            if (r.gn) ctx->graveyard.push_back(r.gn);
            if (r.ga) ctx->graveyard.push_back(r.ga);
            r.gn = r.ga = nullptr;
        }
    ph_tail.reset();
    if (timing) {
        {
            WinPhase ph(9);
            for (WinRun& r : w) {
                delete r.gn;
                delete r.ga;
                r.gn = r.ga = nullptr;
            }
        }
        fprintf(stderr, "[mr_windows_batch] %d windows, %.3f ms:", n_windows, (win_now() - t_call) * 1e-6);
        for (int i = 0; i < 10; ++i) fprintf(stderr, " %s %.3f ms;", WIN_PHASE_NAME[i], g_phases->ns[i] * 1e-6);
        fprintf(stderr, "\n");
        g_phases = nullptr;
    }
    return MR_OK;
}
