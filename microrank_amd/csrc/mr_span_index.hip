// Per-trace index of an uploaded span table, built once per table (mr_spans_upload) so that the
// per-window work of online_rca.online_anomaly_detect_RCA (online_rca.py:164-215) never sorts
// span rows again.  From one stable sort of the rows by (trace, code) it keeps, per trace:
//   * distinct pod-ops (podName_operationName, preprocess_data.py:151-155) with span count and
//     first row -> len_o, trace_num_list, node order and the trace-major incidence of
//     get_pagerank_graph (:146-171) for any trace subset;
//   * distinct service-ops with span count -> the detector's expect sum in name order
//     (anormaly_detector.py:56-67, preprocess_data.py:97-122);
//   * the parent join ParentSpanId == spanID (:157-159) resolved once: distinct (parent op,
//     child op) keys with multiplicity for pairs inside the trace, and the rare pairs whose
//     rows lie in different traces (T11) kept as a flat list;
//   * span count, max duration, trace-level start/end, and whether start/end are constant over
//     the trace's rows (then a time window selects whole traces and the window detector is a
//     per-trace pass; otherwise the row-level path runs).
// The index is a derived view of the uploaded columns: no result depends on it being present.
#include <algorithm>
#include <climits>
#include <cstring>

#include "mr_detect_dev.h"
#include "mr_prim.h"
#include "mr_sort.h"

namespace {
constexpr int XB = 256;

__global__ void k_ix_keys(const int32_t* trace, const int32_t* code, int64_t S, int nbc, uint64_t* key, uint32_t* val) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S) return;
    key[i] = ((uint64_t)(uint32_t)trace[i] << nbc) | (uint32_t)code[i];
    val[i] = (uint32_t)i;
}
__global__ void k_ix_heads(const uint64_t* key, int64_t n, int32_t* head) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) head[i] = (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}
// run r = (trace, code): code, first row (stable sort: the smallest), start position; one
// per-trace run count for the trace offsets
__global__ void k_ix_runs(const uint64_t* key, const uint32_t* val, const int32_t* head, const int64_t* hpos, int64_t n,
                          int nbc, int32_t* r_code, int32_t* r_first, int32_t* r_tr, int64_t* r_start, int32_t* truns) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !head[i]) return;
    const int64_t r = hpos[i];
    const uint64_t k = key[i];
    const int32_t t = (int32_t)(k >> nbc);
    r_code[r] = (int32_t)(k & ((1ull << nbc) - 1ull));
    if (r_first) r_first[r] = (int32_t)val[i];
    if (r_tr) r_tr[r] = t;
    r_start[r] = i;
    atomicAdd(&truns[t], 1);
}
__global__ void k_ix_map_rows(int32_t* first, int64_t n, const int32_t* grow) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < n) first[r] = grow[first[r]];
}
__global__ void k_ix_cnt(const int64_t* r_start, int64_t R, int64_t n, int32_t* r_cnt) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < R) r_cnt[r] = (int32_t)((r + 1 < R ? r_start[r + 1] : n) - r_start[r]);
}
// per-trace scalars: rows, max duration, min/max of trace-level start and end
// (rows of a trace are mostly adjacent: lanes of one trace are combined over the wave first and
// the run's last lane alone updates the trace; runs of one trace split over waves merge exactly)
__global__ void k_ix_trace_stats(const int32_t* trace, const int64_t* dur, const int64_t* ts, const int64_t* te, int64_t S,
                                 int32_t* tlen, long long* tmaxd, long long* tsmin, long long* tsmax, long long* temin,
                                 long long* temax) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = i < S;
    const int32_t t = in ? trace[i] : -1;
    int32_t n = in ? 1 : 0;
    long long md = in ? (long long)dur[i] : LLONG_MIN;
    long long s0 = in && ts ? (long long)ts[i] : LLONG_MAX, s1 = in && ts ? (long long)ts[i] : LLONG_MIN;
    long long e0 = in && ts ? (long long)te[i] : LLONG_MAX, e1 = in && ts ? (long long)te[i] : LLONG_MIN;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {   // inclusive segmented scan over runs of equal t
        const int32_t to = __shfl_up(t, off, 64);
        const int32_t no = __shfl_up(n, off, 64);
        const long long mo = __shfl_up(md, off, 64), a0 = __shfl_up(s0, off, 64), a1 = __shfl_up(s1, off, 64),
                        b0 = __shfl_up(e0, off, 64), b1 = __shfl_up(e1, off, 64);
        if (lane >= off && to == t) {
            n += no;
            md = max(md, mo);
            s0 = min(s0, a0);
            s1 = max(s1, a1);
            e0 = min(e0, b0);
            e1 = max(e1, b1);
        }
    }
    const int32_t tn = __shfl_down(t, 1, 64);
    if (!in || (lane != 63 && tn == t)) return;
    atomicAdd(&tlen[t], n);
    atomicMax(&tmaxd[t], md);
    if (ts) {
        atomicMin(&tsmin[t], s0);
        atomicMax(&tsmax[t], s1);
        atomicMin(&temin[t], e0);
        atomicMax(&temax[t], e1);
    }
}
__global__ void k_ix_uniform(const int32_t* tlen, const long long* tsmin, const long long* tsmax, const long long* temin,
                             const long long* temax, int32_t NT, int32_t* bad) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < NT && tlen[t] > 0 && (tsmin[t] != tsmax[t] || temin[t] != temax[t])) atomicOr(bad, 1);
}
// parent join, pass 1: number of internal / cross-trace (child row, parent row) pairs per row
__global__ void k_ix_join_count(const int32_t* trace, const int64_t* parent, int64_t S, const int64_t* id_off,
                                const int32_t* id_rows, int64_t n_codes, int32_t* nin, int32_t* nx) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= S) return;
    int32_t a = 0, b = 0;
    const int64_t p = parent[c];
    if (p >= 0 && p < n_codes) {
        const int32_t tc = trace[c];
        for (int64_t e = id_off[p]; e < id_off[p + 1]; ++e) {
            if (trace[id_rows[e]] == tc) ++a; else ++b;
        }
    }
    nin[c] = a;
    nx[c] = b;
}
// pass 2: internal pairs as sort keys (trace, parent op, child op); cross pairs listed
__global__ void k_ix_join_fill(const int32_t* trace, const int32_t* podop, const int64_t* parent, int64_t S,
                               const int64_t* id_off, const int32_t* id_rows, int64_t n_codes, const int64_t* pin,
                               const int64_t* px, int nbp, uint64_t* ikey, int32_t* xtc, int32_t* xtp, uint64_t* xkey) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= S) return;
    const int64_t p = parent[c];
    if (p < 0 || p >= n_codes) return;
    const int32_t tc = trace[c];
    const uint32_t oc = (uint32_t)podop[c];
    int64_t a = pin[c], b = px[c];
    for (int64_t e = id_off[p]; e < id_off[p + 1]; ++e) {
        const int32_t j = id_rows[e];
        const uint32_t op = (uint32_t)podop[j];
        if (trace[j] == tc) {
            ikey[a++] = ((uint64_t)(uint32_t)tc << (2 * nbp)) | ((uint64_t)op << nbp) | oc;
        } else {
            xtc[b] = tc;
            xtp[b] = trace[j];
            xkey[b] = ((uint64_t)op << 32) | oc;
            ++b;
        }
    }
}
// (parent << 32 | child) -> (parent << nbp | child), internal keys then cross keys
__global__ void k_ix_pack_keys(const uint64_t* ed_key, int64_t n_ed, const uint64_t* xj_key, int64_t n_xj, int nbp,
                               uint64_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_ed + n_xj) return;
    const uint64_t k = i < n_ed ? ed_key[i] : xj_key[i - n_ed];
    out[i] = ((k >> 32) << nbp) | (k & 0xffffffffull);
}
// the distinct edge keys (heads of the sorted packed keys) as (parent << 32 | child), ascending
__global__ void k_ix_ekeys(const uint64_t* key, const int32_t* head, const int64_t* hpos, int64_t n, int nbp,
                           uint64_t* ekey) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !head[i]) return;
    const uint64_t k = key[i], m = (1ull << nbp) - 1ull;
    ekey[hpos[i]] = ((k >> nbp) << 32) | (k & m);
}
// dense edge id of each key: its position among the distinct keys (binary search)
// the edge entries in edge-id order (mr_spans.eb_*): sort keys = the ids, values = the entry
__global__ void k_ix_eb_keys(const int32_t* eid, int64_t n, uint64_t* key, uint32_t* val) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    key[i] = (uint64_t)(uint32_t)eid[i];
    val[i] = (uint32_t)i;
}
__global__ void k_ix_eb_gather(const uint64_t* key, const uint32_t* val, int64_t n, const int32_t* ed_tr,
                               const int32_t* ed_cnt, int32_t* eb_tr, int32_t* eb_cnt, int32_t* eb_eid) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t r = val[i];
    eb_tr[i] = ed_tr[r];
    eb_cnt[i] = ed_cnt[r];
    eb_eid[i] = (int32_t)key[i];
}
__global__ void k_ix_eid(const uint64_t* key, int64_t n, const uint64_t* ekey, int64_t E, int32_t* eid) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = key[i];
    int64_t lo = 0, hi = E;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (ekey[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    eid[i] = (int32_t)lo;
}
__global__ void k_ix_edge_runs(const uint64_t* key, const int32_t* head, const int64_t* hpos, int64_t n, int nbp,
                               uint64_t* ed_key, int32_t* ed_tr, int64_t* r_start, int32_t* truns) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !head[i]) return;
    const int64_t r = hpos[i];
    const uint64_t k = key[i];
    const uint64_t m = (1ull << nbp) - 1ull;
    const int32_t t = (int32_t)(k >> (2 * nbp));
    ed_key[r] = (((k >> nbp) & m) << 32) | (k & m);
    ed_tr[r] = t;
    r_start[r] = i;
    atomicAdd(&truns[t], 1);
}

// ---------------------------------------------------------------- layout order (lo_index)
// the set hash of each trace's kind key (pagerank.py:54-66: op set, fp32(1/len_t), count;
// order-free), read from the trace's pod-op runs in code order
__device__ __forceinline__ uint64_t lo_mix(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ float lo_w(int32_t len) { return len > 0 ? (float)(1.0 / (double)len) : 0.0f; }
__global__ void k_lo_hash(const int64_t* po_off, const int32_t* po_op, const int32_t* tlen, int32_t NT, uint64_t seed,
                          uint64_t* hkey, uint32_t* tr) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= NT) return;
    const int64_t o = po_off[t], n = po_off[t + 1] - o;
    uint64_t acc = 0;
    for (int64_t e = 0; e < n; ++e) acc += lo_mix((uint64_t)po_op[o + e] ^ seed);
    hkey[t] = lo_mix(lo_mix(seed ^ (uint64_t)__float_as_uint(lo_w(tlen[t])) ^ ((uint64_t)n << 32)) + acc);
    tr[t] = (uint32_t)t;
}
// (sorted by hash, stably: trace codes ascending within a hash) key = count << nbt | hash rank
__global__ void k_lo_keys(const uint32_t* tr_h, const int64_t* po_off, int32_t NT, int nbt, uint64_t* key) {
    const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= NT) return;
    const uint32_t t = tr_h[j];
    key[j] = ((uint64_t)(po_off[t + 1] - po_off[t]) << nbt) | (uint32_t)j;
}
// layout index i: the trace, its entry count and span count; head: a new (count, hash) run
__global__ void k_lo_unpack(const uint64_t* key, const uint32_t* tr_h, const uint64_t* hkey_h, int32_t NT, int nbt,
                            const int32_t* tlen, int32_t* lo_tr, int32_t* lo_n, int32_t* lo_len, int32_t* head) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= NT) return;
    const uint64_t m = (1ull << nbt) - 1ull, k = key[i];
    const uint32_t j = (uint32_t)(k & m);
    const int32_t t = (int32_t)tr_h[j];
    lo_tr[i] = t;
    lo_n[i] = (int32_t)(k >> nbt);
    lo_len[i] = tlen[t];
    bool h = i == 0;
    if (!h) {
        const uint64_t kp = key[i - 1];
        h = (kp >> nbt) != (k >> nbt) || hkey_h[(uint32_t)(kp & m)] != hkey_h[j];
    }
    head[i] = h ? 1 : 0;
}
// each trace's entries into its layout slot (code order): pod-op codes / span counts / first rows,
// its detector scalars, and its service-op and join entry counts (the copies below); bad: a count
// or code past the 16-bit packing (the table then keeps the general window path)
__global__ void k_lo_copy(const int32_t* lo_tr, const int64_t* lo_off, int32_t NT, const int64_t* po_off,
                          const int32_t* po_op, const int32_t* po_cnt, const int32_t* po_first, const long long* tts,
                          const long long* tte, const long long* tmaxd, const int64_t* sv_off, const int64_t* ed_off,
                          uint16_t* lo16, uint16_t* lo_cnt, int32_t* lo_first, long long* lo_ts, long long* lo_te,
                          long long* lo_mx, int32_t* nsv, int32_t* ned, int32_t* bad) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= NT) return;
    const int32_t t = lo_tr[i];
    const int64_t a = po_off[t], n = po_off[t + 1] - a, o = lo_off[i];
    bool big = false;
    for (int64_t e = 0; e < n; ++e) {
        const int32_t c = po_cnt[a + e];
        big = big || c > 65535;
        lo16[o + e] = (uint16_t)po_op[a + e];
        lo_cnt[o + e] = (uint16_t)c;
        lo_first[o + e] = po_first[a + e];
    }
    lo_ts[i] = tts[t];
    lo_te[i] = tte[t];
    lo_mx[i] = tmaxd[t];
    nsv[i] = (int32_t)(sv_off[t + 1] - sv_off[t]);
    ned[i] = (int32_t)(ed_off[t + 1] - ed_off[t]);
    if (big) atomicOr(bad, 1);
}
__global__ void k_lo_copy2(const int32_t* lo_tr, int32_t NT, const int64_t* sv_off, const int32_t* sv_op,
                           const int32_t* sv_cnt, const int64_t* ed_off, const int32_t* ed_eid, const int32_t* ed_cnt,
                           const int64_t* lsv_off, const int64_t* le_off, uint32_t* lsv, uint32_t* le, int32_t* bad) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= NT) return;
    const int32_t t = lo_tr[i];
    bool big = false;
    for (int64_t e = sv_off[t], o = lsv_off[i]; e < sv_off[t + 1]; ++e, ++o) {
        const int32_t op = sv_op[e], c = sv_cnt[e];
        big = big || op > 65535 || c > 65535;
        lsv[o] = (uint32_t)(uint16_t)op | ((uint32_t)(uint16_t)c << 16);
    }
    for (int64_t e = ed_off[t], o = le_off[i]; e < ed_off[t + 1]; ++e, ++o) {
        const int32_t id = ed_eid[e], c = ed_cnt[e];
        big = big || id > 65535 || c > 65535;
        le[o] = (uint32_t)(uint16_t)id | ((uint32_t)(uint16_t)c << 16);
    }
    if (big) atomicOr(bad, 1);
}
// classes = the (count, hash) runs of the layout: class id = the run's index; every member is
// compared exactly with the run's first trace (its span-count weight and op list)
__global__ void k_lo_reps(const int32_t* head, const int64_t* hpos, int32_t NT, int32_t* rep) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < NT && head[i]) rep[hpos[i]] = i;
}
__global__ void k_lo_classes(const int32_t* head, const int64_t* hpos, const int32_t* rep, int32_t NT,
                             const int64_t* lo_off, const uint16_t* lo16, const int32_t* lo_len, int32_t* lo_kid,
                             int32_t* bad) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= NT) return;
    const int32_t k = (int32_t)hpos[i] + head[i] - 1, r = rep[k];
    lo_kid[i] = k;
    if (r == i) return;
    const int64_t a = lo_off[i], n = lo_off[i + 1] - a, b = lo_off[r];
    bool eq = n == lo_off[r + 1] - b && __float_as_uint(lo_w(lo_len[i])) == __float_as_uint(lo_w(lo_len[r]));
    for (int64_t e = 0; eq && e < n; ++e) eq = lo16[a + e] == lo16[b + e];
    if (!eq) atomicOr(bad, 1);
}

// ---------------------------------------------------------------- window detector (uniform times)
// (the per-block body: mr_detect_dev.h)
__global__ void __launch_bounds__(DB) k_ix_detect(int32_t NT, DetIn d) {
    __shared__ double term[DB * DCAP];
    (void)detect_block(NT, d, term);
}

// ---------------------------------------------------------------- the driver's window sweep (f3)
// online_rca.py:161-216 visits windows [t_begin + m*grain, + window] (m a whole number of grains:
// the steps of 5 and 5 + 4 minutes are multiples of one minute).  With trace-level times constant
// inside each trace a window selects whole traces and a trace's partition (abnormal / normal /
// dropped) does not depend on the window: its rows are all in or all out, and real and expect are
// sums over its own rows.  So each trace is classified ONCE and adds itself to the contiguous
// range of window starts that contain it:
//   t_begin + m*grain <= ts  and  te <= t_begin + m*grain + window
//   <=>  ceil((te - window - t_begin) / grain) <= m <= floor((ts - t_begin) / grain),
// as +1 / -1 at the range ends of three difference arrays (abnormal, normal, in-window rows);
// a prefix sum over m then gives every window's detector counts.
__device__ __forceinline__ int64_t floor_div(int64_t a, int64_t b) {   // b > 0
    const int64_t q = a / b;
    return (a % b != 0 && a < 0) ? q - 1 : q;
}
constexpr int SWB = 256, SWT = 16;        // threads per block, traces per thread
constexpr int SW_LDS = 4096;              // window starts histogrammed in LDS (else global atomics)
__global__ void __launch_bounds__(SWB) k_ix_sweep(int32_t NT, const int32_t* tlen, const long long* tts,
                                                  const long long* tte, const long long* tmaxd, const int64_t* sv_off,
                                                  const int32_t* sv_op, const int32_t* sv_cnt, const double* a3,
                                                  const uint8_t* a3v, int64_t t_begin, int64_t grain, int64_t window,
                                                  int32_t M, uint8_t* state, unsigned long long* diff) {
    __shared__ uint32_t h[3 * (SW_LDS + 1)];
    const bool lds = M + 1 <= SW_LDS + 1;
    if (lds)
        for (int i = threadIdx.x; i < 3 * (M + 1); i += SWB) h[i] = 0;
    __syncthreads();
    const int32_t tb = blockIdx.x * SWB * SWT;
    for (int j = 0; j < SWT; ++j) {
        const int32_t t = tb + j * SWB + threadIdx.x;
        if (t >= NT) break;
        int st = 0;
        const int32_t n = tlen[t];
        if (n > 0) {
            const long long mx = tmaxd[t];
            if (mx > 0) {   // grouped[grouped['duration'] > 0] (preprocess_data.py:117)
                double expect = 0.0;
                for (int64_t r = sv_off[t]; r < sv_off[t + 1]; ++r) {   // name order, no FMA (T14)
                    const int32_t op = sv_op[r];
                    if (a3v[op]) expect += (double)sv_cnt[r] * a3[op];  // anormaly_detector.py:64-65
                }
                st = (double)mx / 1000.0 > expect ? 2 : 1;            // :58, :69
            }
            state[t] = (uint8_t)st;
            const int64_t hi = floor_div((int64_t)tts[t] - t_begin, grain);
            const int64_t lo = max((int64_t)0, -floor_div(window + t_begin - (int64_t)tte[t], grain));   // ceil
            if (hi >= lo && lo < M && hi >= 0) {
                const int32_t a = (int32_t)lo, b = (int32_t)min(hi + 1, (int64_t)M);
                // counters: 0 abnormal, 1 normal (a dropped trace counts only its rows), 2 rows
                if (lds && n <= 65536) {   // (a block's partial stays below 2^31 in magnitude)
                    if (st) {
                        atomicAdd(&h[(st == 2 ? 0 : 1) * (M + 1) + a], 1u);
                        atomicSub(&h[(st == 2 ? 0 : 1) * (M + 1) + b], 1u);
                    }
                    atomicAdd(&h[2 * (M + 1) + a], (uint32_t)n);
                    atomicSub(&h[2 * (M + 1) + b], (uint32_t)n);
                } else if (lds) {
                    if (st) {
                        atomicAdd(&h[(st == 2 ? 0 : 1) * (M + 1) + a], 1u);
                        atomicSub(&h[(st == 2 ? 0 : 1) * (M + 1) + b], 1u);
                    }
                    atomicAdd(&diff[(size_t)2 * (M + 1) + a], (unsigned long long)n);
                    atomicAdd(&diff[(size_t)2 * (M + 1) + b], (unsigned long long)(-(int64_t)n));
                } else {
                    if (st) {
                        atomicAdd(&diff[(size_t)(st == 2 ? 0 : 1) * (M + 1) + a], 1ull);
                        atomicAdd(&diff[(size_t)(st == 2 ? 0 : 1) * (M + 1) + b], ~0ull);   // -1 mod 2^64
                    }
                    atomicAdd(&diff[(size_t)2 * (M + 1) + a], (unsigned long long)n);
                    atomicAdd(&diff[(size_t)2 * (M + 1) + b], (unsigned long long)(-(int64_t)n));
                }
            }
        } else {
            state[t] = 0;
        }
    }
    if (!lds) return;
    __syncthreads();
    // per-block counts are exact mod 2^32; the sign-extended flush keeps the global sums exact
    for (int i = threadIdx.x; i < 3 * (M + 1); i += SWB)
        if (h[i]) atomicAdd(&diff[i], (unsigned long long)(int64_t)(int32_t)h[i]);
}
}  // namespace

// (trace, code) runs of the rows: offsets per trace, code, count and (optionally) first row
static int trace_runs(mr_ctx* ctx, const mr_spans* s, const int32_t* code, int32_t n_codes, DBuf<int64_t>& off,
                      DBuf<int32_t>& r_code, DBuf<int32_t>& r_cnt, DBuf<int32_t>* r_first, DBuf<int32_t>* r_tr,
                      int64_t* n_runs) {
    hipStream_t st = ctx->stream;
    const int64_t S = s->S;
    const int32_t NT = s->n_traces;
    const int nbc = std::max(1, bits_for((uint64_t)std::max(n_codes - 1, 0)));
    DBuf<uint64_t> key;
    DBuf<uint32_t> val;
    DBuf<int32_t> head, truns;
    DBuf<int64_t> hpos, tmp, r_start;
    MR_TRY(key.alloc(ctx, S));
    MR_TRY(val.alloc(ctx, S));
    MR_TRY(head.alloc(ctx, S));
    MR_TRY(hpos.alloc(ctx, S + 1));
    MR_TRY(tmp.alloc(ctx, std::max(scan_tmp_elems(S), scan_tmp_elems(NT))));
    MR_TRY(truns.zero(ctx, NT));
    hipLaunchKernelGGL(k_ix_keys, dim3(cdiv(S, XB)), dim3(XB), 0, st, s->trace.p, code, S, nbc, key.p, val.p);
    SortScratch ws;
    MR_TRY(mr_radix_sort(ctx, key.p, val.p, S, nbc + bits_for((uint64_t)std::max(NT - 1, 0)), ws));
    hipLaunchKernelGGL(k_ix_heads, dim3(cdiv(S, XB)), dim3(XB), 0, st, key.p, S, head.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, head.p, hpos.p, S, tmp.p));
    int64_t R = 0;
    MR_TRY_HIP(ctx, hipMemcpyAsync(&R, hpos.p + S, sizeof R, hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    MR_TRY(r_code.alloc(ctx, R));
    MR_TRY(r_cnt.alloc(ctx, R));
    MR_TRY(r_start.alloc(ctx, R));
    if (r_first) MR_TRY(r_first->alloc(ctx, R));
    if (r_tr) MR_TRY(r_tr->alloc(ctx, R));
    hipLaunchKernelGGL(k_ix_runs, dim3(cdiv(S, XB)), dim3(XB), 0, st, key.p, val.p, head.p, hpos.p, S, nbc, r_code.p,
                       r_first ? r_first->p : nullptr, r_tr ? r_tr->p : nullptr, r_start.p, truns.p);
    hipLaunchKernelGGL(k_ix_cnt, dim3(cdiv(std::max<int64_t>(R, 1), XB)), dim3(XB), 0, st, r_start.p, R, S, r_cnt.p);
    MR_TRY(off.alloc(ctx, (size_t)NT + 1));
    MR_TRY(mr_exclusive_scan_i32(ctx, truns.p, off.p, NT, tmp.p));
    MR_TRY_HIP(ctx, hipGetLastError());
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // scratch is freed on return
    *n_runs = R;
    return MR_OK;
}

// The table's layout order, u16 code lists and exact kind classes (mr_spans.lo_*): window graphs
// of tables within the one-pass limits tile from them (mr_lo_launch_batch).  Layout order: distinct
// pod-op count, then kind hash, then code -- a kind class is a contiguous run of the layout (its id
// the run's index), so a window counts a run's members with one add per wave.  A hash collision
// that the exact comparison finds retries with the next seed; after four the table keeps the
// general window path (lo_ok false).
static int lo_index_try(mr_ctx* ctx, mr_spans* s) {
    hipStream_t st = ctx->stream;
    const int32_t NT = s->n_traces;
    s->lo_ok = false;
    if (getenv("MR_LO_TEST_FAIL")) {   // (tests, read per table: an allocation failing half-way)
        MR_TRY(s->lo_tr.alloc(ctx, (size_t)std::max(NT, 1)));
        return mr_fail(ctx, MR_ERR_HIP, "lo_index: forced failure (MR_LO_TEST_FAIL)");
    }
    if (!mr_lo_fits(s) || s->n_po >= ((int64_t)1 << 31) || s->n_sv >= ((int64_t)1 << 31) ||
        s->n_ed >= ((int64_t)1 << 31))
        return MR_OK;
    const int nbt = std::max(1, bits_for((uint64_t)std::max(NT - 1, 0)));
    const int nbn = bits_for((uint64_t)s->n_podops);
    DBuf<uint64_t> hkey, key;
    DBuf<uint32_t> tr_h;
    DBuf<int32_t> lo_n, nsv, ned, head, rep, bad;
    DBuf<int64_t> hpos, tmp;
    MR_TRY(hkey.alloc(ctx, (size_t)NT));
    MR_TRY(rep.alloc(ctx, (size_t)NT));
    MR_TRY(key.alloc(ctx, (size_t)NT));
    MR_TRY(tr_h.alloc(ctx, (size_t)NT));
    MR_TRY(lo_n.alloc(ctx, (size_t)NT));
    MR_TRY(nsv.alloc(ctx, (size_t)NT));
    MR_TRY(ned.alloc(ctx, (size_t)NT));
    MR_TRY(head.alloc(ctx, (size_t)NT));
    MR_TRY(hpos.alloc(ctx, (size_t)NT + 1));
    MR_TRY(tmp.alloc(ctx, (size_t)scan_tmp_elems(NT)));
    MR_TRY(bad.alloc(ctx, 1));
    MR_TRY(s->lo_tr.alloc(ctx, (size_t)NT));
    MR_TRY(s->lo_len.alloc(ctx, (size_t)NT));
    MR_TRY(s->lo_kid.alloc(ctx, (size_t)NT));
    MR_TRY(s->lo_off.alloc(ctx, (size_t)NT + 1));
    MR_TRY(s->lo16.alloc(ctx, (size_t)std::max<int64_t>(s->n_po, 1)));
    MR_TRY(s->lo_cnt.alloc(ctx, (size_t)std::max<int64_t>(s->n_po, 1)));
    MR_TRY(s->lo_first.alloc(ctx, (size_t)std::max<int64_t>(s->n_po, 1)));
    MR_TRY(s->lo_ts.alloc(ctx, (size_t)NT));
    MR_TRY(s->lo_te.alloc(ctx, (size_t)NT));
    MR_TRY(s->lo_mx.alloc(ctx, (size_t)NT));
    MR_TRY(s->lsv_off.alloc(ctx, (size_t)NT + 1));
    MR_TRY(s->le_off.alloc(ctx, (size_t)NT + 1));
    MR_TRY(s->lsv.alloc(ctx, (size_t)std::max<int64_t>(s->n_sv, 1)));
    MR_TRY(s->le.alloc(ctx, (size_t)std::max<int64_t>(s->n_ed, 1)));
    const bool collide = getenv("MR_KIND_TEST_COLLIDE") != nullptr;   // (tests: every hash equal -> rerun)
    for (int attempt = 0; attempt < 4; ++attempt) {
        const uint64_t seed = 0x51ed270b27a3c0deull + 0x9E3779B97F4A7C15ull * (uint64_t)attempt;
        MR_TRY(bad.zero(ctx, 1));
        hipLaunchKernelGGL(k_lo_hash, dim3(cdiv(NT, XB)), dim3(XB), 0, st, s->po_off.p, s->po_op.p, s->tlen.p, NT, seed,
                           hkey.p, tr_h.p);
        if (collide && attempt == 0) MR_TRY_HIP(ctx, hipMemsetAsync(hkey.p, 0, (size_t)NT * 8, st));
        SortScratch ws;
        MR_TRY(mr_radix_sort(ctx, hkey.p, tr_h.p, NT, 64, ws));   // (stable: codes ascending within a hash)
        hipLaunchKernelGGL(k_lo_keys, dim3(cdiv(NT, XB)), dim3(XB), 0, st, tr_h.p, s->po_off.p, NT, nbt, key.p);
        MR_TRY(mr_radix_sort(ctx, key.p, nullptr, NT, nbt + nbn, ws));
        hipLaunchKernelGGL(k_lo_unpack, dim3(cdiv(NT, XB)), dim3(XB), 0, st, key.p, tr_h.p, hkey.p, NT, nbt, s->tlen.p,
                           s->lo_tr.p, lo_n.p, s->lo_len.p, head.p);
        MR_TRY(mr_exclusive_scan_i32(ctx, lo_n.p, s->lo_off.p, NT, tmp.p));
        hipLaunchKernelGGL(k_lo_copy, dim3(cdiv(NT, XB)), dim3(XB), 0, st, s->lo_tr.p, s->lo_off.p, NT, s->po_off.p,
                           s->po_op.p, s->po_cnt.p, s->po_first.p, s->tts.p, s->tte.p, s->tmaxd.p, s->sv_off.p,
                           s->ed_off.p, s->lo16.p, s->lo_cnt.p, s->lo_first.p, s->lo_ts.p, s->lo_te.p, s->lo_mx.p, nsv.p,
                           ned.p, bad.p);
        int32_t hb = 0;
        MR_TRY(bad.download(ctx, &hb, 1));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
        if (hb) return MR_OK;   // (counts past 16 bits: the general window path)
        MR_TRY(mr_exclusive_scan_i32(ctx, head.p, hpos.p, NT, tmp.p));
        hipLaunchKernelGGL(k_lo_reps, dim3(cdiv(NT, XB)), dim3(XB), 0, st, head.p, hpos.p, NT, rep.p);
        hipLaunchKernelGGL(k_lo_classes, dim3(cdiv(NT, XB)), dim3(XB), 0, st, head.p, hpos.p, rep.p, NT, s->lo_off.p,
                           s->lo16.p, s->lo_len.p, s->lo_kid.p, bad.p);
        MR_TRY_HIP(ctx, hipGetLastError());
        int64_t nk = 0;
        MR_TRY_HIP(ctx, hipMemcpyAsync(&nk, hpos.p + NT, sizeof nk, hipMemcpyDeviceToHost, st));
        MR_TRY(bad.download(ctx, &hb, 1));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // (the sorts' scratch leaves scope)
        if (hb) continue;   // (a collision: the next seed)
        MR_TRY(mr_exclusive_scan_i32(ctx, nsv.p, s->lsv_off.p, NT, tmp.p));
        MR_TRY(mr_exclusive_scan_i32(ctx, ned.p, s->le_off.p, NT, tmp.p));
        hipLaunchKernelGGL(k_lo_copy2, dim3(cdiv(NT, XB)), dim3(XB), 0, st, s->lo_tr.p, NT, s->sv_off.p, s->sv_op.p,
                           s->sv_cnt.p, s->ed_off.p, s->ed_eid.p, s->ed_cnt.p, s->lsv_off.p, s->le_off.p, s->lsv.p,
                           s->le.p, bad.p);
        MR_TRY_HIP(ctx, hipGetLastError());
        MR_TRY(bad.download(ctx, &hb, 1));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
        if (hb) return MR_OK;   // (codes or counts past 16 bits)
        {   // the window-build blocks: greedy cut of the layout by trace count and entries
            std::vector<int64_t> off((size_t)NT + 1);
            MR_TRY(s->lo_off.download(ctx, off.data(), (size_t)NT + 1));
            MR_TRY_HIP(ctx, hipStreamSynchronize(st));
            std::vector<int32_t> bs;
            bs.push_back(0);
            for (int32_t i = 0; i < NT; ++i) {
                const int32_t b0 = bs.back();
                if (i > b0 && (i - b0 >= LO_BT_MAX || off[(size_t)i + 1] - off[(size_t)b0] > LO_BE)) bs.push_back(i);
            }
            bs.push_back(NT);
            MR_TRY(s->lo_bstart.upload(ctx, bs.data(), bs.size()));
            MR_TRY_HIP(ctx, hipStreamSynchronize(st));
            s->lo_nblk = (int32_t)bs.size() - 1;
        }
        s->lo_nk = (int32_t)nk;
        s->lo_ok = true;
        return MR_OK;
    }
    return MR_OK;   // (four colliding seeds: the general window path)
}
static void lo_release(mr_spans* s) {
    s->lo_ok = false;
    s->lo_nk = 0;
    s->lo_nblk = 0;
    s->lo_tr.reset();
    s->lo_len.reset();
    s->lo_kid.reset();
    s->lo_off.reset();
    s->lo16.reset();
    s->lo_cnt.reset();
    s->lo_first.reset();
    s->lo_ts.reset();
    s->lo_te.reset();
    s->lo_mx.reset();
    s->lo_bstart.reset();
    s->lsv_off.reset();
    s->le_off.reset();
    s->lsv.reset();
    s->le.reset();
}
// Best effort: the layout order is a fast path of the window build.  A table it does not cover
// (codes or counts past 16 bits, four colliding seeds) or an error on the way (an allocation, a
// launch) leaves the table on the general window path with no lo_* buffers held; the index
// itself stays valid and the call succeeds.
static int lo_index(mr_ctx* ctx, mr_spans* s) {
    const int rc = lo_index_try(ctx, s);
    if (rc != MR_OK) {
        (void)hipStreamSynchronize(ctx->stream);
        (void)hipGetLastError();
        ctx->err.clear();
    }
    if (rc != MR_OK || !s->lo_ok) lo_release(s);
    return MR_OK;
}

int mr_spans_index(mr_ctx* ctx, mr_spans* s) {
    hipStream_t st = ctx->stream;
    const int64_t S = s->S;
    const int32_t NT = s->n_traces, NP = s->n_podops;
    s->indexed = false;
    const int nbt = bits_for((uint64_t)std::max(NT - 1, 0));
    const int nbp = std::max(1, bits_for((uint64_t)std::max(NP - 1, 0)));
    const int nbs = std::max(1, bits_for((uint64_t)std::max(s->n_svcops - 1, 0)));
    if (S == 0 || NT == 0 || nbt + 2 * nbp > 64 || nbt + nbs > 64 || nbp > 32) return MR_OK;   // row-level paths only
    // per-trace scalars
    MR_TRY(s->tlen.zero(ctx, NT));
    MR_TRY(s->tmaxd.alloc(ctx, NT));
    MR_TRY(s->tts.alloc(ctx, NT));
    MR_TRY(s->tte.alloc(ctx, NT));
    DBuf<long long> tsmax, temax;
    MR_TRY(tsmax.alloc(ctx, NT));
    MR_TRY(temax.alloc(ctx, NT));
    DBuf<int32_t> bad;
    MR_TRY(bad.zero(ctx, 1));
    MR_TRY_HIP(ctx, hipMemsetAsync(s->tmaxd.p, 0x80, NT * sizeof(long long), st));   // very negative
    MR_TRY_HIP(ctx, hipMemsetAsync(tsmax.p, 0x80, NT * sizeof(long long), st));
    MR_TRY_HIP(ctx, hipMemsetAsync(temax.p, 0x80, NT * sizeof(long long), st));
    MR_TRY_HIP(ctx, hipMemsetAsync(s->tts.p, 0x7f, NT * sizeof(long long), st));     // very positive
    MR_TRY_HIP(ctx, hipMemsetAsync(s->tte.p, 0x7f, NT * sizeof(long long), st));
    hipLaunchKernelGGL(k_ix_trace_stats, dim3(cdiv(S, XB)), dim3(XB), 0, st, s->trace.p, s->duration.p,
                       s->has_times ? s->tstart.p : nullptr, s->has_times ? s->tend.p : nullptr, S, s->tlen.p,
                       s->tmaxd.p, s->tts.p, tsmax.p, s->tte.p, temax.p);
    if (s->has_times)
        hipLaunchKernelGGL(k_ix_uniform, dim3(cdiv(NT, XB)), dim3(XB), 0, st, s->tlen.p, s->tts.p, tsmax.p, s->tte.p,
                           temax.p, NT, bad.p);
    // distinct pod-ops and service-ops per trace
    MR_TRY(trace_runs(ctx, s, s->podop.p, NP, s->po_off, s->po_op, s->po_cnt, &s->po_first, &s->po_tr, &s->n_po));
    if (s->grow.p && s->n_po)   // a shard: first appearances in the whole table's row order
        hipLaunchKernelGGL(k_ix_map_rows, dim3(cdiv(s->n_po, XB)), dim3(XB), 0, st, s->po_first.p, s->n_po, s->grow.p);
    MR_TRY(trace_runs(ctx, s, s->svcop.p, s->n_svcops, s->sv_off, s->sv_op, s->sv_cnt, nullptr, nullptr, &s->n_sv));
    // parent join resolved once
    {
        DBuf<int32_t> nin, nx;
        DBuf<int64_t> pin, px, tmp;
        MR_TRY(nin.alloc(ctx, S));
        MR_TRY(nx.alloc(ctx, S));
        MR_TRY(pin.alloc(ctx, S + 1));
        MR_TRY(px.alloc(ctx, S + 1));
        MR_TRY(tmp.alloc(ctx, std::max(scan_tmp_elems(S), scan_tmp_elems(NT))));
        hipLaunchKernelGGL(k_ix_join_count, dim3(cdiv(S, XB)), dim3(XB), 0, st, s->trace.p, s->parent.p, S, s->id_off.p,
                           s->id_rows.p, s->n_span_codes, nin.p, nx.p);
        MR_TRY(mr_exclusive_scan_i32(ctx, nin.p, pin.p, S, tmp.p));
        MR_TRY(mr_exclusive_scan_i32(ctx, nx.p, px.p, S, tmp.p));
        int64_t h[2] = {0, 0};
        MR_TRY_HIP(ctx, hipMemcpyAsync(&h[0], pin.p + S, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        MR_TRY_HIP(ctx, hipMemcpyAsync(&h[1], px.p + S, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
        const int64_t J = h[0];
        s->n_xj = h[1];
        DBuf<uint64_t> ikey;
        MR_TRY(ikey.alloc(ctx, J));
        MR_TRY(s->xj_tc.alloc(ctx, s->n_xj));
        MR_TRY(s->xj_tp.alloc(ctx, s->n_xj));
        MR_TRY(s->xj_key.alloc(ctx, s->n_xj));
        hipLaunchKernelGGL(k_ix_join_fill, dim3(cdiv(S, XB)), dim3(XB), 0, st, s->trace.p, s->podop.p, s->parent.p, S,
                           s->id_off.p, s->id_rows.p, s->n_span_codes, pin.p, px.p, nbp, ikey.p, s->xj_tc.p, s->xj_tp.p,
                           s->xj_key.p);
        SortScratch ws;
        MR_TRY(mr_radix_sort(ctx, ikey.p, nullptr, J, nbt + 2 * nbp, ws));
        DBuf<int32_t> head, truns;
        DBuf<int64_t> hpos, r_start;
        MR_TRY(head.alloc(ctx, J));
        MR_TRY(hpos.alloc(ctx, J + 1));
        MR_TRY(truns.zero(ctx, NT));
        MR_TRY(tmp.alloc(ctx, std::max({scan_tmp_elems(J), scan_tmp_elems(NT), (int64_t)1})));
        if (J) hipLaunchKernelGGL(k_ix_heads, dim3(cdiv(J, XB)), dim3(XB), 0, st, ikey.p, J, head.p);
        MR_TRY(mr_exclusive_scan_i32(ctx, head.p, hpos.p, J, tmp.p));
        int64_t R = 0;
        MR_TRY_HIP(ctx, hipMemcpyAsync(&R, hpos.p + J, sizeof R, hipMemcpyDeviceToHost, st));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
        s->n_ed = R;
        MR_TRY(s->ed_key.alloc(ctx, R));
        MR_TRY(s->ed_cnt.alloc(ctx, R));
        MR_TRY(s->ed_tr.alloc(ctx, R));
        MR_TRY(r_start.alloc(ctx, R));
        if (J)
            hipLaunchKernelGGL(k_ix_edge_runs, dim3(cdiv(J, XB)), dim3(XB), 0, st, ikey.p, head.p, hpos.p, J, nbp,
                               s->ed_key.p, s->ed_tr.p, r_start.p, truns.p);
        if (R) hipLaunchKernelGGL(k_ix_cnt, dim3(cdiv(R, XB)), dim3(XB), 0, st, r_start.p, R, J, s->ed_cnt.p);
        MR_TRY(s->ed_off.alloc(ctx, (size_t)NT + 1));
        MR_TRY(mr_exclusive_scan_i32(ctx, truns.p, s->ed_off.p, NT, tmp.p));
        MR_TRY_HIP(ctx, hipGetLastError());
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    }
    {   // distinct call-edge keys over the whole table: a bound for any subset's edge set
        const int64_t K = s->n_ed + s->n_xj;
        DBuf<uint64_t> k2;
        DBuf<int32_t> head;
        DBuf<int64_t> hpos, tmp;
        MR_TRY(k2.alloc(ctx, K));
        MR_TRY(head.alloc(ctx, K));
        MR_TRY(hpos.alloc(ctx, K + 1));
        MR_TRY(tmp.alloc(ctx, std::max<int64_t>(scan_tmp_elems(K), 1)));
        if (K) hipLaunchKernelGGL(k_ix_pack_keys, dim3(cdiv(K, XB)), dim3(XB), 0, st, s->ed_key.p, s->n_ed, s->xj_key.p,
                                  s->n_xj, nbp, k2.p);
        SortScratch ws;
        MR_TRY(mr_radix_sort(ctx, k2.p, nullptr, K, 2 * nbp, ws));
        if (K) hipLaunchKernelGGL(k_ix_heads, dim3(cdiv(K, XB)), dim3(XB), 0, st, k2.p, K, head.p);
        MR_TRY(mr_exclusive_scan_i32(ctx, head.p, hpos.p, K, tmp.p));
        MR_TRY_HIP(ctx, hipMemcpyAsync(&s->n_edge_keys, hpos.p + K, sizeof(int64_t), hipMemcpyDeviceToHost, st));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
        // dense edge ids: a window's build counts its edges per id (an LDS histogram) instead of
        // probing a hash set per entry
        const int64_t E = s->n_edge_keys;
        MR_TRY(s->ekey.alloc(ctx, (size_t)std::max<int64_t>(E, 1)));
        MR_TRY(s->ed_eid.alloc(ctx, (size_t)std::max<int64_t>(s->n_ed, 1)));
        MR_TRY(s->xj_eid.alloc(ctx, (size_t)std::max<int64_t>(s->n_xj, 1)));
        if (K) hipLaunchKernelGGL(k_ix_ekeys, dim3(cdiv(K, XB)), dim3(XB), 0, st, k2.p, head.p, hpos.p, K, nbp, s->ekey.p);
        if (s->n_ed)
            hipLaunchKernelGGL(k_ix_eid, dim3(cdiv(s->n_ed, XB)), dim3(XB), 0, st, s->ed_key.p, s->n_ed, s->ekey.p, E,
                               s->ed_eid.p);
        if (s->n_xj)
            hipLaunchKernelGGL(k_ix_eid, dim3(cdiv(s->n_xj, XB)), dim3(XB), 0, st, s->xj_key.p, s->n_xj, s->ekey.p, E,
                               s->xj_eid.p);
        MR_TRY_HIP(ctx, hipGetLastError());
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
        // large tables: the entries in edge-id order as well (a radix sort of the ids carrying the
        // entry index, then a gather), so a build's edge count is a segmented sum per id
        const char* ebe = getenv("MR_IX_EB");
        const bool eb = ebe ? strcmp(ebe, "0") != 0 && (!strcmp(ebe, "force") || s->n_ed >= ED_BYID_MIN)
                            : s->n_ed >= ED_BYID_MIN;
        s->eb_tr.reset();
        s->eb_cnt.reset();
        s->eb_eid.reset();
        if (eb && s->n_ed > 0 && E > 0 && s->n_ed < ((int64_t)1 << 32)) {
            const int64_t n = s->n_ed;
            DBuf<uint64_t> key;
            DBuf<uint32_t> val;
            MR_TRY(key.alloc(ctx, (size_t)n));
            MR_TRY(val.alloc(ctx, (size_t)n));
            hipLaunchKernelGGL(k_ix_eb_keys, dim3(cdiv(n, XB)), dim3(XB), 0, st, s->ed_eid.p, n, key.p, val.p);
            SortScratch ws;
            int bits = 1;
            while (bits < 63 && ((int64_t)1 << bits) < E) ++bits;
            MR_TRY(mr_radix_sort(ctx, key.p, val.p, n, bits, ws));
            MR_TRY(s->eb_tr.alloc(ctx, (size_t)n));
            MR_TRY(s->eb_cnt.alloc(ctx, (size_t)n));
            MR_TRY(s->eb_eid.alloc(ctx, (size_t)n));
            hipLaunchKernelGGL(k_ix_eb_gather, dim3(cdiv(n, XB)), dim3(XB), 0, st, key.p, val.p, n, s->ed_tr.p, s->ed_cnt.p,
                               s->eb_tr.p, s->eb_cnt.p, s->eb_eid.p);
            MR_TRY_HIP(ctx, hipGetLastError());
            MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // (the sort's scratch leaves scope)
        }
    }
    int32_t hb = 0;
    MR_TRY(bad.download(ctx, &hb, 1));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    s->uniform_times = s->has_times && hb == 0;
    s->indexed = true;
    if (!getenv("MR_NO_LO")) MR_TRY(lo_index(ctx, s));   // (A/B and tests, read per table: the general window build)
    return MR_OK;
}

// Window detector on the index (uniform trace times): state[t] 0 out / 1 normal / 2 abnormal for
// EVERY trace; counts (3 * MR_DETECT_SHARDS words, zeroed by the caller) receive the abnormal /
// normal / in-window-row counter shards (mr_detect_sum adds them up on the host).
int mr_detect_indexed_launch(mr_ctx* ctx, const mr_spans* s, int64_t t0, int64_t t1, const double* d_a3,
                             const uint8_t* d_a3v, uint8_t* d_state, unsigned long long* counts) {
    const int32_t NT = s->n_traces;
    if (NT)
        hipLaunchKernelGGL(k_ix_detect, dim3(cdiv(NT, DB)), dim3(DB), 0, ctx->stream, NT,
                           mr_detect_in(s, t0, t1, d_a3, d_a3v, d_state, counts));
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}
void mr_detect_sum(const unsigned long long* sh, int32_t* n_abn, int32_t* n_nor, int64_t* n_in) {
    unsigned long long hc[3] = {0, 0, 0};
    for (int k = 0; k < 3 * CSH; ++k) hc[k % 3] += sh[k];
    *n_abn = (int32_t)hc[0];
    *n_nor = (int32_t)hc[1];
    *n_in = (int64_t)hc[2];
}
int mr_detect_indexed(mr_ctx* ctx, const mr_spans* s, int64_t t0, int64_t t1, const double* d_a3, const uint8_t* d_a3v,
                      uint8_t* d_state, int32_t* n_abn, int32_t* n_nor, int64_t* n_in) {
    DBuf<unsigned long long> counts;
    MR_TRY(counts.zero(ctx, 3 * CSH));
    MR_TRY(mr_detect_indexed_launch(ctx, s, t0, t1, d_a3, d_a3v, d_state, counts.p));
    unsigned char* h = nullptr;
    MR_TRY(mr_read_bytes(ctx, counts.p, 3 * CSH * sizeof(unsigned long long), &h));
    mr_detect_sum((const unsigned long long*)h, n_abn, n_nor, n_in);
    if (*n_in == 0) return mr_fail(ctx, MR_ERR_VALUE, "Current span list is empty");
    return MR_OK;
}

// f3: the detector counts of every window start t_begin + m * grain (m < M) in one pass over the
// traces (k_ix_sweep); state[t] receives each trace's window-independent partition.  diff:
// 3 * (M + 1) words zeroed by the caller (abnormal, normal, rows difference arrays).
int mr_detect_sweep_launch(mr_ctx* ctx, const mr_spans* s, int64_t t_begin, int64_t grain, int64_t window, int32_t M,
                           const double* d_a3, const uint8_t* d_a3v, uint8_t* d_state, unsigned long long* diff) {
    const int32_t NT = s->n_traces;
    if (!s->indexed || !s->uniform_times) return mr_fail(ctx, MR_ERR_STATE, "sweep needs trace-level window times");
    if (NT)
        hipLaunchKernelGGL(k_ix_sweep, dim3(cdiv(NT, SWB * SWT)), dim3(SWB), 0, ctx->stream, NT, s->tlen.p, s->tts.p,
                           s->tte.p, s->tmaxd.p, s->sv_off.p, s->sv_op.p, s->sv_cnt.p, d_a3, d_a3v, t_begin, grain,
                           window, M, d_state, diff);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}
