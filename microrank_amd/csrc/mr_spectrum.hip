// K3: online_rca.calculate_spectrum_without_delay_list (online_rca.py:33-152) on gfx950.
//
// One thread per node computes (ef, nf, ep, np) from the two PageRank weight/coverage vectors
// (:45-69) and applies one of the 13 formulas (:77-142) with the reference's operation
// order (no FMA contraction).  The stable descending sort (:147) is a sort on the composite
// key (score, position): positions break ties exactly like Python's stable `sorted`.  Nodes
// are in the reference's iteration order: anomaly_result nodes, then normal-only nodes.
//
// Python raises ZeroDivisionError only when BOTH operands of a division are Python scalars
// (an np.float64 operand gives inf/nan instead).  Each node carries the "numpy-typed" bits of
// its inputs, the kernel propagates them through the formula and flags a division by zero
// between two Python-typed values.
#include <algorithm>
#include <cstring>

#include "mr_prim.h"
#include "mr_sort.h"

namespace {
enum Method { DSTAR2, OCHIAI, JACCARD, SORENSEN, M1, M2, GOODMAN, TARANTULA, RUSSELLRAO, HAMANN, DICE, SIMPLE, ROGERS };

struct TV {   // typed value: v and whether it is numpy-typed (np.float64) in the reference
    double v;
    bool np;
};
__device__ __forceinline__ TV add(TV a, TV b) { return {a.v + b.v, a.np || b.np}; }
__device__ __forceinline__ TV sub(TV a, TV b) { return {a.v - b.v, a.np || b.np}; }
__device__ __forceinline__ TV mul(TV a, TV b) { return {a.v * b.v, a.np || b.np}; }
__device__ __forceinline__ TV dv(TV a, TV b, bool& zd) {
    if (!a.np && !b.np && b.v == 0.0) zd = true;
    return {a.v / b.v, a.np || b.np};
}

__device__ double spectrum_score(int method, TV ef, TV nf, TV ep, TV np_, bool& zd, bool& res_np) {
    const TV two{2.0, false};
    TV r{0.0, false};
    switch (method) {
        case DSTAR2: r = dv(mul(ef, ef), add(ep, nf), zd); break;                                     // :78
        case OCHIAI: r = dv(ef, TV{sqrt(add(ep, ef).v * add(ef, nf).v), false}, zd); break;           // :81
        case JACCARD: r = dv(ef, add(add(ef, ep), nf), zd); break;                                     // :86
        case SORENSEN: r = dv(mul(two, ef), add(add(mul(two, ef), ep), nf), zd); break;                // :89
        case M1: r = dv(add(ef, np_), add(ep, nf), zd); break;                                         // :94
        case M2: r = dv(ef, add(add(add(mul(two, ep), mul(two, nf)), ef), np_), zd); break;            // :97
        case GOODMAN: r = dv(sub(sub(mul(two, ef), nf), ep), add(add(mul(two, ef), nf), ep), zd); break;  // :101
        case TARANTULA: {                                                                              // :106
            TV a = dv(ef, add(ef, nf), zd);
            TV b = dv(ef, add(ef, nf), zd);
            TV c = dv(ep, add(ep, np_), zd);
            r = dv(a, add(b, c), zd);
        } break;
        case RUSSELLRAO: r = dv(ef, add(add(add(ef, nf), ep), np_), zd); break;                        // :116
        case HAMANN: r = dv(sub(sub(add(ef, np_), ep), nf), add(add(add(ef, nf), ep), np_), zd); break;  // :122
        case DICE: r = dv(mul(two, ef), add(add(ef, nf), ep), zd); break;                              // :128
        case SIMPLE: r = dv(add(ef, np_), add(add(add(ef, np_), nf), ep), zd); break;                  // :134
        case ROGERS: r = dv(add(ef, np_), add(add(add(ef, np_), mul(two, nf)), mul(two, ep)), zd); break;  // :140
    }
    res_np = r.np;
    return r.v;
}

// order-preserving bits for a DESCENDING sort (ascending key = descending score); -0 == +0
__device__ __forceinline__ uint64_t desc_key(double v) {
    if (v == 0.0) v = 0.0;
    uint64_t b = (uint64_t)__double_as_longlong(v);
    b = (b >> 63) ? ~b : (b | 0x8000000000000000ull);   // ascending-orderable
    return ~b;
}

// flags per node: bit0 in anomaly_result, bit1 in normal_result, bit2 a_w numpy-typed,
// bit3 n_w numpy-typed
__global__ void k_spectrum(int32_t n, const uint8_t* flags, const double* a_w, const int64_t* a_num, const double* n_w,
                           const int64_t* n_num, int64_t A, int64_t Nl, int method, double* score, uint8_t* res_np,
                           uint64_t* key, uint32_t* idx, int32_t* zflag) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t f = flags[i];
    const bool ha = f & 1, hn = f & 2, ta = f & 4, tn = f & 8;
    const TV eps{0.0000001, false};
    TV ef, nf, ep, np_;
    if (ha) {   // :45-58
        ef = TV{a_w[i] * (double)a_num[i], ta};
        nf = TV{a_w[i] * (double)(A - a_num[i]), ta};
        if (hn) {
            ep = TV{n_w[i] * (double)n_num[i], tn};
            np_ = TV{n_w[i] * (double)(Nl - n_num[i]), tn};
        } else {
            ep = eps;
            np_ = eps;
        }
    } else {    // :60-69 normal-only
        ep = TV{(1.0 + n_w[i]) * (double)n_num[i], tn};
        np_ = TV{(double)(Nl - n_num[i]), false};
        ef = eps;
        nf = eps;
    }
    bool zd = false, rnp = false;
    const double s = spectrum_score(method, ef, nf, ep, np_, zd, rnp);
    score[i] = s;
    res_np[i] = rnp;
    key[i] = desc_key(s);
    idx[i] = (uint32_t)i;
    if (zd) atomicOr(zflag, 1);
}

// small n: one block sorts (key, idx) pairs in LDS with a bitonic network; (key, idx) pairs are
// unique, so the unstable network still yields the stable order
constexpr int SB = 4096;
__global__ void __launch_bounds__(1024) k_sort_small(uint64_t* key, uint32_t* idx, int32_t n) {
    __shared__ uint64_t k[SB];
    __shared__ uint32_t v[SB];
    int32_t m = 1;
    while (m < n) m <<= 1;
    for (int32_t i = threadIdx.x; i < m; i += blockDim.x) {
        k[i] = i < n ? key[i] : ~0ull;
        v[i] = i < n ? idx[i] : 0xffffffffu;
    }
    __syncthreads();
    for (int32_t size = 2; size <= m; size <<= 1) {
        for (int32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (int32_t i = threadIdx.x; i < m; i += blockDim.x) {
                const int32_t j = i ^ stride;
                if (j > i) {
                    const bool up = (i & size) == 0;
                    const bool gt = k[i] > k[j] || (k[i] == k[j] && v[i] > v[j]);
                    if (gt == up) {
                        uint64_t tk = k[i];
                        k[i] = k[j];
                        k[j] = tk;
                        uint32_t tv = v[i];
                        v[i] = v[j];
                        v[j] = tv;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (int32_t i = threadIdx.x; i < n; i += blockDim.x) {
        key[i] = k[i];
        idx[i] = v[i];
    }
}

__global__ void k_gather_top(const uint32_t* idx, const double* score, const uint8_t* res_np, int32_t top,
                             int32_t* out_idx, double* out_score, uint8_t* out_np) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= top) return;
    const uint32_t j = idx[i];
    out_idx[i] = (int32_t)j;
    out_score[i] = score[j];
    if (out_np) out_np[i] = res_np[j];
}
// A window's whole spectrum step in ONE block (union sizes up to WS_MAX, pod-op codes up to
// WS_PMAX): the union of the two graphs' nodes in the reference's order (anomaly_result nodes,
// then normal-only nodes in normal_result order, online_rca.py:45-69), the scores (k_spectrum's
// formula and typing), the stable descending sort and the top k -- instead of ~10 launches and
// three host round trips.  out: [k] codes (int32, at 0), [k] scores (double, at 8 * WS_KMAX / 2)
constexpr int WS_T = 1024, WS_MAX = 4096, WS_PMAX = 4096, WS_KMAX = 256;
// the bitonic network's stages of stride < 64 inside a wave: lane i's element meets lane i ^ stride
// by a lane exchange (no LDS round trip, no barrier).  size: the merge's block size (direction),
// strides s_hi, s_hi / 2, .., 1.  (key, index) pairs are unique except the padding's, which are
// equal to each other (either order of two equal pairs is the same sequence)
__device__ __forceinline__ void ws_bitonic_lanes(uint64_t& k, uint32_t& v, int32_t i, int32_t size, int32_t s_hi) {
    for (int32_t stride = s_hi; stride > 0; stride >>= 1) {
        const uint64_t pk = (uint64_t)__shfl_xor((long long)k, stride, WAVE);
        const uint32_t pv = (uint32_t)__shfl_xor((int)v, stride, WAVE);
        const bool lower = (i & stride) == 0, up = (i & size) == 0;
        const bool gt = k > pk || (k == pk && v > pv);
        if (lower == up ? gt : !gt) {   // lower half of an ascending pair keeps the min, ...
            k = pk;
            v = pv;
        }
    }
}
__device__ __forceinline__ void win_spectrum_block(int32_t Na, const int32_t* a_podop, const double* a_w,
                                                   const int32_t* a_cov, int32_t Nn, const int32_t* n_podop,
                                                   const double* n_w, const int32_t* n_cov, int32_t NP, int64_t A,
                                                   int64_t Nl, int method, int32_t k, unsigned char* out) {
    __shared__ int32_t nidx[WS_PMAX], apos[WS_PMAX];
    __shared__ uint64_t key[WS_MAX];
    __shared__ uint32_t vix[WS_MAX];
    __shared__ int32_t ucode[WS_MAX];
    __shared__ double score[WS_MAX];
    __shared__ int32_t sbuf[WS_T];
    __shared__ int32_t nonly;
    const int tid = threadIdx.x;
    for (int c = tid; c < NP; c += WS_T) {
        nidx[c] = -1;
        apos[c] = -1;
    }
    __syncthreads();
    for (int j = tid; j < Nn; j += WS_T) nidx[n_podop[j]] = j;
    for (int i = tid; i < Na; i += WS_T) apos[a_podop[i]] = i;
    __syncthreads();
    // normal-only nodes in normal order: each thread a run of j, a block scan of the run counts
    // (inclusive scan per wave by lane exchanges, the waves' totals through LDS: two barriers)
    const int per = (Nn + WS_T - 1) / WS_T, j0 = tid * per, j1 = min(j0 + per, Nn);
    const int lane = tid & (WAVE - 1), wv = tid / WAVE;
    int32_t cnt = 0;
    for (int j = j0; j < j1; ++j) cnt += apos[n_podop[j]] < 0 ? 1 : 0;
    int32_t inc = cnt;
#pragma unroll
    for (int o = 1; o < WAVE; o <<= 1) {
        const int32_t u = __shfl_up(inc, o, WAVE);
        if (lane >= o) inc += u;
    }
    if (lane == WAVE - 1) sbuf[wv] = inc;
    __syncthreads();
    int32_t before = 0, total = 0;
    for (int q = 0; q < WS_T / WAVE; ++q) {
        before += q < wv ? sbuf[q] : 0;
        total += sbuf[q];
    }
    if (tid == 0) nonly = total;
    int32_t pos = Na + before + inc - cnt;
    const TV eps{0.0000001, false};
    for (int j = j0; j < j1; ++j) {   // normal-only entries (:60-69)
        const int32_t c = n_podop[j];
        if (apos[c] >= 0) continue;
        const TV ep{(1.0 + n_w[j]) * (double)n_cov[j], true}, np_{(double)(Nl - n_cov[j]), false};
        bool zd = false, rnp = false;
        const double sc = spectrum_score(method, eps, eps, ep, np_, zd, rnp);
        score[pos] = sc;
        key[pos] = desc_key(sc);
        vix[pos] = (uint32_t)pos;
        ucode[pos] = c;
        ++pos;
    }
    for (int i = tid; i < Na; i += WS_T) {   // anomaly_result entries (:45-58)
        const int32_t c = a_podop[i], j = nidx[c];
        const TV ef{a_w[i] * (double)a_cov[i], true}, nf{a_w[i] * (double)(A - a_cov[i]), true};
        TV ep = eps, np_ = eps;
        if (j >= 0) {
            ep = TV{n_w[j] * (double)n_cov[j], true};
            np_ = TV{n_w[j] * (double)(Nl - n_cov[j]), true};
        }
        bool zd = false, rnp = false;
        const double sc = spectrum_score(method, ef, nf, ep, np_, zd, rnp);
        score[i] = sc;
        key[i] = desc_key(sc);
        vix[i] = (uint32_t)i;
        ucode[i] = c;
    }
    __syncthreads();
    const int32_t n = Na + nonly;
    int32_t m = 1;
    while (m < n) m <<= 1;
    for (int32_t i = n + tid; i < m; i += WS_T) {
        key[i] = ~0ull;
        vix[i] = 0xffffffffu;
    }
    __syncthreads();
    // bitonic network: strides >= 64 through LDS (a barrier each), the rest of every merge inside
    // the waves (ws_bitonic_lanes) -- 10 barriers for m = 512 instead of 45
    auto lanes = [&](int32_t size_lo, int32_t size_hi) {   // merges size_lo..size_hi, strides < 64
        for (int32_t i0 = tid - lane; i0 < m; i0 += WS_T) {   // (whole waves: every lane exchanges)
            const int32_t i = i0 + lane;
            uint64_t kr = i < m ? key[i] : ~0ull;
            uint32_t vr = i < m ? vix[i] : 0xffffffffu;
            for (int32_t size = size_lo; size <= size_hi; size <<= 1)
                ws_bitonic_lanes(kr, vr, i, size, min(size >> 1, WAVE / 2));
            if (i < m) {
                key[i] = kr;
                vix[i] = vr;
            }
        }
        __syncthreads();
    };
    lanes(2, min(m, WAVE));
    for (int32_t size = 2 * WAVE; size <= m; size <<= 1) {
        for (int32_t stride = size >> 1; stride >= WAVE; stride >>= 1) {
            for (int32_t i = tid; i < m; i += WS_T) {
                const int32_t jj = i ^ stride;
                if (jj > i) {
                    const bool up = (i & size) == 0;
                    const bool gt = key[i] > key[jj] || (key[i] == key[jj] && vix[i] > vix[jj]);
                    if (gt == up) {
                        const uint64_t tk = key[i];
                        key[i] = key[jj];
                        key[jj] = tk;
                        const uint32_t tv = vix[i];
                        vix[i] = vix[jj];
                        vix[jj] = tv;
                    }
                }
            }
            __syncthreads();
        }
        lanes(size, size);
    }
    const int32_t kk = min(k, n);
    int32_t* oc = (int32_t*)out;
    double* os = (double*)(out + 4 * WS_KMAX);
    for (int32_t i = tid; i < kk; i += WS_T) {
        oc[i] = ucode[vix[i]];
        os[i] = score[vix[i]];
    }
    if (tid == 0) ((int32_t*)(out + 12 * WS_KMAX))[0] = kk;
}
__global__ void __launch_bounds__(WS_T) k_win_spectrum(int32_t Na, const int32_t* a_podop, const double* a_w,
                                                      const int32_t* a_cov, int32_t Nn, const int32_t* n_podop,
                                                      const double* n_w, const int32_t* n_cov, int32_t NP, int64_t A,
                                                      int64_t Nl, int method, int32_t k, unsigned char* out) {
    win_spectrum_block(Na, a_podop, a_w, a_cov, Nn, n_podop, n_w, n_cov, NP, A, Nl, method, k, out);
}
// a block per window (the window batch's spectra of a group, MR_WS_BATCH per launch)
struct WsBatchArg {
    MrWsWin w[MR_WS_BATCH];
    int method;
    int32_t k;
};
__global__ void __launch_bounds__(WS_T) k_win_spectrum_b(WsBatchArg b) {
    const MrWsWin& x = b.w[blockIdx.x];
    win_spectrum_block(x.Na, x.a_podop, x.a_w, x.a_cov, x.Nn, x.n_podop, x.n_w, x.n_cov, x.NP, x.A, x.Nl, b.method, b.k,
                       x.out);
}
}  // namespace

// The window spectrum in one launch and one read-back (k_win_spectrum), or MR_ERR_STATE when the
// sizes exceed its one-block limits (the caller then takes the general path).
static_assert(MR_WS_SLOT == 12 * WS_KMAX + 16, "window spectrum slot");
int mr_win_spectrum_launch(mr_ctx* ctx, int32_t Na, const int32_t* a_podop, const double* a_w, const int32_t* a_cov,
                           int32_t Nn, const int32_t* n_podop, const double* n_w, const int32_t* n_cov, int32_t NP,
                           int64_t A, int64_t Nl, int method, int32_t k, unsigned char* d_slot) {
    if (!mr_win_spectrum_fits(Na, Nn, NP, k)) return MR_ERR_STATE;
    hipLaunchKernelGGL(k_win_spectrum, dim3(1), dim3(WS_T), 0, ctx->stream, Na, a_podop, a_w, a_cov, Nn, n_podop, n_w,
                       n_cov, NP, A, Nl, method, k, d_slot);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}
bool mr_win_spectrum_fits(int32_t Na, int32_t Nn, int32_t NP, int32_t k) {
    return Na + Nn <= WS_MAX && NP <= WS_PMAX && k <= WS_KMAX && k >= 0;
}
int mr_win_spectrum_launch_n(mr_ctx* ctx, const MrWsWin* ws, int n, int method, int32_t k) {
    if (n < 1 || n > MR_WS_BATCH) return mr_fail(ctx, MR_ERR_ARG, "mr_win_spectrum_launch_n: %d windows", n);
    WsBatchArg b{};
    for (int i = 0; i < n; ++i) {
        if (!mr_win_spectrum_fits(ws[i].Na, ws[i].Nn, ws[i].NP, k)) return MR_ERR_STATE;
        b.w[i] = ws[i];
    }
    b.method = method;
    b.k = k;
    hipLaunchKernelGGL(k_win_spectrum_b, dim3((unsigned)n), dim3(WS_T), 0, ctx->stream, b);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}
void mr_win_spectrum_unpack(const unsigned char* slot, int32_t* out_codes, double* out_score, int32_t* n_out) {
    const int32_t kk = ((const int32_t*)(slot + 12 * WS_KMAX))[0];
    if (out_codes) memcpy(out_codes, slot, (size_t)kk * sizeof(int32_t));
    if (out_score) memcpy(out_score, slot + 4 * WS_KMAX, (size_t)kk * sizeof(double));
    *n_out = kk;
}
int mr_win_spectrum_small(mr_ctx* ctx, int32_t Na, const int32_t* a_podop, const double* a_w, const int32_t* a_cov,
                          int32_t Nn, const int32_t* n_podop, const double* n_w, const int32_t* n_cov, int32_t NP,
                          int64_t A, int64_t Nl, int method, int32_t k, int32_t* out_codes, double* out_score,
                          int32_t* n_out) {
    DBuf<unsigned char> out;
    MR_TRY(out.alloc(ctx, MR_WS_SLOT));
    const int rc = mr_win_spectrum_launch(ctx, Na, a_podop, a_w, a_cov, Nn, n_podop, n_w, n_cov, NP, A, Nl, method, k,
                                          out.p);
    if (rc != MR_OK) return rc;
    unsigned char* h = nullptr;
    MR_TRY(mr_read_bytes(ctx, out.p, MR_WS_SLOT, &h));
    mr_win_spectrum_unpack(h, out_codes, out_score, n_out);
    return MR_OK;
}

// Device-side spectrum over n nodes whose inputs are already in HBM.  Writes the first `top`
// sorted positions / scores to device buffers.
int mr_spectrum_dev(mr_ctx* ctx, int32_t n, const uint8_t* flags, const double* a_w, const int64_t* a_num,
                    const double* n_w, const int64_t* n_num, int64_t A, int64_t Nl, int method, int32_t top,
                    int32_t* d_out_idx, double* d_out_score, uint8_t* d_out_np, int32_t* d_zflag) {
    hipStream_t st = ctx->stream;
    DBuf<double> score;
    DBuf<uint8_t> rnp;
    DBuf<uint64_t> key;
    DBuf<uint32_t> idx;
    MR_TRY(score.alloc(ctx, n));
    MR_TRY(rnp.alloc(ctx, n));
    MR_TRY(key.alloc(ctx, n));
    MR_TRY(idx.alloc(ctx, n));
    hipLaunchKernelGGL(k_spectrum, dim3(cdiv(n, 256)), dim3(256), 0, st, n, flags, a_w, a_num, n_w, n_num, A, Nl,
                       method, score.p, rnp.p, key.p, idx.p, d_zflag);
    if (n <= SB) {
        hipLaunchKernelGGL(k_sort_small, dim3(1), dim3(1024), 0, st, key.p, idx.p, n);
    } else {
        SortScratch ws;
        MR_TRY(mr_radix_sort(ctx, key.p, idx.p, n, 64, ws));   // LSD radix is stable: ties keep position order
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    }
    if (top > 0)
        hipLaunchKernelGGL(k_gather_top, dim3(cdiv(top, 256)), dim3(256), 0, st, idx.p, score.p, rnp.p, top, d_out_idx,
                           d_out_score, d_out_np);
    MR_TRY_HIP(ctx, hipGetLastError());
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // local buffers die here
    return MR_OK;
}

extern "C" int mr_spectrum(mr_ctx* ctx, int32_t n, const uint8_t* has_a, const double* a_w, const int64_t* a_num,
                           const uint8_t* has_n, const double* n_w, const int64_t* n_num, int64_t a_len, int64_t n_len,
                           int method, int32_t top, int32_t* out_idx, double* out_score, int32_t* n_out,
                           int32_t* zerodiv) {
    if (!ctx || n < 0 || !n_out || !zerodiv) return mr_fail(ctx, MR_ERR_ARG, "mr_spectrum: bad arguments");
    *n_out = 0;
    *zerodiv = 0;
    if (method < 0 || method > ROGERS) return MR_OK;   // unknown method: the reference returns empty lists
    if (n == 0) return MR_OK;
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    // has_a/has_n carry the membership bit in bit 0 and the numpy-typed bit in bit 1
    std::vector<uint8_t> fl((size_t)n);
    for (int32_t i = 0; i < n; ++i)
        fl[i] = (uint8_t)((has_a[i] & 1) | ((has_n[i] & 1) << 1) | ((has_a[i] & 2) << 1) | ((has_n[i] & 2) << 2));
    const int32_t k = std::min(n, std::max(top, 0));
    DBuf<uint8_t> dfl;
    DBuf<double> daw, dnw, dsc;
    DBuf<int64_t> dan, dnn;
    DBuf<int32_t> didx, dz;
    MR_TRY(dfl.upload(ctx, fl.data(), n));
    MR_TRY(daw.upload(ctx, a_w, n));
    MR_TRY(dan.upload(ctx, a_num, n));
    MR_TRY(dnw.upload(ctx, n_w, n));
    MR_TRY(dnn.upload(ctx, n_num, n));
    MR_TRY(didx.alloc(ctx, std::max(k, 1)));
    MR_TRY(dsc.alloc(ctx, std::max(k, 1)));
    MR_TRY(dz.zero(ctx, 1));
    MR_TRY(mr_spectrum_dev(ctx, n, dfl.p, daw.p, dan.p, dnw.p, dnn.p, a_len, n_len, method, k, didx.p, dsc.p, nullptr,
                           dz.p));
    if (k) {
        MR_TRY(didx.download(ctx, out_idx, k));
        MR_TRY(dsc.download(ctx, out_score, k));
    }
    MR_TRY(dz.download(ctx, zerodiv, 1));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *n_out = k;
    return MR_OK;
}
