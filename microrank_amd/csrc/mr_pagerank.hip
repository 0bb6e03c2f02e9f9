// K2: personalised PageRank of pagerank.trace_pagerank (pagerank.py:15-130) on gfx950.
//
// Sparse, HBM-bound: no MFMA.  Each Jacobi iteration k -> k+1 (T8) is two launches:
//   k_iter_a, two block roles reading only iteration-k state:
//     trace role  r'[t] = d * sum_{o in rs(t)} u_o * s_k[o] + fp32((1-d) v_t)     (pagerank.py:125)
//                 q'[t] = w_t * r'[t]   (the P_sr-weighted value the op side sums next time)
//                 s_k*u staged in LDS; the block's contiguous id range (u16 ids when N <= 65536)
//                 read coalesced into LDS, then each thread sums its trace in node order.
//     tile role   P_sr in compressed sparse blocks: traces cut in tiles of 2^tshift, the tile's
//                 q_k staged in LDS with coalesced loads, and each (tile, op) pair -- the op's
//                 traces inside the tile as u16 tile-local indices -- summed in trace order
//                 (a thread per short pair, a wave per long one) into part[pair].
//   k_iter_b, a wave per op: s'[o] = d * (sum of the op's pair partials in tile order / M_r(k)
//                 + alpha * sum_{p in ss(o)} pw_p * s_k[p] / M_s(k))                 (:122-124)
// The op side never gathers q from HBM at random (an op-major CSC did: 5% of HBM at 10M
// traces).  Maxima M_s, M_r (np.amax, :126-127) travel as bit patterns of non-negative doubles
// through atomicMax (exact, order-independent).  Normalisation of r is deferred:
// sum_t w_t (r'_t / M_r) is evaluated as (sum_t w_t r'_t) / M_r.  Every float reduction has a
// fixed order (no float atomics), so results are bitwise reproducible run to run.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <queue>
#include <type_traits>

#include "mr_internal.h"
#include "mr_prim.h"
#include "mr_sort.h"

namespace {

constexpr int TB = 256;             // trace-role block size (one trace per thread)
constexpr int LDS_NODES = 8192;     // su staged in LDS up to this many nodes (64 KiB)
constexpr int VCAP = 2048;          // trace-role ids staged per round in LDS (16 KiB of values)
constexpr int LONG_PAIR = 32;       // tile pairs longer than this are summed by a whole wave
constexpr int TSHIFT_MIN = 8, TSHIFT_MAX = 12;   // tiles of 256 .. 4096 traces

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_pr_reset(int32_t T, int64_t cap, int32_t N, float* pref, float* c_t, unsigned long long* hk, KCnt* cr, int32_t* flag,
                           double* scal) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < T) {
        pref[i] = 0.0f;
        c_t[i] = 0.0f;
    }
    if (i < cap) {
        hk[i] = 0ull;
        cr[i] = KCnt{0u, 0x7fffffff};
    }
    if (i < 8) flag[i] = 0;
    if (i < 8) scal[i] = 0.0;
}

// ---------------------------------------------------------------- graph constants
__global__ void k_op_consts(const int32_t* len_o, const int32_t* nchild, float* u_o, float* pw, int32_t N) {
    int32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= N) return;
    u_o[o] = len_o[o] > 0 ? (float)(1.0 / (double)len_o[o]) : 0.0f;
    pw[o] = nchild[o] > 0 ? (float)(1.0 / (double)nchild[o]) : 0.0f;
}
// per-graph constants in one launch: w_t = fp32(1/len_t) (fp64 1/n -> fp32), u_o, pw, and the
// u16 copy of the op ids (N <= 65536)
// (and clears `nz` words of the layout's scratch: tr_layout's histogram and slot counters)
__device__ __forceinline__ void graph_consts_body(int32_t blk, const int32_t* len_t, float* w_t, int32_t T,
                                                  const int32_t* len_o, const int32_t* nchild, float* u_o, float* pw,
                                                  int32_t N, const int32_t* ops, int64_t n, uint16_t* o16,
                                                  int32_t* zero, int32_t nz) {
    const int64_t i = (int64_t)blk * blockDim.x + threadIdx.x;
    if (i < nz) zero[i] = 0;
    if (i < T) w_t[i] = len_t[i] > 0 ? (float)(1.0 / (double)len_t[i]) : 0.0f;
    if (i < N) {
        u_o[i] = len_o[i] > 0 ? (float)(1.0 / (double)len_o[i]) : 0.0f;
        pw[i] = nchild[i] > 0 ? (float)(1.0 / (double)nchild[i]) : 0.0f;
    }
    // the u16 copy, four ids per thread (one 16-B load, one 8-B store instead of 2-B stores)
    if (o16 && 4 * i < n) {
        if (4 * i + 3 < n) {
            const int4 v = *(const int4*)(ops + 4 * i);
            uint2 w;
            w.x = (uint32_t)(uint16_t)v.x | ((uint32_t)(uint16_t)v.y << 16);
            w.y = (uint32_t)(uint16_t)v.z | ((uint32_t)(uint16_t)v.w << 16);
            *(uint2*)(o16 + 4 * i) = w;
        } else {
            for (int64_t k = 4 * i; k < n; ++k) o16[k] = (uint16_t)ops[k];
        }
    }
}
__global__ void k_graph_consts(const int32_t* len_t, float* w_t, int32_t T, const int32_t* len_o, const int32_t* nchild,
                               float* u_o, float* pw, int32_t N, const int32_t* ops, int64_t n, uint16_t* o16,
                               int32_t* zero, int32_t nz) {
    graph_consts_body((int32_t)blockIdx.x, len_t, w_t, T, len_o, nchild, u_o, pw, N, ops, n, o16, zero, nz);
}

// ---------------------------------------------------------------- P_sr tiles (compressed sparse blocks)
// entry (t, o) of the trace-major P_sr incidence -> key (tile(t), o), value t mod tile; a stable
// sort by key leaves every tile's entries in (op, trace) order
__global__ void k_tile_keys(const int64_t* off, const int32_t* ops, int32_t T, int tshift, int nb, uint64_t* key,
                            uint32_t* val) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const uint64_t hi = (uint64_t)(uint32_t)(t >> tshift) << nb;
    const uint32_t lt = (uint32_t)t & ((1u << tshift) - 1u);
    for (int64_t e = off[t]; e < off[t + 1]; ++e) {
        key[e] = hi | (uint32_t)ops[e];
        val[e] = lt;
    }
}
__global__ void k_key_heads(const uint64_t* key, int64_t n, int32_t* head) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) head[i] = (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}
__global__ void k_tile_pairs(const uint64_t* key, const uint32_t* val, const int32_t* head, const int64_t* hpos,
                             int64_t n, int nb, uint16_t* ltr, int32_t* pr_op, int64_t* pr_beg, int32_t* pr_tile) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    ltr[e] = (uint16_t)val[e];
    if (head[e]) {
        const int64_t p = hpos[e];
        const uint64_t k = key[e];
        pr_op[p] = (int32_t)(k & ((1ull << nb) - 1ull));
        pr_beg[p] = e;
        pr_tile[p] = (int32_t)(k >> nb);
    }
    if (e == n - 1) pr_beg[hpos[n]] = n;
}
// out[q] = first i in [0, n) with a[i] >= q (a sorted), q in [0, nq]; n from the device when d_n
template <class K>
__global__ void k_lower_bound(const K* a, int64_t n, const int64_t* d_n, int32_t nq, int32_t* out) {
    const int32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q > nq) return;
    int64_t lo = 0, hi = d_n ? *d_n : n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)a[mid] < (int64_t)q) lo = mid + 1; else hi = mid;
    }
    out[q] = (int32_t)lo;
}
__global__ void k_pair_op_keys(const int32_t* pr_op, int64_t np, uint64_t* key, uint32_t* val) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= np) return;
    key[p] = (uint64_t)(uint32_t)pr_op[p];
    val[p] = (uint32_t)p;
}
__global__ void k_long_flags(const int64_t* pr_beg, int64_t np, int32_t* flag) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < np) flag[p] = (pr_beg[p + 1] - pr_beg[p]) > LONG_PAIR ? 1 : 0;
}
__global__ void k_long_list(const int32_t* flag, const int64_t* pos, const int32_t* pr_tile, int64_t np, int32_t* lp,
                            int32_t* lp_tile) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= np || !flag[p]) return;
    lp[pos[p]] = (int32_t)p;
    lp_tile[pos[p]] = pr_tile[p];
}
__global__ void k_op_pairs(const uint64_t* skey, const uint32_t* sval, int64_t np, int32_t* op_pr, int32_t* op_key) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    op_pr[i] = (int32_t)sval[i];
    op_key[i] = (int32_t)skey[i];
}
// coverage = traces containing the op (trace_num_list, pagerank.py:98-104) = its pair lengths
__global__ void k_cov(const int32_t* op_pr_off, const int32_t* op_pr, const int64_t* pr_beg, int32_t N, int32_t* cov) {
    const int32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= N) return;
    int64_t c = 0;
    for (int32_t i = op_pr_off[o]; i < op_pr_off[o + 1]; ++i) c += pr_beg[op_pr[i] + 1] - pr_beg[op_pr[i]];
    cov[o] = (int32_t)c;
}

// fused-path coverage: histogram of the distinct (trace, op) incidence's op ids (N <= FX_NMAX:
// LDS counters per block, one global add per touched op)
__global__ void __launch_bounds__(256) k_cov_hist(const uint16_t* ids, int64_t n, int32_t N, int32_t* cov) {
    extern __shared__ int32_t hcnt[];
    for (int32_t o = threadIdx.x; o < N; o += 256) hcnt[o] = 0;
    __syncthreads();
    const int64_t per = (int64_t)256 * 64;
    const int64_t b0 = (int64_t)blockIdx.x * per;
    for (int64_t e = b0 + threadIdx.x; e < min(b0 + per, n); e += 256) atomicAdd(&hcnt[ids[e]], 1);
    __syncthreads();
    for (int32_t o = threadIdx.x; o < N; o += 256)
        if (hcnt[o]) atomicAdd(&cov[o], hcnt[o]);
}

// ---------------------------------------------------------------- op relabelling (fused, large N)
// ops by descending coverage (ties by op): key = ~cov << 14 | op (N <= 16384)
__global__ void k_relabel_keys(const int32_t* cov, int32_t N, uint64_t* key) {
    const int32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o < N) key[o] = ((uint64_t)(~(uint32_t)cov[o]) << 14) | (uint32_t)o;
}
__global__ void k_relabel_perm(const uint64_t* key, int32_t N, int32_t* perm, int32_t* inv) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int32_t o = (int32_t)(key[i] & 0x3fffu);
    perm[i] = o;
    inv[o] = i;
}
__global__ void k_relabel_ids(const uint16_t* ids, int64_t n, const int32_t* inv, uint16_t* out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < n) out[e] = (uint16_t)inv[ids[e]];
}

// ---------------------------------------------------------------- wide fused graphs (N > FX_NMAX)
// Ops relabelled by coverage; the WIDE_NA most covered ("hot") ops keep k_tr_a's LDS walk (u16
// ids, su and accumulator in LDS); the other ("cold") entries of each trace are summed per
// position by k_cold_trace and accumulated per op range by k_cold_ops (LDS accumulator of one
// range, (position, op) pairs grouped by range, position order within a range).
#ifndef MR_WIDE_NA
#define MR_WIDE_NA 10000
#endif
constexpr int32_t WIDE_NA = MR_WIDE_NA;   // (WIDE_NA + TR_PAD) * 16 B + the hot-op sums <= k_tr_a's LDS
constexpr int32_t WIDE_RW_MAX = 19456;  // ops per cold range: k_cold_ops' accumulator <= 152 KB
constexpr int WIDE_CB = 256;            // k_cold_ops blocks over all ranges (one per CU: LDS-bound)
constexpr int WIDE_CT = 1024;           // k_cold_ops block size
constexpr int32_t WIDE_HIST = 32768;    // coverage counters in LDS (ops above: global adds)
constexpr int WIDE_RMAX = 255;          // ranges (8-bit sort digit)

__global__ void __launch_bounds__(256) k_cov_hist_w(const int32_t* ids, int64_t n, int32_t N, int32_t* cov) {
    extern __shared__ int32_t hcnt[];
    const int32_t NL = min(N, WIDE_HIST);
    for (int32_t o = threadIdx.x; o < NL; o += 256) hcnt[o] = 0;
    __syncthreads();
    const int64_t per = (int64_t)256 * 256;
    const int64_t b0 = (int64_t)blockIdx.x * per;
    for (int64_t e = b0 + threadIdx.x; e < min(b0 + per, n); e += 256) {
        const int32_t o = ids[e];
        if (o < NL) atomicAdd(&hcnt[o], 1);
        else atomicAdd(&cov[o], 1);
    }
    __syncthreads();
    for (int32_t o = threadIdx.x; o < NL; o += 256)
        if (hcnt[o]) atomicAdd(&cov[o], hcnt[o]);
}
// key = ~cov << nbo | op (descending coverage, ties by op)
__global__ void k_relabel_keys_w(const int32_t* cov, int32_t N, int nbo, uint64_t* key) {
    const int32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o < N) key[o] = ((uint64_t)(~(uint32_t)cov[o]) << nbo) | (uint32_t)o;
}
__global__ void k_relabel_perm_w(const uint64_t* key, int32_t N, uint64_t omask, int32_t* perm, int32_t* inv) {
    const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const int32_t o = (int32_t)(key[i] & omask);
    perm[i] = o;
    inv[o] = i;
}
// per trace: hot entries (at least one: a trace without hot ops walks the pad id NA) and cold ones
__global__ void k_wide_count(const int64_t* off, const int32_t* ops, const int32_t* inv, int32_t T, int32_t NA,
                             int32_t* nh, int32_t* nc) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    int32_t h = 0, c = 0;
    for (int64_t e = off[t]; e < off[t + 1]; ++e) {
        if (inv[ops[e]] < NA) ++h;
        else ++c;
    }
    nh[t] = max(h, 1);
    nc[t] = c;
}
__global__ void k_wide_hot(const int64_t* off, const int32_t* ops, const int32_t* inv, int32_t T, int32_t NA,
                           const int64_t* hoff, uint16_t* hot16) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    int64_t k = hoff[t];
    const int64_t k0 = k;
    for (int64_t e = off[t]; e < off[t + 1]; ++e) {
        const int32_t o = inv[ops[e]];
        if (o < NA) hot16[k++] = (uint16_t)o;
    }
    if (k == k0) hot16[k] = (uint16_t)NA;
}
__global__ void k_wide_cold_cnt(const int32_t* tperm, const int32_t* nc, int32_t T, int32_t* cnt) {
    const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < T) cnt[p] = nc[tperm[p]];
}
// cold entries in position order: op ids for k_cold_trace, and sort keys p << 24 | (op - range
// base) << 8 | range whose one stable 8-bit pass groups them by range (positions stay ascending)
// walked in trace order: thread t reads its own op list (a wave's traces are contiguous in the
// CSR) and writes its cold entries at its position's slots (tpos = inverse of tperm) -- walking
// in position order read a random trace per lane, ~16 lines fetched per trace's 60 B (C5's rank
// share: 21 GB of FETCH_SIZE in one 2.8 ms launch)
__global__ void k_wide_cold_fill_t(const int32_t* tpos, const int64_t* off, const int32_t* ops, const int32_t* inv,
                                   int32_t T, int32_t NA, int32_t RW, const int64_t* coff, int32_t* cops,
                                   uint64_t* key) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const int32_t p = tpos[t];
    int64_t k = coff[p];
    for (int64_t e = off[t]; e < off[t + 1]; ++e) {
        const int32_t o = inv[ops[e]];
        if (o < NA) continue;
        const int32_t r = (o - NA) / RW;
        cops[k] = o;
        key[k] = ((uint64_t)p << 24) | ((uint64_t)(o - NA - r * RW) << 8) | (uint64_t)r;
        ++k;
    }
}
// rb[r] = first pair of range r (rb[R] = n)
__global__ void k_wide_bounds(const uint64_t* key, int64_t n, int32_t R, int64_t* rb) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t r = (int32_t)(key[i] & 0xff);
    const int32_t rp = i ? (int32_t)(key[i - 1] & 0xff) : -1;
    for (int32_t x = rp + 1; x <= r; ++x) rb[x] = i;
    if (i == n - 1)
        for (int32_t x = r + 1; x <= R; ++x) rb[x] = n;
}
__global__ void k_wide_unpack(const uint64_t* key, int64_t n, int32_t* cp_pos, uint16_t* cp_op) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = key[i];
    cp_pos[i] = (int32_t)(k >> 24);
    cp_op[i] = (uint16_t)((k >> 8) & 0xffff);
}
// the widest position span of a k_cold_ops block: an op gets at most that many adds in one row
__global__ void k_wide_span(const int64_t* cb_beg, int32_t n_cb, const int32_t* cp_pos, unsigned long long* span) {
    const int32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_cb) return;
    const int64_t b0 = cb_beg[b], b1 = cb_beg[b + 1];
    if (b1 > b0) atomicMax(span, (unsigned long long)(cp_pos[b1 - 1] - cp_pos[b0] + 1));
}

// Cold entries of the short-tile walk: per wave tile ceil(max cold of its traces / 2) chunks of
// 64 lanes x 2 u32 labels, a lane's entries in cold_ops_p order (k_cold_trace's), pads N + lane
// (a zero su slot).  Secondary sort key of the wide layout (cold count) keeps tiles homogeneous.
__global__ void k_ctile_cnt(const int32_t* coff_p, int32_t T, int32_t W, int32_t* cnt) {
    const int32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= W) return;
    int32_t m = 0;
    for (int32_t p = k * WAVE; p < min(k * WAVE + WAVE, T); ++p) m = max(m, coff_p[p + 1] - coff_p[p]);
    cnt[k] = (m + 1) >> 1;
}
__global__ void k_ctile_fill(const int32_t* coff_p, const int32_t* cops, const int64_t* cc64, int32_t T, int32_t N,
                             int32_t W, uint32_t* ctids) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)W * WAVE) return;
    const int32_t k = (int32_t)(i / WAVE), lane = (int32_t)(i % WAVE);
    const int32_t p = k * WAVE + lane;
    const int32_t a = p < T ? coff_p[p] : 0, n = p < T ? coff_p[p + 1] - a : 0;
    const int64_t c0 = cc64[k], nc = cc64[k + 1] - c0;
    for (int64_t c = 0; c < nc; ++c)
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int64_t e = 2 * c + q;
            ctids[((size_t)(c0 + c) * WAVE + lane) * 2 + q] = e < n ? (uint32_t)cops[a + e] : (uint32_t)(N + lane);
        }
}
// sort keys of a layout with a secondary key: (length << 4 | min(skey, 15)), the trace as value
__global__ void k_tr_skey(const int64_t* off, const int32_t* skey, int32_t T, uint64_t* key, uint32_t* val) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    key[t] = ((uint64_t)(off[t + 1] - off[t]) << 4) | (uint64_t)(skey ? min(skey[t], 15) : 0);
    val[t] = (uint32_t)t;
}
__global__ void k_tr_perm_w(const uint32_t* val, const float* w_t, int32_t T, int32_t* tperm, float* w_tp) {
    const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= T) return;
    const int32_t t = (int32_t)val[p];
    tperm[p] = t;
    w_tp[p] = w_t[t];
}

// ---------------------------------------------------------------- trace-parallel layout (k_tr_a)
// Traces by op count: a counting sort (lengths <= N <= FX_NMAX), order within a length free --
// nothing numeric depends on it (a trace's ids are rotated by trace mod len, not by position;
// the accumulator is integer).  Blocks of TRB threads take TRB * TR_PER traces each: 16 per
// thread for large graphs, 2 for window-sized ones (187k traces in 12 blocks had left the chip idle)
constexpr int TRB = 1024, TR_PER_BIG = 16, TR_PER_SMALL = 2;
template <int TR_PER>
__device__ __forceinline__ void tr_hist_body(int32_t blk, const int64_t* off, int32_t T, int32_t nbin, int32_t* hist) {
    extern __shared__ int32_t lh[];
    for (int32_t i = threadIdx.x; i < nbin; i += TRB) lh[i] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blk * TRB * TR_PER;
    for (int32_t j = 0; j < TR_PER; ++j) {
        const int64_t t = t0 + (int64_t)j * TRB + threadIdx.x;
        if (t < T) atomicAdd(&lh[off[t + 1] - off[t]], 1);
    }
    __syncthreads();
    for (int32_t i = threadIdx.x; i < nbin; i += TRB)
        if (lh[i]) atomicAdd(&hist[i], lh[i]);
}
template <int TR_PER>
__global__ void __launch_bounds__(TRB) k_tr_hist(const int64_t* off, int32_t T, int32_t nbin, int32_t* hist) {
    tr_hist_body<TR_PER>((int32_t)blockIdx.x, off, T, nbin, hist);
}
// positions: bin start (cursor, claimed per block and bin) + the trace's rank in its block's bin
// A bin's slots: boff given -- its start plus the bin's remaining count, handed out from the end
// (hist is consumed, no cursor copy); boff null (nbin <= TP_LSCAN) -- each block scans the
// histogram in LDS itself and claims slots through `taken` (no scan launch)
constexpr int TP_LSCAN = 8192;
template <int TR_PER>
__device__ __forceinline__ void tr_place_body(int32_t blk, const int64_t* off, int32_t T, int32_t nbin,
                                              const int64_t* boff, int32_t* hist, int32_t* taken, const float* w_t,
                                              int32_t* tperm, float* w_tp, int32_t* tpos) {
    extern __shared__ int32_t lh[];
    int32_t* lbase = lh + nbin;
    for (int32_t i = threadIdx.x; i < nbin; i += TRB) lh[i] = 0;
    __syncthreads();
    const int64_t t0 = (int64_t)blk * TRB * TR_PER;
    int32_t rk[TR_PER], ln[TR_PER];
#pragma unroll
    for (int32_t j = 0; j < TR_PER; ++j) {
        const int64_t t = t0 + (int64_t)j * TRB + threadIdx.x;
        ln[j] = t < T ? (int32_t)(off[t + 1] - off[t]) : -1;
        rk[j] = ln[j] >= 0 ? atomicAdd(&lh[ln[j]], 1) : 0;
    }
    __syncthreads();
    if (boff) {
        for (int32_t i = threadIdx.x; i < nbin; i += TRB)
            if (lh[i]) lbase[i] = (int32_t)boff[i] + atomicSub(&hist[i], lh[i]) - lh[i];
    } else {
        __shared__ int32_t sbuf[TRB];
        const int32_t per = (nbin + TRB - 1) / TRB, b0 = threadIdx.x * per, b1 = min(b0 + per, nbin);
        int32_t run = 0;
        for (int32_t i = b0; i < b1; ++i) run += hist[i];
        sbuf[threadIdx.x] = run;
        __syncthreads();
        for (int o = 1; o < TRB; o <<= 1) {
            const int32_t v = threadIdx.x >= o ? sbuf[threadIdx.x - o] : 0;
            __syncthreads();
            sbuf[threadIdx.x] += v;
            __syncthreads();
        }
        run = sbuf[threadIdx.x] - run;   // exclusive start of this thread's bins
        for (int32_t i = b0; i < b1; ++i) {
            const int32_t c = hist[i];
            lbase[i] = run + (lh[i] ? atomicAdd(&taken[i], lh[i]) : 0);
            run += c;
        }
    }
    __syncthreads();
#pragma unroll
    for (int32_t j = 0; j < TR_PER; ++j) {
        if (ln[j] < 0) continue;
        const int32_t t = (int32_t)(t0 + (int64_t)j * TRB + threadIdx.x);
        const int32_t p = lbase[ln[j]] + rk[j];
        tperm[p] = t;
        w_tp[p] = w_t[t];
        if (tpos) tpos[t] = p;   // (the inverse, stored in trace order)
    }
}
template <int TR_PER>
__global__ void __launch_bounds__(TRB) k_tr_place(const int64_t* off, int32_t T, int32_t nbin, const int64_t* boff,
                                                  int32_t* hist, int32_t* taken, const float* w_t, int32_t* tperm,
                                                  float* w_tp) {
    tr_place_body<TR_PER>((int32_t)blockIdx.x, off, T, nbin, boff, hist, taken, w_t, tperm, w_tp, nullptr);
}
// chunks of 4 ids per wave tile (its last position holds its longest trace: lengths ascend), their
// exclusive prefix and its int32 copy in one launch: runs of TS_TILE wave tiles per block, chained
// by decoupled look-back
constexpr int TS_T = 256, TS_I = 8, TS_TILE = TS_T * TS_I;
__device__ __forceinline__ void tr_chunk_scan_body(int32_t tile_, int32_t ntiles, const int32_t* tperm,
                                                   const int64_t* off, int32_t T, int32_t n_wt, int64_t* c64,
                                                   int32_t* coff, unsigned long long* st, uint64_t epoch) {
    __shared__ int64_t sa[TS_T];
    __shared__ int64_t ex;
    const int tid = threadIdx.x;
    const int64_t tile = tile_, base = tile * TS_TILE + (int64_t)tid * TS_I;
    int64_t v[TS_I], a = 0;
#pragma unroll
    for (int i = 0; i < TS_I; ++i) {
        const int64_t k = base + i;
        v[i] = 0;
        if (k < n_wt) {
            const int32_t t = tperm[min(k * WAVE + WAVE - 1, (int64_t)T - 1)];
            v[i] = (off[t + 1] - off[t] + 3) >> 2;
        }
        a += v[i];
    }
    sa[tid] = a;
    __syncthreads();
    for (int o = 1; o < TS_T; o <<= 1) {
        const int64_t x = tid >= o ? sa[tid - o] : 0;
        __syncthreads();
        sa[tid] += x;
        __syncthreads();
    }
    if (tid < WAVE) {
        const int64_t e = dl_lookback_wave(st, tile, sa[TS_T - 1], epoch);
        if (tid == 0) ex = e;
        if (tid == 0 && tile == (int64_t)ntiles - 1) {
            c64[n_wt] = ex + sa[TS_T - 1];
            coff[n_wt] = (int32_t)(ex + sa[TS_T - 1]);
        }
    }
    __syncthreads();
    int64_t r = ex + sa[tid] - a;
#pragma unroll
    for (int i = 0; i < TS_I; ++i) {
        const int64_t k = base + i;
        if (k < n_wt) {
            c64[k] = r;
            coff[k] = (int32_t)r;
        }
        r += v[i];
    }
}
__global__ void __launch_bounds__(TS_T) k_tr_chunk_scan(const int32_t* tperm, const int64_t* off, int32_t T, int32_t n_wt,
                                                        int64_t* c64, int32_t* coff, unsigned long long* st,
                                                        uint64_t epoch) {
    tr_chunk_scan_body((int32_t)blockIdx.x, (int32_t)gridDim.x, tperm, off, T, n_wt, c64, coff, st, epoch);
}
__global__ void k_tr_coff(const int64_t* c64, int32_t n, int32_t* coff) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) coff[i] = (int32_t)c64[i];
}
// k_tr_a's per-wave runs of tiles of about equal cost (chunks + 2 per tile: a tile's q / r words
// weigh about two chunks), in one block on the device (no host round trip): cut[i] = first tile
// whose cost prefix reaches total * i / nw.  A block (NW waves) must stay within 1023 tiles (65472
// traces: the fixed-point budget); a cost cut that breaks it falls back to equal tile counts (the
// host sizes the grid so those fit).  scale = {2^SC, 2^-SC}: SC = 64 - bits(most traces of a block)
// (the finest scale whose row entries stay below 2^64), or scfix > 0: a scale that does not depend
// on the cut -- window graphs (layout order) take 64 - bits(min(T, 65472)), so a trace's X, hence
// every exact limb sum, is the same however a batch's group cuts the graph into blocks, and a window
// ranks bitwise alike in any batch or group.
constexpr int TC_T = 1024, TC_MAX = 16384;
__device__ __forceinline__ void tr_cut_body(const int32_t* coff, int32_t W, int32_t nw, int32_t NW, int32_t* cut,
                                            double* scale, double tw, int scfix) {
    __shared__ int32_t lc[TC_MAX + 1];
    __shared__ int32_t mx;
    if (threadIdx.x == 0) mx = 0;
    const double total = W ? (double)coff[W] + tw * (double)W : 0.0;
    for (int32_t i = threadIdx.x; i <= nw; i += TC_T) {
        const double target = total * (double)i / (double)nw;
        int32_t lo = 0, hi = W;
        while (lo < hi) {
            const int32_t mid = (lo + hi) >> 1;
            if ((double)coff[mid] + tw * (double)mid < target) lo = mid + 1;
            else hi = mid;
        }
        lc[i] = i == nw ? W : lo;
    }
    __syncthreads();
    const int32_t nb = nw / NW;
    for (int32_t b = threadIdx.x; b < nb; b += TC_T) atomicMax(&mx, lc[(b + 1) * NW] - lc[b * NW]);
    __syncthreads();
    if (mx > 1023) {   // (uniform: read after the barrier)
        __syncthreads();
        if (threadIdx.x == 0) mx = 0;
        for (int32_t i = threadIdx.x; i <= nw; i += TC_T) lc[i] = (int32_t)((int64_t)W * i / nw);
        __syncthreads();
        for (int32_t b = threadIdx.x; b < nb; b += TC_T) atomicMax(&mx, lc[(b + 1) * NW] - lc[b * NW]);
        __syncthreads();
    }
    for (int32_t i = threadIdx.x; i <= nw; i += TC_T) cut[i] = lc[i];
    if (threadIdx.x == 0) {
        const int sc = scfix > 0 ? scfix : __clzll((unsigned long long)max(mx, 1) * WAVE);   // 64 - bits(traces)
        scale[0] = __longlong_as_double((long long)(1023 + sc) << 52);
        scale[1] = __longlong_as_double((long long)(1023 - sc) << 52);
    }
}
__global__ void __launch_bounds__(TC_T) k_tr_cut(const int32_t* coff, int32_t W, int32_t nw, int32_t NW, int32_t* cut,
                                                 double* scale, double tw, int scfix) {
    tr_cut_body(coff, W, nw, NW, cut, scale, tw, scfix);
}
// the cuts of a batch's graphs in one launch (block g: graph g)
struct CutArg {
    const int32_t* coff;
    int32_t* cut;
    double* scale;
    int32_t W, nw, NW;
    float tw;   // a tile's fixed cost in chunks
    int32_t scfix;   // > 0: the graph's cut-independent scale
};
constexpr int TC_BATCH = 64;
struct CutBatch {
    CutArg a[TC_BATCH];
};
__global__ void __launch_bounds__(TC_T) k_tr_cut_b(CutBatch b) {
    const CutArg& x = b.a[blockIdx.x];
    tr_cut_body(x.coff, x.W, x.nw, x.NW, x.cut, x.scale, (double)x.tw, x.scfix);
}
// thread per (tile, lane): the lane's trace rotated by (trace mod len), then pads N + lane
__device__ __forceinline__ void tr_fill_body(int32_t blk, const int32_t* tperm, const int64_t* off, const uint16_t* ids,
                                             const int64_t* c64, int32_t T, int32_t N, int32_t n_wt, uint16_t* tids) {
    const int64_t i = (int64_t)blk * blockDim.x + threadIdx.x;
    if (i >= (int64_t)n_wt * WAVE) return;
    const int32_t k = (int32_t)(i / WAVE), lane = (int32_t)(i % WAVE);
    const int64_t p = (int64_t)k * WAVE + lane;
    int64_t a = 0, len = 0, rot = 0;
    if (p < T) {
        const int32_t t = tperm[p];
        a = off[t];
        len = off[t + 1] - a;
        rot = len ? t % len : 0;
    }
    const int64_t nc = c64[k + 1] - c64[k];
    unsigned long long* dst = (unsigned long long*)tids + (size_t)c64[k] * WAVE + lane;   // 4 ids per 8-B store
    // the ids from the rotation start, padded with N + lane; TF_CH chunks per round, their loads
    // issued together (id e of the rotation sits at (rot + e) mod len: no carried index), so a
    // window trace of <= 16 ids costs one load latency instead of one per chunk
    constexpr int TF_CH = 4;
    for (int64_t c0 = 0; c0 < nc; c0 += TF_CH) {
        uint16_t idv[4 * TF_CH];
#pragma unroll
        for (int q = 0; q < 4 * TF_CH; ++q) {
            const int64_t e = 4 * c0 + q, jx = rot + e;
            idv[q] = e < len ? ids[a + (jx >= len ? jx - len : jx)] : (uint16_t)(N + lane);
        }
#pragma unroll
        for (int u = 0; u < TF_CH; ++u)
            if (c0 + u < nc)
                dst[(size_t)(c0 + u) * WAVE] = (unsigned long long)idv[4 * u] | (unsigned long long)idv[4 * u + 1] << 16 |
                                               (unsigned long long)idv[4 * u + 2] << 32 |
                                               (unsigned long long)idv[4 * u + 3] << 48;
    }
}
__global__ void k_tr_fill(const int32_t* tperm, const int64_t* off, const uint16_t* ids, const int64_t* c64, int32_t T,
                          int32_t N, int32_t n_wt, uint16_t* tids) {
    tr_fill_body((int32_t)blockIdx.x, tperm, off, ids, c64, T, N, n_wt, tids);
}
// Register-accumulated hot ops (large graphs): the HOT_MAX ops present in the most traces leave the
// id chunks -- op 0 of the C4 graph is in every trace, so each 16-lane atomic group of every step
// that holds it adds to ONE LDS address 16 times -- and trace t keeps the bit set of the hot ops it
// holds instead (hmask).  A trace whose ops are all hot keeps its first one in the list (no empty
// traces: every tile has a chunk).  hidx[o] = h or -1.
#ifndef MR_TR_TIERS512
#define MR_TR_TIERS512 4   // short-tile tiers of the 512-thread k_tr_a (window graphs: occupancy)
#endif
constexpr int TR_TIERS_EXT = 8;   // short-tile tiers of the EXT (kind-compressed / wide) variants
#ifndef MR_TR_TIERS_W32
#define MR_TR_TIERS_W32 5   // ... of the fp32 wide variant (EXT & 8: its pipelined cold registers; 6 spilled)
#endif
constexpr int TR_TIERS_W32 = MR_TR_TIERS_W32;
#ifndef MR_HOT_MAX
#define MR_HOT_MAX 8
#endif
constexpr int HOT_MAX = MR_HOT_MAX;
__global__ void __launch_bounds__(256) k_hot_count(const int64_t* off, const uint16_t* ids, int32_t T, const int8_t* hidx,
                                                   int32_t N, int32_t* rlen, uint8_t* mask) {
    extern __shared__ int8_t lh8[];
    for (int32_t o = threadIdx.x; o < N; o += 256) lh8[o] = hidx[o];
    __syncthreads();
    const int32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= T) return;
    uint32_t m = 0, first = 0xffu;
    int32_t n = 0;
    for (int64_t e = off[t]; e < off[t + 1]; ++e) {
        const int h = lh8[ids[e]];
        if (h >= 0) {
            if (first == 0xffu) first = (uint32_t)h;
            m |= 1u << h;
        } else {
            ++n;
        }
    }
    if (n == 0 && m) {   // all hot: the first stays in the list
        m &= ~(1u << first);
        n = 1;
    }
    rlen[t] = n;
    mask[t] = (uint8_t)m;
}
__global__ void __launch_bounds__(256) k_hot_fill(const int64_t* off, const uint16_t* ids, int32_t T, const int8_t* hidx,
                                                  int32_t N, const uint8_t* mask, const int64_t* roff, uint16_t* rids) {
    extern __shared__ int8_t lh8[];
    for (int32_t o = threadIdx.x; o < N; o += 256) lh8[o] = hidx[o];
    __syncthreads();
    const int32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= T) return;
    const uint32_t m = mask[t];
    int64_t w = roff[t];
    for (int64_t e = off[t]; e < off[t + 1]; ++e) {
        const uint16_t o = ids[e];
        const int h = lh8[o];
        if (h < 0 || !((m >> h) & 1u)) rids[w++] = o;
    }
}
__global__ void k_hot_perm(const int32_t* tperm, const uint8_t* mask, int32_t T, uint8_t* hmask) {
    const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < T) hmask[p] = mask[tperm[p]];
}

constexpr int64_t TR_LARGE = (int64_t)1 << 20;   // "large graph": the hot-op threshold

// The prepare of several small fused graphs (a window's two) in one launch per step: block ranges
// per graph, the same bodies (mr_graph_prepare_batch)
struct PDev {
    int32_t T, N, nbin, W, nz, n_cs;
    int64_t nnz, st_off;
    int32_t b_gc, b_th, b_cs, b_fill;
    const int32_t *len_t, *len_o, *nchild, *rs_ops;
    const int64_t* rs_off;
    float *w_t, *u_o, *pw, *w_tp;
    uint16_t *rs16, *tids;
    int32_t *trz, *tperm, *coff, *tpos;
    int64_t* c64;
};
__device__ __forceinline__ int32_t pd_graph(const PDev* pd, int32_t n, int32_t blk, int which) {
    int32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const int32_t mid = (lo + hi + 1) >> 1;
        const PDev& g = pd[mid];
        const int32_t s0 = which == 0 ? g.b_gc : which == 1 ? g.b_th : which == 2 ? g.b_cs : g.b_fill;
        if (s0 <= blk) lo = mid; else hi = mid - 1;
    }
    return lo;
}
__global__ void k_graph_consts_b(const PDev* __restrict__ pd, int32_t n) {
    const PDev& G = pd[pd_graph(pd, n, (int32_t)blockIdx.x, 0)];
    graph_consts_body((int32_t)blockIdx.x - G.b_gc, G.len_t, G.w_t, G.T, G.len_o, G.nchild, G.u_o, G.pw, G.N, G.rs_ops,
                      G.nnz, G.rs16, G.trz, G.nz);
}
__global__ void __launch_bounds__(TRB) k_tr_hist_b(const PDev* __restrict__ pd, int32_t n) {
    const PDev& G = pd[pd_graph(pd, n, (int32_t)blockIdx.x, 1)];
    tr_hist_body<TR_PER_SMALL>((int32_t)blockIdx.x - G.b_th, G.rs_off, G.T, G.nbin, G.trz);
}
__global__ void __launch_bounds__(TRB) k_tr_place_b(const PDev* __restrict__ pd, int32_t n) {
    const PDev& G = pd[pd_graph(pd, n, (int32_t)blockIdx.x, 1)];
    tr_place_body<TR_PER_SMALL>((int32_t)blockIdx.x - G.b_th, G.rs_off, G.T, G.nbin, nullptr, G.trz, G.trz + G.nbin,
                                G.w_t, G.tperm, G.w_tp, G.tpos);
}
__global__ void __launch_bounds__(TS_T) k_tr_chunk_scan_b(const PDev* __restrict__ pd, int32_t n, unsigned long long* st,
                                                         uint64_t epoch) {
    const PDev& G = pd[pd_graph(pd, n, (int32_t)blockIdx.x, 2)];
    tr_chunk_scan_body((int32_t)blockIdx.x - G.b_cs, G.n_cs, G.tperm, G.rs_off, G.T, G.W, G.c64, G.coff, st + G.st_off,
                       epoch);
}
__global__ void k_tr_fill_b(const PDev* __restrict__ pd, int32_t n) {
    const PDev& G = pd[pd_graph(pd, n, (int32_t)blockIdx.x, 3)];
    tr_fill_body((int32_t)blockIdx.x - G.b_fill, G.tperm, G.rs_off, G.rs16, G.c64, G.T, G.N, G.W, G.tids);
}
__global__ void k_tr_gather(const float* src, const int32_t* tperm, int32_t T, float* dst) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < T) dst[p] = src[tperm[p]];
}

// ---------------------------------------------------------------- kinds (pagerank.py:54-66)
// kind[t] = size of the class of traces with an equal P_sr column: key = (op set, fp32(1/len_t)).
// Open-addressing hash table of 64-bit keys; a second pass verifies every member against the
// slot's representative, so a hash collision is detected (flag) rather than miscounted.
constexpr int KB = 256, KLDS = 512;   // kinds: block size, LDS table slots

// Set hash of a trace's key (its distinct ascending op ids, fp32(1/len_t), the id count):
// mix64(mix64(seed ^ wb ^ n << 32) + sum_op mix64(op ^ seed)).  Order-free, so the per-thread
// walk below and k_kind_insert's cooperative u16 form give the same key for the same trace (a
// requirement across ranks of a sharded graph).  CHK: a second, independently seeded hash of
// the same words, which travels with the key between ranks to catch a 64-bit key collision.
__device__ __forceinline__ uint64_t kind_fold(uint64_t seed, uint64_t wb, int64_t n, uint64_t acc) {
    const uint64_t h = mix64(mix64(seed ^ wb ^ ((uint64_t)n << 32)) + acc);
    return h ? h : 1;
}
template <bool CHK>
__device__ __forceinline__ uint64_t kind_hash2(const int64_t* off, const int32_t* ops, const float* w_t,
                                               int32_t t, uint64_t seed, uint64_t seed2, uint64_t* h2) {
    const int64_t e0 = off[t], e1 = off[t + 1];
    const uint64_t wb = e1 > e0 ? (uint64_t)__float_as_uint(w_t[t]) : 0ull;
    uint64_t a = 0, a2 = 0;
    for (int64_t e = e0; e < e1; ++e) {
        const uint64_t o = (uint64_t)(uint32_t)ops[e];
        a += mix64(o ^ seed);
        if (CHK) a2 += mix64(o ^ seed2);
    }
    if (CHK) *h2 = kind_fold(seed2, wb, e1 - e0, a2);
    return kind_fold(seed, wb, e1 - e0, a);
}
constexpr uint64_t KCHK_SEED = 0x0ddba11cafeull;

// Two-level insertion: traces of a block are first counted in an LDS table (hot kinds -- the
// same few call paths in thousands of traces -- would otherwise serialise on one global
// counter), then each distinct key of the block does ONE global insert + add.
// CHK (sharded graphs on >1 rank): the representative's check hash is stored per global slot
// (chk) for the cross-rank merge, computed in the same walk instead of a later re-read.
// IDW 2 / 4 (u16 ids, N <= 65536 / int32 ids): the block's 256 traces are hashed cooperatively --
// the threads stream the block's contiguous id range in aligned 16-B chunks (8 / 4 ids), coalesced
// across the wave, and add mix64(op) into per-trace LDS sums (an order-free SET hash: the ids of a
// trace are distinct and ascending, so the set is the list).  The walk-per-thread form (IDW 0,
// MR_KIND_WALK) reads one trace per lane, ~60 B apart (C5's kinds: 4.6 ms of dependent loads).
// Either hash only buckets traces; membership is decided by an exact comparison.
// Set hashes of the block's KB traces (tb = first trace), through per-trace LDS sums (loff, lacc,
// lacc2: KB + 1 / KB / KB entries) or a walk per thread.  Every thread of the block must call it;
// *h (and *h2 with CHK) is set for t < T.
// IDW (id width of the cooperative walk): 2 -- u16 ids (rs16, N <= 65536), 4 -- int32 ids (wide
// graphs: C5's 100k ops; the same 16-B chunks, 4 ids each), 0 -- a walk per thread (MR_KIND_WALK).
template <bool CHK, int IDW>
__device__ __forceinline__ void kind_block_hash(const int64_t* off, const int32_t* ops, const uint16_t* o16,
                                                const float* w_t, int32_t T, int32_t tb, uint64_t seed, int64_t* loff,
                                                unsigned long long* lacc, unsigned long long* lacc2, uint64_t* h,
                                                uint64_t* h2) {
    const int32_t t = tb + threadIdx.x;
    if constexpr (IDW != 0) {
        constexpr int IPC = IDW == 2 ? 8 : 4;   // ids per 16-B chunk
        __shared__ int64_t s_end;               // the id array's end (the last chunk's loads stop there)
        const int nt = min(KB, T - tb);
        if ((int)threadIdx.x < nt) {
            loff[threadIdx.x] = off[t];
            lacc[threadIdx.x] = 0ull;
            if (CHK) lacc2[threadIdx.x] = 0ull;
        }
        if (threadIdx.x == 0) {
            loff[nt] = off[tb + nt];
            s_end = off[T];
        }
        __syncthreads();
        const int64_t b = loff[0], e = loff[nt], eall = s_end;
        for (int64_t c = (b & ~(int64_t)(IPC - 1)) + (int64_t)IPC * threadIdx.x; c < e; c += (int64_t)IPC * KB) {
            uint32_t wd[4];
            if (IDW == 2 || c + IPC <= eall) {   // (rs16 holds nnz + 8 ids)
                const uint4 v = IDW == 2 ? *reinterpret_cast<const uint4*>(o16 + c)
                                         : *reinterpret_cast<const uint4*>(ops + c);
                wd[0] = v.x, wd[1] = v.y, wd[2] = v.z, wd[3] = v.w;
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) wd[k] = c + k < eall ? (uint32_t)ops[c + k] : 0u;
            }
            const int64_t p0 = c > b ? c : b;
            int lo = 0, hi = nt - 1;   // the trace holding p0: last lt with loff[lt] <= p0
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (loff[mid] <= p0) lo = mid;
                else hi = mid - 1;
            }
            int lt = lo;
            int64_t nb = loff[lt + 1];
            unsigned long long a = 0ull, a2 = 0ull;
            bool any = false;
#pragma unroll
            for (int k = 0; k < IPC; ++k) {
                const int64_t idx = c + k;
                if (idx < b || idx >= e) continue;
                while (idx >= nb) {
                    if (any) {
                        atomicAdd(&lacc[lt], a);
                        if (CHK) atomicAdd(&lacc2[lt], a2);
                    }
                    a = a2 = 0ull;
                    any = false;
                    ++lt;
                    nb = loff[lt + 1];
                }
                const uint64_t op = IDW == 2 ? (wd[k >> 1] >> ((k & 1) * 16)) & 0xffffu : (uint64_t)wd[k];
                a += mix64(op ^ seed);
                if (CHK) a2 += mix64(op ^ KCHK_SEED);
                any = true;
            }
            if (any) {
                atomicAdd(&lacc[lt], a);
                if (CHK) atomicAdd(&lacc2[lt], a2);
            }
        }
        __syncthreads();
    }
    if (t < T) {
        if constexpr (IDW != 0) {
            const int64_t n = loff[threadIdx.x + 1] - loff[threadIdx.x];
            const uint64_t wb = n > 0 ? (uint64_t)__float_as_uint(w_t[t]) : 0ull;
            *h = kind_fold(seed, wb, n, lacc[threadIdx.x]);
            if (CHK) *h2 = kind_fold(KCHK_SEED, wb, n, lacc2[threadIdx.x]);
        } else {
            *h = kind_hash2<CHK>(off, ops, w_t, t, seed, KCHK_SEED, h2);
        }
    }
}

template <bool CHK, int IDW>
__device__ __forceinline__ void kind_insert_body(int32_t blk, const int64_t* off, const int32_t* ops, const uint16_t* o16,
                                                 const float* w_t, int32_t T, unsigned long long* hk, KCnt* cr,
                                                 int32_t* slot_of, uint64_t mask, uint64_t seed, uint64_t* chk,
                                                 uint64_t hmask) {
    __shared__ unsigned long long lkey[KLDS];
    __shared__ uint32_t lcnt[KLDS];
    __shared__ int32_t lrep[KLDS];
    __shared__ int32_t lglob[KLDS];
    __shared__ uint64_t lchk[CHK ? KLDS : 1];
    __shared__ int64_t loff[IDW ? KB + 1 : 1];
    __shared__ unsigned long long lacc[IDW ? KB : 1], lacc2[IDW && CHK ? KB : 1];
    for (int i = threadIdx.x; i < KLDS; i += KB) {
        lkey[i] = 0ull;
        lcnt[i] = 0u;
        lrep[i] = 0x7fffffff;
    }
    const int32_t tb = blk * KB;
    const int32_t t = tb + threadIdx.x;
    uint64_t h = 0, h2 = 0;
    kind_block_hash<CHK, IDW>(off, ops, o16, w_t, T, tb, seed, loff, lacc, lacc2, &h, &h2);
    __syncthreads();
    int myslot = -1;
    if (t < T) {
        h &= hmask;   // ~0 (tests narrow it to force collisions)
        if (!h) h = 1;
        int s = (int)(h & (KLDS - 1));
        for (;;) {
            unsigned long long k = atomicCAS(&lkey[s], 0ull, (unsigned long long)h);
            if (k == 0ull || k == h) break;
            s = (s + 1) & (KLDS - 1);
        }
        atomicAdd(&lcnt[s], 1u);
        atomicMin(&lrep[s], t);   // the class's lowest trace of the block (deterministic)
        myslot = s;
    }
    __syncthreads();
    if (CHK && myslot >= 0 && lrep[myslot] == t) lchk[myslot] = h2;
    __syncthreads();
    for (int i = threadIdx.x; i < KLDS; i += KB) {
        const uint64_t h = lkey[i];
        if (!h) continue;
        uint64_t slot = h & mask;
        for (;;) {
            const uint64_t k = atomicCAS(&hk[slot], 0ull, (unsigned long long)h);
            if (k == 0 || k == h) {   // the representative: the class's lowest trace over the blocks
                atomicMin(&cr[slot].rep, lrep[i]);   // (read after this kernel; deterministic)
                if (k == 0 && CHK) chk[slot] = lchk[i];
                break;
            }
            slot = (slot + 1) & mask;
        }
        atomicAdd(&cr[slot].cnt, lcnt[i]);
        lglob[i] = (int32_t)slot;
    }
    __syncthreads();
    if (t < T) slot_of[t] = lglob[myslot];
}
template <bool CHK, int IDW>
__global__ void __launch_bounds__(KB) k_kind_insert(const int64_t* off, const int32_t* ops, const uint16_t* o16,
                                                    const float* w_t, int32_t T, unsigned long long* hk, KCnt* cr, int32_t* slot_of,
                                                    uint64_t mask, uint64_t seed, uint64_t* chk, uint64_t hmask) {
    kind_insert_body<CHK, IDW>((int32_t)blockIdx.x, off, ops, o16, w_t, T, hk, cr, slot_of, mask, seed, chk, hmask);
}

template <typename ID>   // int32 ids, or their u16 copy (rs16)
__global__ void k_kind_verify(const int64_t* off, const ID* ops, const float* w_t, int32_t T,
                              const KCnt* cr, const int32_t* slot_of, double* kind, int32_t* flag, int32_t* krep) {
    int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const KCnt ks = cr[slot_of[t]];
    const int32_t r = ks.rep;
    kind[t] = (double)ks.cnt;
    if (krep) krep[t] = r;   // (kind compression: the class representative)
    if (r == t) return;
    int64_t a0 = off[t], a1 = off[t + 1], b0 = off[r], b1 = off[r + 1];
    bool eq = (a1 - a0) == (b1 - b0);
    if (eq && a1 > a0) eq = __float_as_uint(w_t[t]) == __float_as_uint(w_t[r]);
    for (int64_t i = 0; eq && i < a1 - a0; ++i) eq = ops[a0 + i] == ops[b0 + i];
    if (!eq) atomicOr(flag, 1);
}

// Kinds by partition (graphs on one rank), no global hash table:
//   k_kind_rec     per block of KB traces: set hashes, equal keys merged in an LDS table into
//                  RECORDS (key, count, first trace) -- a hot kind (thousands of traces on one
//                  call path) leaves one record per block, so no later atomic serialises on it --
//                  and the records counted per partition (the key's top bits);
//   k_kind_rscatter a counting sort of the records into partitions of ~KP_MEAN;
//   k_kind_part    a block per partition merges its records in an LDS table (count sum, first
//                  trace min): every record then holds its class's size and representative;
//   k_kind_final   per trace: kind = its record's class size; every member is checked against
//                  the representative (ops and fp32(1/len_t), exactly): a hash collision raises
//                  flag word 0 (retry with the next seed), never a miscount.
// graphs of at least this many traces take the partition path (below: the LDS-aggregated global
// table).  1M measured ahead of 2M for C4's rank-0-of-8 share (1.25M traces: step 1.50 -> 1.44 ms,
// profiles/r05/r05r_kind_part_ab.txt); MR_KIND_PART_MIN overrides (read per call)
constexpr int64_t KIND_PART_MIN_DEFAULT = (int64_t)1 << 20;
constexpr int KP_MEAN = 1024;   // mean records per partition (at most)
constexpr int KP_LDS = 4096;    // LDS table slots of a partition block
constexpr int KP_B = 256;
__device__ __forceinline__ int32_t kind_part(uint64_t h, int pb) { return pb ? (int32_t)(h >> (64 - pb)) : 0; }
// a record: key, count, first trace -- one 16-B store / load where three arrays cost three
// scattered partial-line writes per record in k_kind_rscatter
struct __attribute__((aligned(16))) KRec {
    unsigned long long h;
    uint32_t c;
    int32_t r;
};
template <int IDW>
__global__ void __launch_bounds__(KB) k_kind_rec(const int64_t* off, const int32_t* ops, const uint16_t* o16,
                                                 const float* w_t, int32_t T, uint64_t seed, uint64_t hmask, int pb,
                                                 KRec* rec_out, int32_t* nrec, int32_t* rec_of, int32_t* hist) {
    __shared__ unsigned long long lkey[KLDS];
    __shared__ uint32_t lcnt[KLDS];
    __shared__ int32_t lrep[KLDS];
    __shared__ int32_t lidx[KLDS];
    __shared__ int32_t ln;
    __shared__ int64_t loff[IDW ? KB + 1 : 1];
    __shared__ unsigned long long lacc[IDW ? KB : 1], lacc2[1];
    for (int i = threadIdx.x; i < KLDS; i += KB) {
        lkey[i] = 0ull;
        lcnt[i] = 0u;
        lrep[i] = 0x7fffffff;
    }
    if (threadIdx.x == 0) ln = 0;
    const int32_t tb = blockIdx.x * KB, t = tb + threadIdx.x;
    uint64_t h = 0, h2 = 0;
    kind_block_hash<false, IDW>(off, ops, o16, w_t, T, tb, seed, loff, lacc, lacc2, &h, &h2);
    __syncthreads();
    int s = -1;
    if (t < T) {
        h &= hmask;   // ~0 (tests narrow it to force collisions)
        if (!h) h = 1;
        s = (int)(h & (KLDS - 1));
        for (;;) {   // <= KB distinct keys in KLDS = 2 KB slots: always a free slot
            const unsigned long long k = atomicCAS(&lkey[s], 0ull, (unsigned long long)h);
            if (k == 0ull || k == h) break;
            s = (s + 1) & (KLDS - 1);
        }
        atomicAdd(&lcnt[s], 1u);
        atomicMin(&lrep[s], t);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < KLDS; i += KB) {
        const uint64_t k = lkey[i];
        if (!k) continue;
        const int32_t r = atomicAdd(&ln, 1);   // record order within the block: free (sums / mins)
        lidx[i] = r;
        KRec v;
        v.h = k;
        v.c = lcnt[i];
        v.r = lrep[i];
        rec_out[(int64_t)tb + r] = v;
        if (hist) atomicAdd(&hist[kind_part(k, pb)], 1);   // (the cursor scatter's counts)
    }
    __syncthreads();
    if (t < T) rec_of[t] = tb + lidx[s];
    if (threadIdx.x == 0) nrec[blockIdx.x] = ln;
}
__global__ void k_kind_rscatter(const KRec* rin, const int32_t* nrec, int32_t T, int pb, unsigned long long* cur,
                                KRec* e, int32_t* rpos) {
    const int32_t rec = blockIdx.x * blockDim.x + threadIdx.x;
    if (rec >= T || (rec % KB) >= nrec[rec / KB]) return;
    const KRec v = rin[rec];
    const int32_t pos = (int32_t)atomicAdd(&cur[kind_part(v.h, pb)], 1ull);
    e[pos] = v;
    rpos[rec] = pos;
}
// The records grouped by partition in two passes over the partition's bits, with no device atomic
// per record (the cursor scatter above takes two: its counts and its cursor, 7.4 ms of C5's
// 100M records):
//   k_kp1_count   tiles of KT slots: per tile a histogram of the partition's top b1 bits (the
//                 coarse bucket), written bucket-major (cnt[b * ntile + tile]), so ONE exclusive
//                 scan of it gives every (bucket, tile)'s first position;
//   k_kp1_scatter the tile's records to their buckets through LDS cursors, each with its slot;
//   k_kp2         a block per bucket: counts its fine partitions (the next pb - b1 bits) in LDS,
//                 writes their starts, and scatters the bucket's records into partition order
//                 inside the bucket's range, each beside its block-order slot (eslot).
// The order inside a partition depends on LDS atomics; k_kind_part's merge (sums, minimum) does
// not: the same classes and representatives.
constexpr int KP1_B = 8;    // coarse bits (1024 buckets over tiles of 16384 measured slower at C4: 584 vs 553 us)
constexpr int KT = 4096;    // slots per level-1 tile
constexpr int KT_T = 256;   // threads of a level-1 block
constexpr int KP2_T = 1024;
__device__ __forceinline__ int32_t kbits(uint64_t h, int n) { return n ? (int32_t)(h >> (64 - n)) : 0; }
// (the three loops take KP_BATCH records per thread per round: loads first, then the LDS atomics
// and stores -- one round's loads in flight together instead of one dependent chain per record)
constexpr int KP_BATCH = 4;
__global__ void __launch_bounds__(KT_T) k_kp1_count(const KRec* __restrict__ rec, const int32_t* __restrict__ nrec,
                                                    int64_t R, int b1, int32_t ntile, int32_t* __restrict__ cnt) {
    __shared__ int32_t hb[1 << KP1_B];
    const int nbk = 1 << b1;
    for (int i = threadIdx.x; i < nbk; i += KT_T) hb[i] = 0;
    __syncthreads();
    const int64_t s0 = (int64_t)blockIdx.x * KT;
    for (int k0 = 0; k0 < KT / KT_T; k0 += KP_BATCH) {
        int bk[KP_BATCH];
#pragma unroll
        for (int j = 0; j < KP_BATCH; ++j) {
            const int64_t sl = s0 + (k0 + j) * KT_T + threadIdx.x;
            bk[j] = sl < R && (int32_t)(sl % KB) < nrec[sl / KB] ? kbits(rec[sl].h, b1) : -1;
        }
#pragma unroll
        for (int j = 0; j < KP_BATCH; ++j)
            if (bk[j] >= 0) atomicAdd(&hb[bk[j]], 1);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nbk; i += KT_T) cnt[(int64_t)i * ntile + blockIdx.x] = hb[i];
}
__global__ void __launch_bounds__(KT_T) k_kp1_scatter(const KRec* __restrict__ rec, const int32_t* __restrict__ nrec,
                                                      int64_t R, int b1, int32_t ntile, const int64_t* __restrict__ off,
                                                      KRec* __restrict__ out, uint32_t* __restrict__ oslot) {
    __shared__ int64_t base[1 << KP1_B];   // the (bucket, tile)'s first position, and 32-bit cursors after it
    __shared__ uint32_t cur[1 << KP1_B];
    const int nbk = 1 << b1;
    for (int i = threadIdx.x; i < nbk; i += KT_T) {
        base[i] = off[(int64_t)i * ntile + blockIdx.x];
        cur[i] = 0u;
    }
    __syncthreads();
    const int64_t s0 = (int64_t)blockIdx.x * KT;
    for (int k0 = 0; k0 < KT / KT_T; k0 += KP_BATCH) {
        KRec v[KP_BATCH];
        bool ok[KP_BATCH];
#pragma unroll
        for (int j = 0; j < KP_BATCH; ++j) {
            const int64_t sl = s0 + (k0 + j) * KT_T + threadIdx.x;
            ok[j] = sl < R && (int32_t)(sl % KB) < nrec[sl / KB];
            if (ok[j]) v[j] = rec[sl];
        }
#pragma unroll
        for (int j = 0; j < KP_BATCH; ++j) {
            if (!ok[j]) continue;
            const int b = kbits(v[j].h, b1);
            const int64_t pos = base[b] + (int64_t)atomicAdd(&cur[b], 1u);
            out[pos] = v[j];
            oslot[pos] = (uint32_t)(s0 + (k0 + j) * KT_T + threadIdx.x);
        }
    }
}
__global__ void __launch_bounds__(KP2_T) k_kp2(const KRec* __restrict__ in, const uint32_t* __restrict__ islot,
                                               const int64_t* __restrict__ off, int pb, int b1, int32_t ntile,
                                               KRec* __restrict__ out, uint32_t* __restrict__ eslot,
                                               int64_t* __restrict__ pstart) {
    extern __shared__ int64_t kp2[];   // [KP2_T] scan partials, then [nf] 32-bit counts / cursors (from B0)
    const int nf = 1 << (pb - b1), b = (int)blockIdx.x, tid = (int)threadIdx.x;
    const int64_t B0 = off[(int64_t)b * ntile], B1 = off[(int64_t)(b + 1) * ntile];
    int64_t* part = kp2;
    uint32_t* cur = (uint32_t*)(kp2 + KP2_T);
    for (int f = tid; f < nf; f += KP2_T) cur[f] = 0u;
    __syncthreads();
    const uint64_t fm = (uint64_t)nf - 1;
    for (int64_t i0 = B0 + tid; i0 < B1; i0 += (int64_t)KP2_T * KP_BATCH) {
        int fk[KP_BATCH];
#pragma unroll
        for (int j = 0; j < KP_BATCH; ++j) {
            const int64_t i = i0 + (int64_t)j * KP2_T;
            fk[j] = i < B1 ? (int)((uint64_t)kbits(in[i].h, pb) & fm) : -1;
        }
#pragma unroll
        for (int j = 0; j < KP_BATCH; ++j)
            if (fk[j] >= 0) atomicAdd(&cur[fk[j]], 1u);
    }
    __syncthreads();
    // exclusive scan of the nf counts: a run of consecutive counts per thread, then its partials
    const int per = (nf + KP2_T - 1) / KP2_T, f0 = tid * per, f1 = min(f0 + per, nf);
    int64_t a = 0;
    for (int f = f0; f < f1; ++f) a += cur[f];
    part[tid] = a;
    __syncthreads();
    for (int o = 1; o < KP2_T; o <<= 1) {
        const int64_t x = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += x;
        __syncthreads();
    }
    int64_t run = part[tid] - a;   // (relative to B0)
    for (int f = f0; f < f1; ++f) {
        const uint32_t c = cur[f];
        cur[f] = (uint32_t)run;
        pstart[(int64_t)b * nf + f] = B0 + run;
        run += c;
    }
    if (b == (int)gridDim.x - 1 && tid == 0) pstart[(int64_t)gridDim.x * nf] = B1;
    __syncthreads();
    for (int64_t i0 = B0 + tid; i0 < B1; i0 += (int64_t)KP2_T * KP_BATCH) {
        KRec v[KP_BATCH];
        uint32_t sl[KP_BATCH];
#pragma unroll
        for (int j = 0; j < KP_BATCH; ++j) {
            const int64_t i = i0 + (int64_t)j * KP2_T;
            if (i < B1) {
                v[j] = in[i];
                sl[j] = islot[i];
            }
        }
#pragma unroll
        for (int j = 0; j < KP_BATCH; ++j) {
            if (i0 + (int64_t)j * KP2_T >= B1) continue;
            const int64_t pos = B0 + (int64_t)atomicAdd(&cur[(uint64_t)kbits(v[j].h, pb) & fm], 1u);
            out[pos] = v[j];
            eslot[pos] = sl[j];   // (beside the record, in partition order: k_kind_part writes back through it)
        }
    }
}
// eslot (two-pass grouping): each record's slot in the block-order records `back`, where the class
// (count, first trace) is written -- k_kind_final then reads it at rec_of[t] (a block's own range)
// instead of through a per-record position (a random read per trace); null: into e itself
__global__ void __launch_bounds__(KP_B) k_kind_part(const int64_t* pstart, KRec* e, int32_t* flag,
                                                    const uint32_t* eslot, KRec* back) {
    __shared__ unsigned long long tkey[KP_LDS];
    __shared__ uint32_t tcnt[KP_LDS];
    __shared__ int32_t trep[KP_LDS];
    const int64_t b = pstart[blockIdx.x], en = pstart[blockIdx.x + 1];
    for (int i = threadIdx.x; i < KP_LDS; i += KP_B) {
        tkey[i] = 0ull;
        tcnt[i] = 0u;
        trep[i] = 0x7fffffff;
    }
    __syncthreads();
    // (KP_BATCH records per thread per round: their loads go out together)
    for (int64_t i0 = b + threadIdx.x; i0 < en; i0 += (int64_t)KP_B * KP_BATCH) {
        KRec vv[KP_BATCH];
#pragma unroll
        for (int j = 0; j < KP_BATCH; ++j)
            if (i0 + (int64_t)j * KP_B < en) vv[j] = e[i0 + (int64_t)j * KP_B];
#pragma unroll
        for (int j = 0; j < KP_BATCH; ++j) {
            if (i0 + (int64_t)j * KP_B >= en) continue;
            const KRec& v = vv[j];
            const uint64_t h = v.h;
            int s = (int)(h & (KP_LDS - 1));
            for (int probe = 0;; ++probe) {
                if (probe == KP_LDS) {   // more distinct keys than slots: not with hashed partitions
                    atomicOr(flag + 2, 1);
                    break;
                }
                const unsigned long long k = atomicCAS(&tkey[s], 0ull, (unsigned long long)h);
                if (k == 0ull || k == h) {
                    atomicAdd(&tcnt[s], v.c);
                    atomicMin(&trep[s], v.r);   // the class's first trace (deterministic)
                    break;
                }
                s = (s + 1) & (KP_LDS - 1);
            }
        }
    }
    __syncthreads();
    for (int64_t i0 = b + threadIdx.x; i0 < en; i0 += (int64_t)KP_B * KP_BATCH) {
        uint64_t hh[KP_BATCH];
#pragma unroll
        for (int j = 0; j < KP_BATCH; ++j) hh[j] = i0 + (int64_t)j * KP_B < en ? e[i0 + (int64_t)j * KP_B].h : 0ull;
#pragma unroll
        for (int j = 0; j < KP_BATCH; ++j) {
            const int64_t i = i0 + (int64_t)j * KP_B;
            if (i >= en) continue;
            const uint64_t h = hh[j];
            int s = (int)(h & (KP_LDS - 1));
            for (int probe = 0; probe < KP_LDS && tkey[s] != h; ++probe) s = (s + 1) & (KP_LDS - 1);
            if (tkey[s] != h) continue;   // (overflowed: flagged above)
            *(uint2*)&(eslot ? back[eslot[i]] : e[i]).c = make_uint2(tcnt[s], (uint32_t)trep[s]);   // (c, r): one 8-B store
        }
    }
}
template <typename ID>
__global__ void k_kind_final(const int32_t* rec_of, const int32_t* rpos, const KRec* e, const int64_t* off,
                             const ID* ops, const float* w_t, int32_t T, double* kind, int32_t* flag, int32_t* krep) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const int32_t pos = rpos ? rpos[rec_of[t]] : rec_of[t];   // (null: e holds the classes in slot order)
    const uint2 cr = *(const uint2*)&e[pos].c;
    kind[t] = (double)cr.x;
    const int32_t r = (int32_t)cr.y;
    if (krep) krep[t] = r;   // (kind compression: the class representative)
    if (r == t) return;
    // exact membership: same ids and the same fp32(1/len_t) as the representative
    const int64_t a0 = off[t], a1 = off[t + 1], b0 = off[r], b1 = off[r + 1];
    bool eq = (a1 - a0) == (b1 - b0);
    if (eq && a1 > a0) eq = __float_as_uint(w_t[t]) == __float_as_uint(w_t[r]);
    for (int64_t j = 0; eq && j < a1 - a0; ++j) eq = ops[a0 + j] == ops[b0 + j];
    if (!eq) atomicOr(flag, 1);
}

// ---------------------------------------------------------------- kind compression (§8(f) f4)
// Traces of one kind have identical r (same op set and len_t, hence the same v_t): the iteration
// runs over one representative per kind whose q carries the kind's multiplicity.
__global__ void k_kc_flags(const int32_t* krep, int32_t T, int32_t* flag) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < T) flag[t] = krep[t] == t ? 1 : 0;
}
__global__ void k_kc_reps(const int32_t* flag, const int64_t* pos, int32_t T, const int64_t* off, const int32_t* len_t,
                          const double* kind, int32_t* rep, int32_t* len_c, double* mult, int32_t* cnt) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T || !flag[t]) return;
    const int64_t k = pos[t];
    rep[k] = t;
    len_c[k] = len_t[t];
    mult[k] = kind[t];
    cnt[k] = (int32_t)(off[t + 1] - off[t]);
}
__global__ void k_kc_ops(const int32_t* rep, const int64_t* off_c, int32_t K, const int64_t* off, const int32_t* ops,
                         int32_t* ops_c) {
    const int32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= K) return;
    const int32_t t = rep[k];
    const int64_t a = off[t], n = off[t + 1] - a, b = off_c[k];
    for (int64_t j = 0; j < n; ++j) ops_c[b + j] = ops[a + j];
}
__global__ void k_kc_mw(const int32_t* tperm, const float* w_tp, const double* mult, int32_t T, double* mw_tp) {
    const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < T) mw_tp[p] = (double)w_tp[p] * mult[tperm[p]];   // exact: a 24-bit mantissa times an integer < 2^29
}
__global__ void k_kc_tile_mult(const int32_t* tperm, const double* mult, int32_t T, int32_t n_wt, int64_t* out) {
    const int32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_wt) return;
    int64_t m = 0;
    for (int32_t p = k * WAVE; p < min(k * WAVE + WAVE, T); ++p) m += (int64_t)mult[tperm[p]];
    out[k] = m;
}

// ---------------------------------------------------------------- preference (pagerank.py:68-85)
// sums over pr_trace entries: [0] sum 1/k, [1] sum 1/len; block partials then one fixed-order pass
// mult (kind-compressed graphs): trace i stands for mult[i] traces of its kind
__global__ void k_pref_partial(const double* kind, const int32_t* pr_trace, const int32_t* pr_len,
                               const int32_t* len_t, int32_t n_pr, const double* mult, double* part, int32_t* flag) {
    __shared__ double red[TB / WAVE];
    double a = 0.0, b = 0.0;
    int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_pr) {
        int32_t t = pr_trace ? pr_trace[i] : i;
        int32_t ln = pr_len ? pr_len[i] : len_t[t];
        a = 1.0 / kind[t];
        if (ln == 0) atomicOr(flag + 1, 1);   // 1.0/len(pr_trace[t]) -> ZeroDivisionError (word 1)
        b = ln ? 1.0 / (double)ln : 0.0;
        if (mult) {
            a *= mult[t];
            b *= mult[t];
        }
    }
    a = block_sum(a, red);
    b = block_sum(b, red);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = a;
        part[2 * blockIdx.x + 1] = b;
    }
}

// (a last-block total inside k_pref_partial was measured slower: the per-block release fence
// writes back the XCD's L2, 21 us against 6.7 + 5.6 us for the two launches)
__global__ void k_pref_total(const double* part, int32_t nb, double* scal) {
    __shared__ double red[1024 / WAVE];
    double a = 0.0, b = 0.0;
    for (int32_t i = threadIdx.x; i < nb; i += blockDim.x) {
        a += part[2 * i];
        b += part[2 * i + 1];
    }
    a = block_sum(a, red);
    b = block_sum(b, red);
    if (threadIdx.x == 0) {
        scal[2] = a;
        scal[3] = b;
    }
}

// reference order, one thread (MR_PR_EXACT_SUMS, T7)
__global__ void k_pref_total_exact(const double* kind, const int32_t* pr_trace, const int32_t* pr_len,
                                   const int32_t* len_t, int32_t n_pr, double* scal) {
    if (threadIdx.x || blockIdx.x) return;
    double a = 0.0, b = 0.0;
    for (int32_t i = 0; i < n_pr; ++i) {
        int32_t t = pr_trace ? pr_trace[i] : i;
        int32_t ln = pr_len ? pr_len[i] : len_t[t];
        a += 1.0 / kind[t];
        b += ln ? 1.0 / (double)ln : 0.0;
    }
    scal[2] = a;
    scal[3] = b;
}

// tperm (k_tr_a graphs with pr_trace = operation_trace): thread i is position i, and c_t goes to
// c_tp[i] too (formerly k_tr_gather)
__global__ void k_pref_apply(const double* kind, const int32_t* pr_trace, const int32_t* pr_len,
                             const int32_t* len_t, int32_t n_pr, const double* scal, int anomaly,
                             float cd, double phi, float* pref, float* c_t, const int32_t* tperm, float* c_tp) {
    int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pr) return;
    int32_t t = tperm ? tperm[i] : pr_trace ? pr_trace[i] : i;
    int32_t ln = pr_len ? pr_len[i] : len_t[t];
    double k = kind[t];
    double v;
    if (!anomaly) {
        v = 1.0 / k / scal[2];                                               // :74
    } else {
        v = 1.0 / (k / scal[2] * phi + 1.0 / (double)ln) / scal[3] * phi;   // :80-85 (phi = 0.5)
    }
    float vf = (float)v;
    pref[t] = vf;
    c_t[t] = cd * vf;   // (1.0 - d) * v: float32 array times a Python float stays float32 (T4)
    if (tperm) c_tp[i] = cd * vf;
}

// Large k_tr_a graphs (pr_trace = operation_trace): the same values in TRACE order -- kind[t],
// len_t[t] read and pref[t] written coalesced, only c_tp scattered (through tpos, the inverse of
// tperm).  The position-order form above gathers kind / len_t and scatters pref / c_t at random
// t: four random streams per trace, 11 ms at C5's 100M traces.  c_t itself
// is not written: the fused iteration reads only c_tp.
__global__ void k_pref_apply_t(const double* __restrict__ kind, const int32_t* __restrict__ len_t, int32_t T,
                               const double* __restrict__ scal, int anomaly, float cd, double phi, float* __restrict__ pref,
                               const int32_t* __restrict__ tpos, float* __restrict__ c_tp) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const double k = kind[t];
    const double v = !anomaly ? 1.0 / k / scal[2]                                               // :74
                              : 1.0 / (k / scal[2] * phi + 1.0 / (double)len_t[t]) / scal[3] * phi;   // :80-85
    const float vf = (float)v;
    pref[t] = vf;
    c_tp[tpos[t]] = cd * vf;   // (1.0 - d) * v in float32 (T4)
}
__global__ void k_inv_perm(const int32_t* __restrict__ perm, int32_t n, int32_t* __restrict__ inv) {
    const int32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < n) inv[perm[p]] = p;
}

// ---------------------------------------------------------------- iteration
// M_s / M_r per iteration live in MSH shards (an atomicMax per block or op on ONE word would
// serialise ~2k same-address atomics per iteration); readers reduce the shards.
constexpr int MSH = 64;
// mslot: [3 iterations][s | r][MSH] maxima, then words of the hand-offs (6 MSH + 1: the last-block ticket)
constexpr int MSLOT_WORDS = 6 * MSH + 8;
__device__ __forceinline__ double bits2d(unsigned long long b) { return __longlong_as_double((long long)b); }
__device__ __forceinline__ unsigned long long d2bits(double v) {
    return (unsigned long long)__double_as_longlong(v);
}

constexpr int TR_PAD = WAVE;   // k_tr_a's pad ids N .. N + 63 (su = 0)
__device__ __forceinline__ int32_t cdiv_d(int32_t a, int32_t b) { return (a + b - 1) / b; }
// ---------------------------------------------------------------- batched set-up
// The set-up of many window graphs (reset + iteration state, kinds, preference) as ONE launch per
// step for all of them (a block range per graph, as the iteration's launches are), instead of six
// launches per graph from the windows' host threads.  Same bodies, same results.
struct SDev {
    int32_t T, N, anomaly, fp32;
    int64_t cap, T_all;
    float cd;
    double phi;                                 // the anomaly preference's 0.5 (pagerank.py:82-84)
    int32_t b_reset, b_kins, b_kver, b_pref;   // the graph's first block in each launch
    float *pref, *c_t, *c_tp;
    const int32_t *tperm, *tpos;
    unsigned long long* hk;
    KCnt* cr;
    int32_t *slot_of, *flag;
    double *kind, *scal, *ppart;
    const float *w_t, *w_tq, *u_o;              // w_t by trace; in q's order (position order for k_tr_a graphs)
    double *sp0, *su0, *su1, *q64;
    float* q32;
    unsigned long long* mslot;
    const int32_t* perm;
    const int64_t* off;
    const uint16_t* o16;
    const int32_t* len_t;
};
__device__ __forceinline__ int32_t sd_graph(const SDev* sd, int32_t ng, int32_t blk, int which) {
    int32_t lo = 0, hi = ng - 1;
    while (lo < hi) {
        const int32_t mid = (lo + hi + 1) >> 1;
        const SDev& g = sd[mid];
        const int32_t s0 = which == 0 ? g.b_reset : which == 1 ? g.b_kins : which == 2 ? g.b_kver : g.b_pref;
        if (s0 <= blk) lo = mid; else hi = mid - 1;
    }
    return lo;
}
__global__ void k_reset_init_b(const SDev* __restrict__ sd, int32_t ng) {
    const SDev& G = sd[sd_graph(sd, ng, (int32_t)blockIdx.x, 0)];
    const int64_t i = (int64_t)((int32_t)blockIdx.x - G.b_reset) * blockDim.x + threadIdx.x;
    const int32_t T = G.T, N = G.N;
    if (i < T) {
        G.pref[i] = 0.0f;
        G.c_t[i] = 0.0f;
    }
    if (i < G.cap) {
        G.hk[i] = 0ull;
        G.cr[i] = KCnt{0u, 0x7fffffff};
    }
    if (i < 8) G.flag[i] = 0;
    if (i < 8) G.scal[i] = 0.0;
    const double v0 = 1.0 / (double)((int64_t)N + G.T_all);      // pagerank.py:118-119
    if (i < N) {
        G.sp0[i] = v0;
        G.su0[i] = (double)G.u_o[G.perm ? G.perm[i] : i] * v0;
    }
    if (i >= N && i < N + TR_PAD) G.su0[i] = G.su1[i] = 0.0;
    if (i < T) {
        const double q = (double)G.w_tq[i] * v0;
        if (G.fp32) G.q32[i] = (float)q; else G.q64[i] = q;
    }
    if (i < MSLOT_WORDS) G.mslot[i] = i < 2 * MSH ? d2bits(1.0) : 0ull;
}
__global__ void __launch_bounds__(KB) k_kind_insert_b(const SDev* __restrict__ sd, int32_t ng, uint64_t seed,
                                                      uint64_t hmask) {
    const SDev& G = sd[sd_graph(sd, ng, (int32_t)blockIdx.x, 1)];
    kind_insert_body<false, 2>((int32_t)blockIdx.x - G.b_kins, G.off, nullptr, G.o16, G.w_t, G.T, G.hk, G.cr,
                                  G.slot_of, (uint64_t)(G.cap - 1), seed, nullptr, hmask);
}
__global__ void k_kind_verify_b(const SDev* __restrict__ sd, int32_t ng) {
    const SDev& G = sd[sd_graph(sd, ng, (int32_t)blockIdx.x, 2)];
    const int32_t t = ((int32_t)blockIdx.x - G.b_kver) * blockDim.x + threadIdx.x;
    if (t >= G.T) return;
    const KCnt ks = G.cr[G.slot_of[t]];
    const int32_t r = ks.rep;
    G.kind[t] = (double)ks.cnt;
    if (r == t) return;
    const int64_t a0 = G.off[t], a1 = G.off[t + 1], b0 = G.off[r], b1 = G.off[r + 1];
    bool eq = (a1 - a0) == (b1 - b0);
    if (eq && a1 > a0) eq = __float_as_uint(G.w_t[t]) == __float_as_uint(G.w_t[r]);
    for (int64_t i = 0; eq && i < a1 - a0; ++i) eq = G.o16[a0 + i] == G.o16[b0 + i];
    if (!eq) atomicOr(G.flag, 1);
}
__global__ void k_pref_partial_b(const SDev* __restrict__ sd, int32_t ng) {
    __shared__ double red[TB / WAVE];
    const SDev& G = sd[sd_graph(sd, ng, (int32_t)blockIdx.x, 3)];
    const int32_t blk = (int32_t)blockIdx.x - G.b_pref;
    double a = 0.0, b = 0.0;
    const int32_t i = blk * blockDim.x + threadIdx.x;
    if (i < G.T) {
        const int32_t ln = G.len_t[i];
        a = 1.0 / G.kind[i];
        if (ln == 0) atomicOr(G.flag + 1, 1);
        b = ln ? 1.0 / (double)ln : 0.0;
    }
    a = block_sum(a, red);
    b = block_sum(b, red);
    if (threadIdx.x == 0) {
        G.ppart[2 * blk] = a;
        G.ppart[2 * blk + 1] = b;
    }
}
__global__ void k_pref_total_b(const SDev* __restrict__ sd) {   // block g: graph g
    __shared__ double red[1024 / WAVE];
    const SDev& G = sd[blockIdx.x];
    const int32_t nb = cdiv_d(G.T, TB);
    double a = 0.0, b = 0.0;
    for (int32_t i = threadIdx.x; i < nb; i += blockDim.x) {
        a += G.ppart[2 * i];
        b += G.ppart[2 * i + 1];
    }
    a = block_sum(a, red);
    b = block_sum(b, red);
    if (threadIdx.x == 0) {
        G.scal[2] = a;
        G.scal[3] = b;
    }
}
// in trace order (as k_pref_apply_t): the per-trace reads and writes are coalesced, the one
// scattered store is c_tp at the trace's position (tpos, the inverse of tperm)
__global__ void k_pref_apply_b(const SDev* __restrict__ sd, int32_t ng) {
    const SDev& G = sd[sd_graph(sd, ng, (int32_t)blockIdx.x, 3)];
    const int32_t t = ((int32_t)blockIdx.x - G.b_pref) * blockDim.x + threadIdx.x;
    if (t >= G.T) return;
    const int32_t i = G.tpos[t];
    const double k = G.kind[t];
    double v;
    if (!G.anomaly) v = 1.0 / k / G.scal[2];                                               // :74
    else v = 1.0 / (k / G.scal[2] * G.phi + 1.0 / (double)G.len_t[t]) / G.scal[3] * G.phi;   // :80-85
    const float vf = (float)v;
    G.pref[t] = vf;
    G.c_t[t] = G.cd * vf;   // (1.0 - d) * v in float32 (T4)
    G.c_tp[i] = G.cd * vf;
}

// ---------------------------------------------------------------- window graphs in layout order
// (mr_lo_prepare_batch) A graph whose positions come from its table's layout order (pinv[p] =
// the layout index of position p): chunk offsets, the lane-interleaved ids (the table's u16 codes
// relabelled to node ids: node_of_code), w_t / span count / kind class size by position and the
// preference partials, then the totals, then the preference and iteration state -- the work of
// k_graph_consts .. k_tr_fill and k_reset_init .. k_pref_apply for these graphs, in four launches.
constexpr int LO_NOC_MAX = 4096;   // (mr_lo_fits: tables of <= NS_PMAX pod-ops)
struct LDev {
    int32_t T, N, W, anomaly, fp32, NP;
    int32_t b_cs, n_cs, b_fill, nbp, b_app;   // first block in each launch; partial blocks
    int64_t st_off;
    float cd;
    double phi, v0;
    const int32_t* pinv;
    const int64_t* lo_off;
    const uint16_t* lo16;
    const int32_t *lo_len, *lo_kid, *noc;
    const uint32_t* kcnt;
    int64_t* c64;
    int32_t* coff;
    uint16_t* tids;
    float *w_tp, *c_tp;
    double* kind;
    int32_t* lenp;
    uint8_t* trun;
    double *ppart, *scal;
    int32_t* flag;
    unsigned long long* mslot;
    double *sp0, *su0, *su1, *q64;
    float* q32;
    const float* u_o;
};
__device__ __forceinline__ int32_t ld_graph(const LDev* ld, int32_t n, int32_t blk, int which) {
    int32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const int32_t mid = (lo + hi + 1) >> 1;
        const LDev& g = ld[mid];
        const int32_t s0 = which == 0 ? g.b_cs : which == 1 ? g.b_fill : g.b_app;
        if (s0 <= blk) lo = mid; else hi = mid - 1;
    }
    return lo;
}
__global__ void __launch_bounds__(TS_T) k_lo_cs_b(const LDev* __restrict__ ld, int32_t n, unsigned long long* st,
                                                 uint64_t epoch) {
    const LDev& G = ld[ld_graph(ld, n, (int32_t)blockIdx.x, 0)];
    tr_chunk_scan_body((int32_t)blockIdx.x - G.b_cs, G.n_cs, G.pinv, G.lo_off, G.T, G.W, G.c64, G.coff, st + G.st_off,
                       epoch);
}
// thread per (tile, lane) = position: as tr_fill_body (the trace rotated by its index mod len, pads
// N + lane), ids relabelled; w_t = fp32(1/len_t), the span count and the class size by position;
// the block's 1/k and 1/len_t sums (pagerank.py:71-78) into ppart
__global__ void __launch_bounds__(256) k_lo_fill_b(const LDev* __restrict__ ld, int32_t n) {
    __shared__ double red[256 / WAVE];
    __shared__ uint16_t lnoc[LO_NOC_MAX];   // the code -> node id table (one LDS read per id)
    const LDev& G = ld[ld_graph(ld, n, (int32_t)blockIdx.x, 1)];
    const int32_t blk = (int32_t)blockIdx.x - G.b_fill;
    const int64_t i = (int64_t)blk * 256 + threadIdx.x;
    const int32_t T = G.T, N = G.N;
    for (int32_t c = threadIdx.x; c < G.NP; c += 256) lnoc[c] = (uint16_t)G.noc[c];
    __syncthreads();
    double a = 0.0, b = 0.0;
    if (i < (int64_t)G.W * WAVE) {   // (uniform per wave: a wave is one tile)
        const int32_t k = (int32_t)(i / WAVE), lane = (int32_t)(i % WAVE);
        int64_t e0 = 0, len = 0, rot = 0;
        // every trace rotated by its own layout index mod length.  Run-merged graphs (MR_TR_MERGE=1,
        // trun set; kind compression inside the walk, SURVEY 8(f)4 -- never the headline): runs of
        // identical traces (adjacent positions of one kind class: the layout keeps a class
        // contiguous) share their head's rotation instead, so its members walk the same ids in the
        // same order and k_tr_a lets the head walk for the run
        const int32_t ix = i < T ? G.pinv[i] : -1;
        const int32_t kid = i < T ? G.lo_kid[ix] : -1;
        const int32_t kp = __shfl_up(kid, 1, WAVE);
        const bool hd = lane == 0 || kid < 0 || kid != kp;
        const unsigned long long hm = __ballot(hd);
        const unsigned long long below = hm & (lane == WAVE - 1 ? ~0ull : (2ull << lane) - 1ull);
        const int32_t ixh = __shfl(ix, 63 - __builtin_clzll(below), WAVE);
        // only a tile of the 512-thread walk's short tiers merges (the general loop walks every
        // lane): there its runs share the head's rotation and are marked; a longer tile keeps one
        // rotation per trace (a shared rotation there would put a run's adds on one word at a time)
        const bool mt = G.trun && G.c64[k + 1] - G.c64[k] <= MR_TR_TIERS512;
        if (i < T && G.trun) {
            const unsigned long long above = lane == WAVE - 1 ? 0ull : hm & (~0ull << (lane + 1));
            G.trun[i] = !mt ? (uint8_t)1 : hd ? (uint8_t)((above ? __builtin_ctzll(above) : WAVE) - lane) : (uint8_t)0;
        }
        if (i < T) {
            e0 = G.lo_off[ix];
            len = G.lo_off[ix + 1] - e0;
            rot = len ? (int64_t)((uint32_t)(mt ? ixh : ix) % (uint32_t)len) : 0;
            const int32_t L = G.lo_len[ix];
            const uint32_t kc = G.kcnt[G.lo_kid[ix]];
            G.w_tp[i] = L > 0 ? (float)(1.0 / (double)L) : 0.0f;
            G.lenp[i] = L;
            G.kind[i] = (double)kc;
            a = 1.0 / (double)kc;
            b = L ? 1.0 / (double)L : 0.0;
        }
        const int64_t nc = G.c64[k + 1] - G.c64[k];
        unsigned long long* dst = (unsigned long long*)G.tids + (size_t)G.c64[k] * WAVE + lane;
        constexpr int TF_CH = 4;
        for (int64_t c0 = 0; c0 < nc; c0 += TF_CH) {
            uint16_t idv[4 * TF_CH];
#pragma unroll
            for (int q = 0; q < 4 * TF_CH; ++q) {
                const int64_t e = 4 * c0 + q, jx = rot + e;
                idv[q] = e < len ? lnoc[G.lo16[e0 + (jx >= len ? jx - len : jx)]] : (uint16_t)(N + lane);
            }
#pragma unroll
            for (int u = 0; u < TF_CH; ++u)
                if (c0 + u < nc)
                    dst[(size_t)(c0 + u) * WAVE] = (unsigned long long)idv[4 * u] | (unsigned long long)idv[4 * u + 1] << 16 |
                                                   (unsigned long long)idv[4 * u + 2] << 32 |
                                                   (unsigned long long)idv[4 * u + 3] << 48;
        }
    }
    a = block_sum(a, red);
    b = block_sum(b, red);
    if (threadIdx.x == 0) {
        G.ppart[2 * blk] = a;
        G.ppart[2 * blk + 1] = b;
    }
}
__global__ void __launch_bounds__(1024) k_lo_total_b(const LDev* __restrict__ ld) {   // block g: graph g
    __shared__ double red[1024 / WAVE];
    const LDev& G = ld[blockIdx.x];
    double a = 0.0, b = 0.0;
    for (int32_t i = threadIdx.x; i < G.nbp; i += blockDim.x) {
        a += G.ppart[2 * i];
        b += G.ppart[2 * i + 1];
    }
    a = block_sum(a, red);
    b = block_sum(b, red);
    if (threadIdx.x == 0) {
        G.scal[2] = a;
        G.scal[3] = b;
    }
}
// the preference (pagerank.py:68-85, T4) and the iteration state (k_reset_init_b's) by position
__global__ void k_lo_apply_b(const LDev* __restrict__ ld, int32_t n) {
    const LDev& G = ld[ld_graph(ld, n, (int32_t)blockIdx.x, 2)];
    const int64_t i = (int64_t)((int32_t)blockIdx.x - G.b_app) * blockDim.x + threadIdx.x;
    const int32_t T = G.T, N = G.N;
    const double v0 = G.v0;
    if (i < T) {
        const double k = G.kind[i];
        double v;
        if (!G.anomaly) v = 1.0 / k / G.scal[2];                                                    // :74
        else v = 1.0 / (k / G.scal[2] * G.phi + 1.0 / (double)G.lenp[i]) / G.scal[3] * G.phi;   // :80-85
        const float vf = (float)v;
        G.c_tp[i] = G.cd * vf;   // (1.0 - d) * v in float32 (T4)
        const double q = (double)G.w_tp[i] * v0;
        if (G.fp32) G.q32[i] = (float)q; else G.q64[i] = q;
    }
    if (i < N) {
        G.sp0[i] = v0;
        G.su0[i] = (double)G.u_o[i] * v0;
    }
    if (i >= N && i < N + TR_PAD) G.su0[i] = G.su1[i] = 0.0;
    if (i < MSLOT_WORDS) G.mslot[i] = i < 2 * MSH ? d2bits(1.0) : 0ull;
    if (i < 4) G.flag[i] = 0;
    if (i < 8 && i != 2 && i != 3) G.scal[i] = 0.0;
}

// T_all: traces of the whole graph (all shards) for the initial value
// perm (relabelled fused graphs): su is kept in the kernel's op labels, su[new] = u_o[perm[new]] s
// w_t: in position order for k_tr_a (w_tp: q is then indexed by position), else by trace
__global__ void k_iter_init(const float* w_t, const double* mw, const float* u_o, int32_t N, int32_t T, int64_t T_all,
                            double* sp0, double* su0, double* su1, double* q64, float* q32, int fp32,
                            unsigned long long* mslot, const int32_t* perm) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const double v0 = 1.0 / (double)((int64_t)N + T_all);      // pagerank.py:118-119
    if (i < N) {
        sp0[i] = v0;
        su0[i] = (double)u_o[perm ? perm[i] : i] * v0;
    }
    if (i >= N && i < N + TR_PAD) su0[i] = su1[i] = 0.0;   // the fused walks' pad slots
    if (i < T) {
        double q = (mw ? mw[i] : (double)w_t[i]) * v0;   // mw: w_t times the kind's multiplicity
        if (fp32) q32[i] = (float)q; else q64[i] = q;
    }
    // M_s(0) = M_r(0) = 1: s_0, r_0 are used as they are; slots 1, 2 start cleared
    if (i < MSLOT_WORDS) mslot[i] = i < 2 * MSH ? d2bits(1.0) : 0ull;
}
// k_pr_reset and k_iter_init in one launch (the iteration state depends on nothing the kinds or
// the preference compute)
__global__ void k_pr_reset_init(int32_t T, int64_t cap, int32_t N, float* pref, float* c_t, unsigned long long* hk,
                                KCnt* cr, int32_t* flag, double* scal, const float* w_t, const double* mw,
                                const float* u_o, int64_t T_all, double* sp0, double* su0, double* su1, double* q64,
                                float* q32, int fp32, unsigned long long* mslot, const int32_t* perm, int su32,
                                float* suf0, float* suf1) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < T) {
        pref[i] = 0.0f;
        c_t[i] = 0.0f;
    }
    if (i < cap) {
        hk[i] = 0ull;
        cr[i] = KCnt{0u, 0x7fffffff};
    }
    if (i < 8) flag[i] = 0;
    if (i < 8) scal[i] = 0.0;
    const double v0 = 1.0 / (double)((int64_t)N + T_all);      // pagerank.py:118-119
    if (i < N) {
        sp0[i] = v0;
        const double su = (double)u_o[perm ? perm[i] : i] * v0;
        su0[i] = su32 ? (double)(float)su : su;   // (fp32 wide graphs: k_tr_a's float copies are exact)
        if (su32) suf0[i] = (float)su;
    }
    if (i >= N && i < N + TR_PAD) su0[i] = su1[i] = 0.0;
    if (su32 && i >= N && i < N + TR_PAD) suf0[i] = suf1[i] = 0.0f;
    if (i < T) {
        const double q = (mw ? mw[i] : (double)w_t[i]) * v0;
        if (fp32) q32[i] = (float)q; else q64[i] = q;
    }
    if (i < MSLOT_WORDS) mslot[i] = i < 2 * MSH ? d2bits(1.0) : 0ull;
}

// Per-graph view for the batched iteration: one k_iter_a / k_iter_b pair per Jacobi iteration
// covers every graph of a batch (the two graphs of an RCA window, or many windows); graph i owns
// blocks [blk0, blk0 + n_tb + n_tiles) of k_iter_a and [blk0b, blk0b + n_ob) of k_iter_b.
struct GDev {
    const int64_t* rs_off;
    const int32_t* rs_ops;
    const uint16_t* rs16;       // u16 copy of rs_ops (N <= 65536) or null
    const uint16_t* rsw;        // the fused kernel's ids: rs16, or rsp in relabelled ops
    const int32_t* perm;        // relabelled ops: perm[new] = old (null: identity)
    int32_t n_hot;              // k_tr_a: su of ops [0, n_hot) in LDS (relabelled graphs)
    const uint16_t* tids;       // k_tr_a: lane-interleaved id chunks of the wave tiles
    const int32_t* coff;        // [n_wt+1] first chunk of a tile
    const int32_t* wtile;       // [waves+1] first tile of each wave of the launch
    const float* c_tp;          // c_t, w_t in position order (tperm)
    const float* w_tp;
    const double* mw_tp;        // kind-compressed graphs: w_t * multiplicity (position order), else null
    const uint8_t* hmask;       // register-accumulated hot ops: trace bits in position order (nhr > 0)
    const uint8_t* trun;        // layout-order graphs: run lengths of identical traces by position (or null)
    const uint32_t* ctids;      // wide graphs: cold chunks of the short-tile walk ([chunk][lane] x 2 labels)
    const int32_t* ccoff;       // [n_wt+1] first cold chunk of a tile
    int32_t nhr;
    int32_t hop[8];
    const float* c_t;
    const float* w_t;
    const float* u_o;
    const float* pw;
    const uint16_t* ltr;
    const int64_t* pr_beg;
    const int32_t* tile_pr0;
    const int32_t* lp;
    const int32_t* tile_lp0;
    const int32_t* op_pr_off;
    const int32_t* op_pr;
    const int64_t* ss_off;
    const int32_t* ss_par;
    void* q[2];
    double* sub[2];
    float* suf[2];                 // su32 graphs: the same su as floats (k_tr_a EXT & 8 gathers these)
    double* spb[2];
    double* part;
    unsigned long long* mslot;
    double *sn, *weight, *scal;    // k_weights_batch: normalised s, weights, scalars
    const int32_t* flag;           // the graph's error words (gathered after the iterations)
    unsigned long long* fx_part;
    double* fx_ssv;
    unsigned long long* fx_limb;   // sharded: [2N] (lo, hi) limb sums per op, then [nranks] r' maxima
    int32_t rank, nranks;          // sharded: this rank's slot of the r' maxima appended to the sum
    double* op_sum;                // sharded tile path: [N] pair-partial sums per op
    double fx_scale, fx_iscale;
    const double* dscale;          // k_tr_a graphs cut on the device: {2^SC, 2^-SC} (k_tr_cut), else null
    // wide fused graphs: k_tr_a's ops [0, NA) (NA = N otherwise); ops [NA, N) in ranges of
    // cold_rw ops whose rows (cold_part, blocks cold_rowbase[r] .. [r+1]) carry scale cx_scale
    int32_t NA, cold_rw;
    int32_t ns_warm;               // k_tr_a EXT & 8: labels [NA, ns_warm) have their su in LDS (else NA)
    int32_t su32;                  // fp32 wide graphs: su rounded to float where k_fx_b makes it
    const double* cold_acc;        // [T] per position: the cold half of the trace's su sum
    const unsigned long long* cold_part;
    const int32_t* cold_rowbase;
    double cx_scale, cx_iscale;
    double alpha;                  // P_ss weight (k_fx_b's call-graph term)
    int32_t T, N, n_tb, n_tiles, tshift, lds_su, blk0, n_ob, blk0b;
    int32_t blk0f, n_fa, blk0fb, n_fb;   // fused path: k_tr_a / k_fx_b block ranges
    int32_t fb_ops;                      // k_fx_b ops per block
    int32_t lastfin;                     // k_tr_a's last block of the graph finishes the iteration (no k_fx_b)
    int32_t pf;                          // k_tr_a(it) first finishes iteration it - 1 itself (no k_fx_b between)
    int64_t pf_stride;                   // pf: words of one partial-row buffer (rows and terms double-buffered)
    int32_t lf_acq;                      // lastfin: the finishing block takes an agent acquire (else the launch
                                         // runs one workgroup per CU and the sc1 hand-off of the guide's row 1 holds)
    int32_t ssv_pre;                     // k_tr_a's blocks compute the call-graph terms (fx_ssv) for k_fx_b
    int32_t row_wt;                      // k_tr_a's partial rows stored write-through (sc1)
};

// graph owning block `blk` of launch kind `which` (0 k_iter_a, 1 k_iter_b, 2 k_tr_a, 3 k_fx_b);
// the start offsets are non-decreasing over graphs (graphs without blocks in a launch repeat it)
__device__ __forceinline__ int32_t graph_of(const GDev* gs, int32_t ng, int32_t blk, int which) {
    int32_t lo = 0, hi = ng - 1;
    while (lo < hi) {
        const int32_t mid = (lo + hi + 1) >> 1;
        const GDev& g = gs[mid];
        const int32_t s = which == 0 ? g.blk0 : which == 1 ? g.blk0b : which == 2 ? g.blk0f : g.blk0fb;
        if (s <= blk) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// One collective per sharded iteration: the r' maximum of this rank travels with the per-op sums
// in a one-hot slot per rank (its bit pattern, or the double itself in an fp64 sum: x + 0 = x),
// so the SUM all-reduce also delivers every rank's maximum.  put: a wave reduces this rank's MSH
// shards into slot[rank] and zeroes the other slots; take: the max over the slots joins the shards.
template <class W>
__device__ __forceinline__ void rmax_put(const GDev& G, const unsigned long long* Mnext, W* slots, int lane) {
    const double m = wave_max(bits2d(Mnext[MSH + lane]));
    for (int j = lane; j < G.nranks; j += WAVE) {
        if constexpr (sizeof(W) == 8 && (W)0.5 == (W)0) slots[j] = j == G.rank ? (W)d2bits(m) : (W)0;
        else slots[j] = j == G.rank ? (W)m : (W)0;
    }
}
__device__ __forceinline__ void rmax_take_bits(const unsigned long long* slots, int n, unsigned long long* Mnext, int lane) {
    unsigned long long b = 0ull;
    for (int j = lane; j < n; j += WAVE) b = max(b, slots[j]);
    const double m = wave_max(bits2d(b));
    if (lane == 0) atomicMax(&Mnext[MSH], d2bits(m));
}
__device__ __forceinline__ void rmax_take_f64(const double* slots, int n, unsigned long long* Mnext, int lane) {
    double b = 0.0;
    for (int j = lane; j < n; j += WAVE) b = nmax(b, slots[j]);
    const double m = wave_max(b);
    if (lane == 0) atomicMax(&Mnext[MSH], d2bits(m));
}

// trace role inner loop: the block's id range in rounds of VCAP ids, all loads in flight before
// the LDS gathers, then each thread continues its own trace's sum in node order
template <class ID>
__device__ __forceinline__ double trace_sums(const ID* __restrict__ ids, int64_t e0, int64_t e1, int64_t a, int64_t b,
                                             const double* su, double* vals) {
    double acc = 0.0;
    for (int64_t lo = e0; lo < e1; lo += VCAP) {
        const int64_t hi = min(lo + (int64_t)VCAP, e1);
        __syncthreads();
        int32_t id[VCAP / TB];
#pragma unroll
        for (int j = 0; j < VCAP / TB; ++j) id[j] = (int32_t)ids[min(lo + threadIdx.x + (int64_t)j * TB, hi - 1)];
#pragma unroll
        for (int j = 0; j < VCAP / TB; ++j) {
            const int64_t e = lo + threadIdx.x + (int64_t)j * TB;
            if (e < hi) vals[e - lo] = su[id[j]];
        }
        __syncthreads();
        const int64_t x0 = max(a, lo), x1 = min(b, hi);
        int64_t e = x0;
        for (; e + 4 <= x1; e += 4) {
            const double v0 = vals[e - lo], v1 = vals[e + 1 - lo], v2 = vals[e + 2 - lo], v3 = vals[e + 3 - lo];
            acc += v0;
            acc += v1;
            acc += v2;
            acc += v3;
        }
        for (; e < x1; ++e) acc += vals[e - lo];
    }
    return acc;
}

// Iteration k, first half.  Maxima are exchanged as the bit patterns of non-negative doubles
// through atomicMax; slot k%3 holds (M_s(k), M_r(k)), slot (k+1)%3 collects iteration k+1, slot
// (k+2)%3 is cleared here for k+2.  s' is carried unnormalised together with su'[o] = u_o*s'[o];
// the division by M_s(k) is applied to each finished sum instead of to every term.
template <class Q>
__global__ void __launch_bounds__(TB) k_iter_a(const GDev* __restrict__ gs, int32_t ng, double d, int it) {
    extern __shared__ double lds[];
    __shared__ double red[TB / WAVE];
    __shared__ double msr;
    __shared__ int32_t sg;
    if (threadIdx.x == 0) sg = graph_of(gs, ng, (int32_t)blockIdx.x, 0);
    __syncthreads();
    const GDev& G = gs[sg];
    const int32_t lb = (int32_t)blockIdx.x - G.blk0;
    const int cur = it & 1, nxt = cur ^ 1, k3 = it % 3;
    const int32_t T = G.T, N = G.N;
    unsigned long long* mslot = G.mslot;
    const unsigned long long* Mcur = mslot + (size_t)2 * MSH * k3;   // [k%3][s|r][MSH]
    unsigned long long* Mnext = mslot + (size_t)2 * MSH * ((k3 + 1) % 3);
    if (lb == 0 && threadIdx.x < 2 * MSH) mslot[(size_t)2 * MSH * ((k3 + 2) % 3) + threadIdx.x] = 0ull;
    if (lb < G.n_tb) {
        // ---- trace role (pagerank.py:125)
        const int32_t t0 = lb * TB;
        const int32_t t1 = min(t0 + TB, T);
        const int32_t t = t0 + threadIdx.x;
        const bool own = t < T;
        const int64_t e0 = G.rs_off[t0], e1 = G.rs_off[t1];
        const int64_t a = own ? G.rs_off[t] : 0, b = own ? G.rs_off[t + 1] : 0;
        const double* su = G.sub[cur];
        if (G.lds_su) {
            for (int32_t o = threadIdx.x; o < N; o += TB) lds[o] = su[o];
            su = lds;
        }
        if (threadIdx.x < WAVE) {
            const double ms = wave_max(bits2d(Mcur[threadIdx.x]));
            if (threadIdx.x == 0) msr = ms;
        }
        double* vals = lds + (G.lds_su ? N : 0);
        const double acc = G.rs16 ? trace_sums(G.rs16, e0, e1, a, b, su, vals) : trace_sums(G.rs_ops, e0, e1, a, b, su, vals);
        __syncthreads();   // msr (also when the block's id range is empty)
        double rmax = -__builtin_huge_val();
        if (own) {
            const double rp = d * (acc / msr) + (double)G.c_t[t];
            ((Q*)G.q[nxt])[t] = (Q)((double)G.w_t[t] * rp);
            rmax = rp;
        }
        rmax = block_max(rmax, red);
        // a block with no trace (an empty shard's placeholder) leaves -inf: no bits to max in
        if (threadIdx.x == 0 && rmax >= 0.0) atomicMax(&Mnext[MSH + blockIdx.x % MSH], d2bits(rmax));
        return;
    }
    // ---- tile role: partial sums of q_k over each (tile, op) pair  (pagerank.py:122-124, P_sr r)
    const int32_t tile = lb - G.n_tb;
    if (tile >= G.n_tiles) return;
    Q* qs = (Q*)lds;
    const Q* __restrict__ qg = (const Q*)G.q[cur];
    const int32_t tb0 = tile << G.tshift;
    const int32_t nt = min(1 << G.tshift, T - tb0);
    const int32_t p0 = G.tile_pr0[tile], p1 = G.tile_pr0[tile + 1];
    const int32_t l0 = G.tile_lp0[tile], l1 = G.tile_lp0[tile + 1];
    for (int32_t i = threadIdx.x; i < nt; i += TB) qs[i] = qg[tb0 + i];
    __syncthreads();
    const uint16_t* __restrict__ ltr = G.ltr;
    const int64_t* __restrict__ pr_beg = G.pr_beg;
    double* part = G.part;
    for (int32_t p = p0 + (int32_t)threadIdx.x; p < p1; p += TB) {   // short pairs: one thread each
        const int64_t b = pr_beg[p], e = pr_beg[p + 1];
        if (e - b > LONG_PAIR) continue;
        double sum = 0.0;
        for (int64_t j = b; j < e; ++j) sum += (double)qs[ltr[j]];
        part[p] = sum;
    }
    const int lane = threadIdx.x & (WAVE - 1);
    for (int32_t i = l0 + (int32_t)(threadIdx.x / WAVE); i < l1; i += TB / WAVE) {   // long pairs: one wave each
        const int32_t p = G.lp[i];
        const int64_t b = pr_beg[p], e = pr_beg[p + 1];
        double sum = 0.0;
        for (int64_t j = b + lane; j < e; j += WAVE) sum += (double)qs[ltr[j]];
        sum = wave_sum(sum);
        if (lane == 0) part[p] = sum;
    }
}

// Iteration k, second half: a wave per op combines the op's pair partials in tile order and adds
// the call-graph term: s'[o] = d * (sum / M_r(k) + alpha * sum_p pw_p s_k[p] / M_s(k))  (:122-124)
// Sharded graphs (traces split over ranks) run it twice around an fp64 SUM all-reduce of the
// per-op sums: mode 1 writes this rank's sum to op_sum, mode 2 finishes from the reduced op_sum.
__global__ void __launch_bounds__(TB) k_iter_b(const GDev* __restrict__ gs, int32_t ng, double d, double alpha, int it,
                                               int mode) {
    __shared__ int32_t sg;
    if (threadIdx.x == 0) sg = graph_of(gs, ng, (int32_t)blockIdx.x, 1);
    __syncthreads();
    const GDev& G = gs[sg];
    const int32_t o = ((int32_t)blockIdx.x - G.blk0b) * (TB / WAVE) + (int32_t)(threadIdx.x / WAVE);
    if (o >= G.N) return;
    const int lane = threadIdx.x & (WAVE - 1);
    const int cur = it & 1, nxt = cur ^ 1, k3 = it % 3;
    const unsigned long long* Mcur = G.mslot + (size_t)2 * MSH * k3;
    unsigned long long* Mnext = G.mslot + (size_t)2 * MSH * ((k3 + 1) % 3);
    double sum = 0.0;
    if (mode != 2) {
        for (int32_t i = G.op_pr_off[o] + lane; i < G.op_pr_off[o + 1]; i += WAVE) sum += G.part[G.op_pr[i]];
        sum = wave_sum(sum);
        if (mode == 1) {
            if (lane == 0) G.op_sum[o] = sum;
            if (o == 0) rmax_put(G, Mnext, G.op_sum + G.N, lane);   // this rank's r' max, one-hot
            return;
        }
    } else {
        sum = G.op_sum[o];
        if (o == 0) rmax_take_f64(G.op_sum + G.N, G.nranks, Mnext, lane);
    }
    const double Ms = wave_max(bits2d(Mcur[lane])), Mr = wave_max(bits2d(Mcur[MSH + lane]));
    const double* sp_cur = G.spb[cur];
    double bb = 0.0;
    for (int64_t e = G.ss_off[o] + lane; e < G.ss_off[o + 1]; e += WAVE) {
        const int32_t p = G.ss_par[e];
        bb += (double)G.pw[p] * sp_cur[p];
    }
    bb = wave_sum(bb);
    if (lane == 0) {
        const double v = d * (sum / Mr + alpha * (bb / Ms));      // pagerank.py:122-124
        G.spb[nxt][o] = v;
        G.sub[nxt][o] = (double)G.u_o[o] * v;
        atomicMax(&Mnext[o % MSH], d2bits(v));
    }
}

// ---------------------------------------------------------------- fused single-pass iteration
// For graphs with N <= FX_NMAX and P_rs == P_sr (every graph built from spans): ONE read of the
// trace-major u16 ids per iteration serves both products of pagerank.py:122-125.
//   k_tr_a  lane = trace (wave tiles of 64 traces, below):
//     r'[t]   = d * sum_{o in ops(t)} su_k[o] / M_s(k) + fp32((1-d) v_t)        (layout order)
//     lacc[o] += X_t for o in ops(t),   X_t = rint(w_t r'_k[t] / M_r(k) * 2^SC)   (LDS, u64)
//   The block's N accumulators go out as one dense row part[block][0..N).  Because X_t <= 2^SC
//   (w_t <= 1, r'_k <= M_r(k)) and SC = 64 - bits(traces of the block), a row entry stays < 2^64.
//   k_fx_b  wave per op: S_o = sum over blocks of part[.][o] as two exact 32-bit-limb sums, one
//   rounding to double, then s'[o] = d * (S_o 2^-SC + alpha * sum_p pw_p s_k[p] / M_s(k)).
// Integer sums are exact, so the result does not depend on atomic or reduction order: runs are
// bitwise reproducible, and the quantisation (2^-SC absolute per term, SC >= 53) sits below
// fp64's own rounding of the reference's dot products.
constexpr int FX_NMAX = 16384;
// global-memory views of pointers read from GDev: loads through them compile to global_load
// (vmcnt only) instead of flat_load, whose lgkmcnt share would make every LDS wait also wait
// for outstanding HBM loads
#define GLB __attribute__((address_space(1)))
__device__ __forceinline__ int64_t rfl64(int64_t v) {   // a wave-uniform value held in VGPRs -> SGPRs
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <class T>
__device__ __forceinline__ const GLB T* gp(const T* p) { return (const GLB T*)p; }
template <class T>
__device__ __forceinline__ GLB T* gpw(T* p) { return (GLB T*)p; }

// graph of a fused-launch block: ng <= 2 resolves from the scalar split (no memory hop)
__device__ __forceinline__ int32_t fx_graph(const GDev* gs, int32_t ng, int32_t split, int which) {
    if (ng == 1) return 0;
    if (ng == 2) return (int32_t)blockIdx.x >= split ? 1 : 0;
    return graph_of(gs, ng, (int32_t)blockIdx.x, which);
}

// ---------------------------------------------------------------- fused iteration: LDS budget and su modes
constexpr size_t WV_LDS_MAX = 160 * 1024 - 512;
// su modes of k_tr_a: global gathers only / every op's su in LDS / the n_hot most covered ops' su in
// LDS (relabelled graphs, ops [0, n_hot)), the rest gathered
enum { WV_SU_GLOBAL = 0, WV_SU_ALL = 1, WV_SU_HOT = 2 };

// ---------------------------------------------------------------- fused iteration, trace-parallel (k_tr_a)
// The single-pass iteration with lane = trace.  At prepare a graph's traces are sorted by op
// count (tperm: position -> trace) and cut into wave tiles of 64 positions; a tile stores its
// traces' ids lane-interleaved in chunks of 4 (chunk c = 64 lanes x 4 u16: one coalesced 512-B
// load), padded to the tile's longest trace with N + lane (a zero su slot and a dummy
// accumulator per lane, so pads neither branch nor collide), and each trace rotated by
// (lane mod len): a trace's first op is often a root shared by the whole tile, and rotation
// spreads those atomics over the chunk's four instructions and many lanes' addresses.
// Each wave streams a contiguous run of tiles as ONE chunk stream -- ids three chunks ahead,
// the su of cold ops (WV_SU_HOT / GLOBAL) one chunk ahead, a tile's q, (1-d) v and w one tile
// ahead -- with every load unconditional (clamped), so each use waits for exactly its own load.
// Per entry: one su read (LDS, or the prefetched gather), one add into the lane's own trace sum
// (sequential: deterministic), one LDS u64 atomic of the lane's X_t (integers: order-free).  The
// block synchronises only to clear the accumulator and to write its partial row.
struct TrLds {
    size_t su, lacc, hs, sp, total;
    bool su_lds;      // every op's su fits beside the accumulator (interleaved: 16 B per op)
    bool hot_ok;      // WV_SU_ALL: the hot-op mask sums (256 doubles) fit too
    int32_t n_hot;    // WV_SU_HOT: su of ops [0, n_hot) in LDS
    // the accumulator first, then su (8-B strides: a 32-lane read group spreads over 32 bank
    // pairs, a 16-lane atomic group over 16)
    // pf (every op's su in LDS only): s itself beside su (the launch finished the previous iteration)
    // w32 (fp32 wide graphs, k_tr_a EXT & 8): su as 4-B floats -- the hot ops, their 64 pad slots,
    // then n_warm "warm" cold labels (NA + j at slot NA + 64 + j) in the space the floats free
    int32_t n_warm;
    __host__ __device__ TrLds(int32_t N, int mode, bool pf = false, bool w32 = false) {
        const size_t ns = (size_t)N + TR_PAD;
        su_lds = ns * 16 <= WV_LDS_MAX;
        const bool all = mode == WV_SU_ALL && su_lds;
        const size_t accb = (ns * 8 + 15) / 16 * 16;
        n_hot = 0;
        n_warm = 0;
        if (mode == WV_SU_HOT && accb < WV_LDS_MAX)
            n_hot = (int32_t)std::min<size_t>((size_t)N, (WV_LDS_MAX - accb) / 8 / 64 * 64);
        lacc = 0;
        su = accb;
        total = all ? 2 * accb : accb + (size_t)n_hot * 8;
        if (all && w32 && !pf) {   // (the hot-op mask sums keep their 2 KB)
            const size_t fl = (WV_LDS_MAX - accb - 256 * 8 - 16) / 4;
            n_warm = fl > ns ? (int32_t)((fl - ns) / 64 * 64) : 0;
            total = accb + ((ns + (size_t)n_warm) * 4 + 15) / 16 * 16;
        }
        sp = total;
        if (pf && all) total += accb;
        hs = total;
        hot_ok = all && total + 256 * 8 <= WV_LDS_MAX;
        if (hot_ok) total += 256 * 8;
    }
};

__device__ __forceinline__ double uni_d(double v) {   // a block-uniform double into SGPRs
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(unsigned)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// Short tiles (tiles of exactly NC chunks, NC <= 8: traces of <= 32 ops), su in LDS: a tile is ONE register
// set -- its NC id chunks, q, c = (1-d) v, w (EXT & 1: the kind multiplicity's mw instead),
// the cold half of the sums (EXT & 2), and the chunk offsets of the next two tiles -- loaded
// unconditionally (addresses clamped) one whole tile ahead.  The tile loop is unrolled by two so
// the two register sets alternate by renaming: no register with a load in flight is ever copied,
// so the only memory waits are for loads issued a tile earlier (the ring of tr_walk's general
// loop below rotates per chunk and at tile ends has to copy the next tile's q, which made every
// tile end wait for all loads in flight, the ids three chunks ahead included).  Tiles are sorted
// by length, so a wave's run is a sequence of short-tile tiers (NC = 1, 2, .., 8, each a code copy
// with every count static) and a suffix of longer tiles the general loop takes.  Same per-lane sums
// in the same order as the general loop: bitwise equal results.
// su in k_tr_a's LDS: doubles, or 4-B floats on fp32 wide graphs (EXT & 8: every su value of such
// a graph is rounded to float where it is made, so the float copy is exact)
template <class Q, int EXT>
using TrSu = std::conditional_t<((EXT & 8) != 0) && std::is_same<Q, float>::value, float, double>;
template <class Q, int NC, int EXT>
struct TrTile {
    u32x2 id[NC];
    Q q;
    float c;
    float w;
    double mw;     // EXT & 1: w times the kind multiplicity (kind-compressed graphs)
    u32x2 cid[2];  // EXT & 2: the tile's first two cold chunks (wide graphs: 2 cold labels per lane each)
    double xo;     // EXT & 2: k_cold_trace's sum when the tile has more cold chunks (else a dummy)
    int32_t ccw;   // EXT & 2: lane j: ccoff[k + 1 + j] (the next tile's cold chunk range)
    int32_t cw;    // lane j: coff[k + 1 + j] (readlane 0 / 1: the next tile's chunk range)
    uint32_t hm;   // the trace's hot-op bits (nhr > 0)
    uint32_t rl;   // the run of identical traces this lane heads (0: another lane's run; 1: its own)
    uint32_t rln;  // the next tile's rl (a tail loads nothing of its own: its loads need it a tile ahead)
    u32x2 cidn[2]; // EXT & 8: the NEXT tile's first two cold chunks (its gathers go out a tile early)
    float cf[4];   // EXT & 8: this tile's non-warm cold su, gathered while the previous tile walked
    float xw;      // EXT & 8: this tile's warm cold su (LDS), summed at the previous tile's end
};
// the hot ops of a trace: their su first in the lane's sum (the same order in both walks), X into
// the lane's register accumulators (integers: order-free; flushed once per walk)
// The su part is one LDS read of hs[hm] = the sum of the trace's hot su in h order (k_tr_a builds
// the 256 sums per iteration: adding the absent ops' +0.0 would not change a sum, so hs[hm] is the
// lane's own sequential sum over its hot ops).
constexpr int HOT_MAX_WIDE = 4;   // wide graphs' k_tr_a variant (its cold registers): 4 accumulators
template <int HN>
struct TrHot {
    int32_t n;
    const double* hs;   // LDS [256]
    unsigned long long acc[HN];
};
// (every one of the HOT_MAX accumulators is updated: ops past nhr are never in a mask, so they
// add 0 -- no per-op condition, no duplicated registers)
template <int HN>
__device__ __forceinline__ double tr_hot_init(TrHot<HN>& H, uint32_t hm, unsigned long long X) {
#pragma unroll
    for (int h = 0; h < HN; ++h) {
        const unsigned long long sel = (unsigned long long)(long long)(((int32_t)(hm << (31 - h))) >> 31);
        H.acc[h] += X & sel;
    }
    return H.hs[hm];
}
// hs[m] for m = tid < 256 (su of every op in LDS; the caller synchronises before and after)
template <class SU>
__device__ __forceinline__ void tr_hot_sums(const GDev& G, const SU* su_l, double* hs, int32_t tid) {
    if (tid < 256) {
        double a = 0.0;
        for (int h = 0; h < G.nhr; ++h)
            if ((tid >> h) & 1) a += su_l[G.hop[h]];
        hs[tid] = a;
    }
}
template <class Q, int NC, int EXT, int HN>
__device__ __forceinline__ int32_t tr_walk_short(const GDev& G, int32_t k, const int32_t ke, int32_t T, int32_t lane,
                                                 int cur, int nxt, double d, double Ms, double xsc, const TrSu<Q, EXT>* su_l,
                                                 unsigned long long* lacc, double& rmax, TrHot<HN>& H, int32_t& c0,
                                                 int32_t& n, int32_t& q0, int32_t& nq) {
    const GLB int32_t* coff = gp(G.coff);
    const GLB Q* qc = gp((const Q*)G.q[cur]);
    GLB Q* qn = gpw((Q*)G.q[nxt]);
    const GLB float* c_tp = gp(G.c_tp);
    const GLB float* w_tp = gp(G.w_tp);
    // EXT: a graph of the launch may carry mw / cold sums; graphs without them load a valid dummy
    // (su[0]) and select the plain value -- unconditional loads, no branches around them
    const GLB double* sug = gp(G.sub[cur]);
    const bool kc = (EXT & 1) && G.mw_tp, cx = (EXT & 2) && G.cold_acc;
    const GLB double* mw_tp = kc ? gp(G.mw_tp) : sug;
    // wide graphs: the cold entries' su gathered here (issued when a tile starts, summed when it
    // ends: a tile of LDS work hides the L2 latency), no cold_acc pass for these tiles
    const GLB u32x2* cids = gp((const u32x2*)G.ctids) + lane;
    const GLB int32_t* ccoff = cx ? gp(G.ccoff) : coff;
    const int32_t ccl = max(__builtin_amdgcn_readfirstlane(ccoff[ke]) - 1, 0);
    const uint32_t cpad = (uint32_t)(G.N + lane);
    // EXT & 8: cold labels below ns_warm ("warm") read their su from LDS slot label + TR_PAD; the
    // other labels from global memory.  Both reads issue for every slot: the LDS one of a non-warm
    // label reads the lane's zero pad slot NA + lane, the global one of a warm label the lane's zero
    // pad N + lane (one coalesced line per wave) -- the sum of the two is the label's su exactly
    constexpr bool W32 = (EXT & 8) != 0;
    const uint32_t nsw = W32 ? (uint32_t)G.ns_warm : 0u, lzero = W32 ? (uint32_t)(G.NA + lane) : 0u;
    const GLB float* sugf = W32 ? gp((const float*)G.suf[cur]) : nullptr;
    const bool hot = H.n > 0;
    const GLB uint8_t* hmk = hot ? gp(G.hmask) : (const GLB uint8_t*)coff;
    // EXT & 4: run-merged graphs (trun).  Without it the run logic is compiled out: every lane walks
    // its own trace (the headline walk)
    constexpr bool RUNS = (EXT & 4) != 0;
    const GLB uint8_t* trn = RUNS ? gp(G.trun) : nullptr;
    const int32_t cl = __builtin_amdgcn_readfirstlane(coff[ke]) - 1;   // the run's last chunk
    // the first tile's chunk ranges: handed over by the previous tier (n >= 0), else loaded
    if (n < 0) {
        const int32_t v = coff[min(k + lane, ke)];
        c0 = __builtin_amdgcn_readfirstlane(v);
        n = __builtin_amdgcn_readlane(v, 1) - c0;
        if constexpr ((EXT & 2) != 0) {
            const int32_t u = ccoff[min(k + lane, ke)];
            q0 = __builtin_amdgcn_readfirstlane(u);
            nq = __builtin_amdgcn_readlane(u, 1) - q0;
        }
    }
    if (n != NC) return k;
    using R = TrTile<Q, NC, EXT>;
    const GLB double* cacc = cx ? gp(G.cold_acc) : sug;
    // run marks of tile kk's lanes (1 on graphs without runs)
    auto rl_of = [&](int32_t kk) -> uint32_t {
        if constexpr (!RUNS) return 1u;
        return trn ? (uint32_t)trn[min(min(kk, ke - 1) * WAVE + lane, T - 1)] : 1u;
    };
    // a run's tail (rl 0) needs none of its own ids, q, c or w -- the head walks for it and its r'
    // comes by shuffle -- so its loads go to one shared word each (one cache line per load, not
    // its own): unconditional loads, no branch
    const GLB u32x2* idb = gp((const u32x2*)G.tids);
    auto load = [&](R& r, int32_t kk, int32_t cc0, int32_t qq0, int32_t nqq, uint32_t rl, int32_t qn1 = 0) {
        const int32_t kq = min(kk, ke - 1);
        const int32_t p = min(kq * WAVE + lane, T - 1);
        const bool hd = !RUNS || rl != 0u;
        const int32_t ph = hd ? p : 0;
#pragma unroll
        for (int j = 0; j < NC; ++j) r.id[j] = idb[hd ? (size_t)min(cc0 + j, cl) * WAVE + lane : 0];
        r.q = qc[ph];
        r.c = c_tp[ph];
        r.w = w_tp[ph];
        if constexpr ((EXT & 1) != 0) r.mw = mw_tp[kc ? p : 0];
        if constexpr ((EXT & 2) != 0) {
            if (cx) {   // (uniform; ctids exists only on wide graphs)
                if constexpr (W32) {   // tile kk + 1's labels (its first cold chunk qn1)
                    r.cidn[0] = cids[(size_t)min(qn1, ccl) * WAVE];
                    r.cidn[1] = cids[(size_t)min(qn1 + 1, ccl) * WAVE];
                } else {
                    r.cid[0] = cids[(size_t)min(qq0, ccl) * WAVE];
                    r.cid[1] = cids[(size_t)min(qq0 + 1, ccl) * WAVE];
                }
            }
            r.xo = cacc[nqq > 2 ? p : 0];   // (unconditional: a branch here costs ~50 VGPRs)
            r.ccw = ccoff[min(kq + 1 + lane, ke)];
        }
        r.cw = coff[min(kq + 1 + lane, ke)];
        r.hm = hot ? hmk[p] : 0u;   // (uniform)
        r.rl = rl;
        r.rln = rl_of(kk + 1);
    };
    // tile kk from r: lane = position kk * 64 + lane
    // EXT & 8: a tile's cold labels (l4: pads past its cold chunk count), their non-warm su gathered
    // into dst.cf (global; warm labels read the lane's zero pad) and their warm su summed into
    // dst.xw (LDS; non-warm labels read the lane's zero pad slot)
    auto labels = [&](const u32x2 (&cid)[2], int32_t nqq, uint32_t (&l4)[4]) {
        l4[0] = nqq > 0 ? cid[0].x : cpad;
        l4[1] = nqq > 0 ? cid[0].y : cpad;
        l4[2] = nqq > 1 ? cid[1].x : cpad;
        l4[3] = nqq > 1 ? cid[1].y : cpad;
    };
    auto gissue = [&](R& dst, const u32x2 (&cid)[2], int32_t nqq) {
        uint32_t l4[4];
        labels(cid, nqq, l4);
#pragma unroll
        for (int i = 0; i < 4; ++i) dst.cf[i] = sugf[l4[i] < nsw ? cpad : l4[i]];
    };
    auto wsum = [&](R& dst, const u32x2 (&cid)[2], int32_t nqq) {
        uint32_t l4[4];
        labels(cid, nqq, l4);
        float a = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i) a += (float)su_l[l4[i] < nsw ? l4[i] + (uint32_t)TR_PAD : lzero];
        dst.xw = a;
    };
    // W32: nx = the next tile's register set (its gathers issued here from r.cidn, its warm sum at
    // the end), nqn = the next tile's cold chunk count
    auto run = [&](const R& r, int32_t kk, int32_t qq0, int32_t nqq, R* nx = nullptr, int32_t nqn = 0) {
        const int32_t p = kk * WAVE + lane;
        const bool own = p < T;
        double cg[4] = {0.0, 0.0, 0.0, 0.0};
        if constexpr (W32)
            if (cx) gissue(*nx, r.cidn, nqn);
        if constexpr ((EXT & 2) != 0 && !W32)
            if (cx) {   // the first two cold chunks' su (pads past the tile's chunk count: N + lane, 0)
#ifdef MR_AB_NOGATHER   // (A/B timing builds only: every gather at the lane's pad -- wrong sums)
                const uint32_t z = (r.cid[0].x ^ r.cid[1].y) & 0u;
                cg[0] = sug[cpad + z]; cg[1] = sug[cpad + z]; cg[2] = sug[cpad + z]; cg[3] = sug[cpad + z];
#else
                const uint32_t l4[4] = {nqq > 0 ? r.cid[0].x : cpad, nqq > 0 ? r.cid[0].y : cpad,
                                        nqq > 1 ? r.cid[1].x : cpad, nqq > 1 ? r.cid[1].y : cpad};
#pragma unroll
                for (int i = 0; i < 4; ++i) cg[i] = sug[l4[i]];
#endif
            }
        // a run of rl identical traces (the same ops in the same order, the same q, c and w: the
        // same sum and r') is walked by its head alone: its X times rl into the accumulators (integers:
        // exactly the rl separate adds), its r' broadcast to the run below
        const bool hd = !RUNS || r.rl != 0u;
        const unsigned long long X0 = own && hd ? (unsigned long long)__double2ull_rn((double)r.q * xsc) : 0ull;
        const unsigned long long X = RUNS ? X0 * (unsigned long long)r.rl : X0;
        double acc = H.n ? tr_hot_init(H, r.hm, X) : 0.0;
        if (hd) {
            double sv[2][4];
            auto rd = [&](const u32x2 w, double* s) {
                s[0] = su_l[w.x & 0xffffu];
                s[1] = su_l[w.x >> 16];
                s[2] = su_l[w.y & 0xffffu];
                s[3] = su_l[w.y >> 16];
            };
            rd(r.id[0], sv[0]);
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                if (j + 1 < NC) rd(r.id[j + 1], sv[(j + 1) & 1]);
                const u32x2 w = r.id[j];
                atomicAdd(&lacc[(w.x & 0xffffu)], X);
                atomicAdd(&lacc[(w.x >> 16)], X);
                atomicAdd(&lacc[(w.y & 0xffffu)], X);
                atomicAdd(&lacc[(w.y >> 16)], X);
#pragma unroll
                for (int i = 0; i < 4; ++i) acc += sv[j & 1][i];
            }
        }
        double x = 0.0;   // the cold half, sequential in the trace's cold order (k_cold_trace's)
        if constexpr ((EXT & 2) != 0)
            if (cx) {
#pragma unroll
                for (int i = 0; i < 4; ++i) x += W32 ? (double)r.cf[i] : cg[i];
                if constexpr (W32) {
                    x += (double)r.xw;   // (the warm part after the global one: a fixed order)
                    wsum(*nx, r.cidn, nqn);   // the next tile's warm sum (its labels still in r)
                }
                if (nqq > 2) x = r.xo;   // (rare: > 4 cold entries in a trace of the tile: k_cold_trace's sum)
            }
        double rp = d * ((acc + x) / Ms) + (double)r.c;   // pagerank.py:125
        if (RUNS && trn) {   // (uniform) the run's head's r'
            const unsigned long long hb = __ballot(hd) & (lane == WAVE - 1 ? ~0ull : (2ull << lane) - 1ull);
            rp = __shfl(rp, 63 - __builtin_clzll(hb), WAVE);
        }
        if (own) rmax = nmax(rmax, rp);
        const double wq = kc ? r.mw : (double)r.w;
        qn[own && hd ? p : T] = (Q)(wq * rp);   // q[T]: pad slot (a run's tails never read theirs)
    };
    R A, B;
    if constexpr (W32) {
        // the tier's first tile: its cold labels and gathers here (later tiles' go out a tile early),
        // the next tile's cold range from lanes 1 and 2 of the cold offsets
        const int32_t u3 = ccoff[min(k + lane, ke)];
        const int32_t q1 = __builtin_amdgcn_readlane(u3, 1), nq1 = __builtin_amdgcn_readlane(u3, 2) - q1;
        u32x2 c0v[2];
        c0v[0] = cids[(size_t)min(q0, ccl) * WAVE];
        c0v[1] = cids[(size_t)min(q0 + 1, ccl) * WAVE];
        if (cx) {
            gissue(A, c0v, nq);
            wsum(A, c0v, nq);
        }
        load(A, k, c0, q0, nq, rl_of(k), q1);
        int32_t nqA1 = nq1;   // tile k + 1's cold chunk count
        for (;;) {
            const int32_t c0B = __builtin_amdgcn_readfirstlane(A.cw);
            const int32_t nB = __builtin_amdgcn_readlane(A.cw, 1) - c0B;
            const int32_t qB = __builtin_amdgcn_readfirstlane(A.ccw);
            const int32_t nqB = __builtin_amdgcn_readlane(A.ccw, 1) - qB;
            const int32_t qB1 = __builtin_amdgcn_readlane(A.ccw, 1), nqB1 = __builtin_amdgcn_readlane(A.ccw, 2) - qB1;
            load(B, k + 1, c0B, qB, nqB, A.rln, qB1);
            run(A, k, q0, nq, &B, nqA1);
            if (++k == ke || nB != NC) {
                c0 = c0B, n = nB, q0 = qB, nq = nqB;
                break;
            }
            const int32_t c0A = __builtin_amdgcn_readfirstlane(B.cw);
            const int32_t nA2 = __builtin_amdgcn_readlane(B.cw, 1) - c0A;
            const int32_t qA2 = __builtin_amdgcn_readfirstlane(B.ccw);
            const int32_t nqA2 = __builtin_amdgcn_readlane(B.ccw, 1) - qA2;
            const int32_t qA1 = __builtin_amdgcn_readlane(B.ccw, 1);
            nqA1 = __builtin_amdgcn_readlane(B.ccw, 2) - qA1;
            load(A, k + 1, c0A, qA2, nqA2, B.rln, qA1);
            run(B, k, qB, nqB, &A, nqB1);
            if (++k == ke || nA2 != NC) {
                c0 = c0A, n = nA2, q0 = qA2, nq = nqA2;
                break;
            }
            q0 = qA2, nq = nqA2;
        }
        return k;
    }
    load(A, k, c0, q0, nq, rl_of(k));
    int32_t nA = n, qA = q0, nqA = nq;
    for (;;) {
        // B = tile k + 1 (its ranges from A's offsets), then A's tile
        const int32_t c0B = __builtin_amdgcn_readfirstlane(A.cw);
        const int32_t nB = __builtin_amdgcn_readlane(A.cw, 1) - c0B;
        int32_t qB = 0, nqB = 0;
        if constexpr ((EXT & 2) != 0) {
            qB = __builtin_amdgcn_readfirstlane(A.ccw);
            nqB = __builtin_amdgcn_readlane(A.ccw, 1) - qB;
        }
        load(B, k + 1, c0B, qB, nqB, A.rln);
        run(A, k, qA, nqA);
        if (++k == ke || nB != NC) {
            c0 = c0B, n = nB, q0 = qB, nq = nqB;
            break;
        }
        const int32_t c0A = __builtin_amdgcn_readfirstlane(B.cw);
        nA = __builtin_amdgcn_readlane(B.cw, 1) - c0A;
        if constexpr ((EXT & 2) != 0) {
            qA = __builtin_amdgcn_readfirstlane(B.ccw);
            nqA = __builtin_amdgcn_readlane(B.ccw, 1) - qA;
        }
        load(A, k + 1, c0A, qA, nqA, B.rln);
        run(B, k, qB, nqB);
        if (++k == ke || nA != NC) {
            c0 = c0A, n = nA, q0 = qA, nq = nqA;
            break;
        }
    }
    return k;
}

// The wave's walk of k_tr_a over its run of wave tiles: per entry one
// su read, one add into the lane's trace sum, one LDS u64 atomic of X_t; per tile r' of its traces
// and their next q.  Returns the wave's largest r' (-inf when it owns no trace).
template <class Q, int SUM, int NT, int EXT = 0, bool HOTT = false>
__device__ __forceinline__ double tr_walk(const GDev& G, int32_t lb, int cur, int nxt, int32_t N, int32_t NH, double d,
                                          double Ms, double xsc, const TrSu<Q, EXT>* su_l, unsigned long long* lacc,
                                          const double* hs = nullptr) {
    constexpr bool SUL = SUM == WV_SU_ALL, HOT = SUM == WV_SU_HOT;
    constexpr int NW = NT / WAVE;
    const int32_t T = G.T;
    const int32_t tid = (int32_t)threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
    const GLB u32x2* ids = gp((const u32x2*)G.tids) + lane;   // chunk c of this lane: ids[c * WAVE]
    const GLB int32_t* coff = gp(G.coff);
    const GLB Q* qc = gp((const Q*)G.q[cur]);
    GLB Q* qn = gpw((Q*)G.q[nxt]);
    const GLB float* c_tp = gp(G.c_tp);
    const GLB float* w_tp = gp(G.w_tp);
    const GLB double* sug = gp(G.sub[cur]);   // ids >= N are pads (su 0)
    // this wave's tiles [k, ke) (a contiguous run: the host cuts them by chunk count)
    const GLB int32_t* wt = gp(G.wtile) + ((size_t)lb * NW + wv);
    int32_t k = __builtin_amdgcn_readfirstlane(wt[0]);
    const int32_t ke = __builtin_amdgcn_readfirstlane(wt[1]);
    double rmax = -__builtin_huge_val();
    constexpr int HN = (EXT & 2) ? HOT_MAX_WIDE : HOT_MAX;
    TrHot<HN> H;
    H.n = SUL && HOTT ? __builtin_amdgcn_readfirstlane(G.nhr) : 0;   // (the host strips only such graphs)
    H.hs = hs;
#pragma unroll
    for (int h = 0; h < HN; ++h) H.acc[h] = 0ull;
    const int32_t k_first = k;
    if constexpr (SUL) {
        // one tier per chunk count (the run's tiles ascend in it): every count static, no branch
        // inside a tile, so each wait is for exactly the LDS reads and loads it consumes
        int32_t tc0 = 0, tn = -1, tq0 = 0, tnq = 0;   // the next tile's ranges, handed from tier to tier
#define TR_TIER(NC_) if (NC_ <= ((EXT & 8) ? TR_TIERS_W32 : NT == 1024 || (EXT & 3) ? TR_TIERS_EXT : MR_TR_TIERS512) && k < ke) k = tr_walk_short<Q, NC_, EXT, HN>(G, k, ke, T, lane, cur, nxt, d, Ms, xsc, su_l, lacc, rmax, H, tc0, tn, tq0, tnq);
        TR_TIER(1) TR_TIER(2) TR_TIER(3) TR_TIER(4) TR_TIER(5) TR_TIER(6) TR_TIER(7) TR_TIER(8)
#undef TR_TIER
    }
    const GLB uint8_t* hmk = gp(G.hmask);
    if (k < ke) {
        auto pos = [&](int32_t kk) { return min(kk * WAVE + lane, T - 1); };
        // cold-op su of a chunk (LDS-resident ops load sug[0]: one line, no traffic; pads read as 0)
        auto gather = [&](const u32x2 w, double* g) {
            const int32_t o[4] = {(int32_t)(w.x & 0xffffu), (int32_t)(w.x >> 16), (int32_t)(w.y & 0xffffu),
                                  (int32_t)(w.y >> 16)};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const double v = SUL ? 0.0 : sug[HOT && o[j] < NH ? 0 : min(o[j], N - 1)];
                g[j] = o[j] < N ? v : 0.0;
            }
        };
        int32_t c = __builtin_amdgcn_readfirstlane(coff[k]);
        int32_t ce = __builtin_amdgcn_readfirstlane(coff[k + 1]);   // end of tile k
        const int32_t cl = __builtin_amdgcn_readfirstlane(coff[ke]) - 1;   // the run's last chunk
        // tile k's words; tile k + 1's q and end chunk (one tile ahead, clamped into the run).  The
        // end chunk is loaded per lane (lane-varying address: a vector load -- a scalar load would
        // share lgkmcnt with the LDS traffic and force full drains)
        const int32_t kn = min(k + 1, ke - 1);
        // w_t of a position: times the kind's multiplicity on a kind-compressed graph (uniform branch)
        const GLB double* mw_tp = gp(G.mw_tp);
        auto wq = [&](int32_t kk) { return mw_tp ? mw_tp[pos(kk)] : (double)w_tp[pos(kk)]; };
        double q_cur = (double)qc[pos(k)];
        float c_cur = c_tp[pos(k)];
        // wide graphs: the cold half of the trace's sum (k_cold_trace), else 0 (acc + 0 = acc)
        const GLB double* cacc = gp(G.cold_acc);
        double x_cur = cacc ? cacc[pos(k)] : 0.0;
        double w_cur = wq(k);
        double q_nx = (double)qc[pos(kn)];
        int32_t ce_nx = coff[min(kn + 1 + lane, ke)];
        // su of a chunk's ops from LDS (HOT: the hot part; the cold part comes from gather)
        auto lds_su = [&](const u32x2 w, double* sv) {
            const int32_t o[4] = {(int32_t)(w.x & 0xffffu), (int32_t)(w.x >> 16), (int32_t)(w.y & 0xffffu),
                                  (int32_t)(w.y >> 16)};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                sv[j] = SUL ? su_l[o[j]] : HOT ? su_l[min(o[j], NH - 1)] : 0.0;
            }
        };
        // ids ring (4 chunks: the current one and three ahead), su ping-pong (current, next)
        u32x2 wa = ids[(size_t)c * WAVE];
        u32x2 wb = ids[(size_t)min(c + 1, cl) * WAVE];
        u32x2 wc = ids[(size_t)min(c + 2, cl) * WAVE];
        u32x2 wd;
        double gA[4], gB[4], sA[4], sB[4];
        if (!SUL) gather(wa, gA);
        if (SUL || HOT) lds_su(wa, sA);
        unsigned long long X = k * WAVE + lane < T ? (unsigned long long)__double2ull_rn(q_cur * xsc) : 0ull;
        double acc = H.n ? tr_hot_init(H, hmk[pos(k)], X) : 0.0;
        // One chunk: ids CUR (here), su SC / GC (LDS here, cold gathers in flight); NXT's cold
        // gathers and LDS reads go out before CUR's atomics (their latency, bank conflicts
        // included, overlaps a whole chunk), and the ids three chunks ahead land in LD.  The loop
        // is unrolled 4x so the ring rotates by renaming, not by register moves (a move of an
        // in-flight register would wait for it).
#define TR_STEP(CUR, NXT, LD, GC, SC, GN, SN)                                                              \
        {                                                                                                  \
            LD = ids[(size_t)min(c + 3, cl) * WAVE];                                                       \
            if (!SUL) gather(NXT, GN);                                                                     \
            if (SUL || HOT) lds_su(NXT, SN);                                                               \
            const int32_t o_[4] = {(int32_t)(CUR.x & 0xffffu), (int32_t)(CUR.x >> 16),                     \
                                   (int32_t)(CUR.y & 0xffffu), (int32_t)(CUR.y >> 16)};                    \
            _Pragma("unroll") for (int j = 0; j < 4; ++j) atomicAdd(&lacc[o_[j]], X);                         \
            _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                  \
                acc += SUL ? SC[j] : HOT ? (o_[j] < NH ? SC[j] : GC[j]) : GC[j];                          \
            if (++c == ce) {                                                                               \
                /* tile k done: r' of its traces (pagerank.py:125) and the next q */                      \
                const int32_t p_ = k * WAVE + lane;                                                        \
                const bool own_ = p_ < T;                                                                  \
                const double rp_ = d * ((acc + x_cur) / Ms) + (double)c_cur;                               \
                if (own_) rmax = nmax(rmax, rp_);                                                          \
                qn[own_ ? p_ : T] = (Q)(w_cur * rp_);   /* q[T]: pad slot */                              \
                if (++k == ke) goto tr_done;                                                               \
                ce = __builtin_amdgcn_readfirstlane(ce_nx);                                                \
                q_cur = q_nx;                                                                              \
                const int32_t kk_ = min(k + 1, ke - 1);                                                    \
                c_cur = c_tp[pos(k)];                                                                      \
                x_cur = cacc ? cacc[pos(k)] : 0.0;                                                         \
                w_cur = wq(k);                                                                             \
                q_nx = (double)qc[pos(kk_)];                                                               \
                ce_nx = coff[min(kk_ + 1 + lane, ke)];                                                     \
                X = p_ + WAVE < T ? (unsigned long long)__double2ull_rn(q_cur * xsc) : 0ull;               \
                acc = H.n ? tr_hot_init(H, hmk[pos(k)], X) : 0.0;                                          \
            }                                                                                              \
        }
        for (;;) {
            TR_STEP(wa, wb, wd, gA, sA, gB, sB)
            TR_STEP(wb, wc, wa, gB, sB, gA, sA)
            TR_STEP(wc, wd, wb, gA, sA, gB, sB)
            TR_STEP(wd, wa, wc, gB, sB, gA, sA)
        }
#undef TR_STEP
    tr_done:;
    }
    // the hot ops' accumulators: a wave sum each (integers), one LDS add
    if (k_first < ke)
#pragma unroll
        for (int h = 0; h < HN; ++h)
            if (h < H.n) {
                unsigned long long a = H.acc[h];
#pragma unroll
                for (int m = WAVE / 2; m >= 1; m >>= 1) a += (unsigned long long)__shfl_xor((long long)a, m, WAVE);
                if (lane == 0) atomicAdd(&lacc[G.hop[h]], a);
            }
    return rmax;
}

// The call-graph term alpha (P_ss s_k)[o] / M_s(k) of k_fx_b (pagerank.py:122-124), computed in
// k_tr_a instead: block lb owns the columns [lb N / n_fa, (lb + 1) N / n_fa), and every wave that
// has finished its walk takes chunks of 64 of them (an LDS counter) -- the chains of dependent
// loads (ss_off -> ss_par -> pw, s_k) then run in the slack of the block's slowest wave, not in
// k_fx_b's critical path.  The same arithmetic as k_fx_b (a lane per column of <= 8 parents with
// wave_sum's butterfly value, a wave per column of more): fx_ssv[o], read there bitwise.
// (pf: s_k from the block's LDS copy spl -- this launch computed it -- and the terms into buffer
// it & 1 of fx_ssv, read by the next launch's prologue or the final k_fx_b)
__device__ __forceinline__ void tr_ssv_share(const GDev& G, int32_t lb, int cur, double Ms, int* ctr, int lane,
                                             const double* spl = nullptr, int64_t ssv_off = 0) {
    const int32_t N = G.N;
    const int32_t oa = (int32_t)((int64_t)lb * N / G.n_fa), ob = (int32_t)((int64_t)(lb + 1) * N / G.n_fa);
    for (;;) {
        int c = 0;
        if (lane == 0) c = atomicAdd(ctr, WAVE);
        c = __builtin_amdgcn_readfirstlane(c);
        if (oa + c >= ob) return;
        const int32_t o = oa + c + lane;
        const bool on = o < ob;
        const int32_t op = on && G.perm ? G.perm[o] : o;
        const GLB int64_t* ss_off = gp(G.ss_off);
        const GLB int32_t* ss_par = gp(G.ss_par);
        const GLB float* pw = gp(G.pw);
        const GLB double* spg = gp(G.spb[cur]);
        auto sp = [&](int32_t p) -> double { return spl ? spl[p] : spg[p]; };
        double ssv = 0.0;
        bool big = false;
        if (on) {
            const int64_t e0 = ss_off[op], e1 = ss_off[op + 1];
            if (e1 - e0 <= 8) {
                int32_t pp[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) pp[k] = e0 + k < e1 ? ss_par[e0 + k] : -1;
                double t[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) t[k] = pp[k] >= 0 ? (double)pw[pp[k]] * sp(pp[k]) : 0.0;
                const double bb = ((t[0] + t[4]) + (t[2] + t[6])) + ((t[1] + t[5]) + (t[3] + t[7]));
                ssv = G.alpha * (bb / Ms);
            } else {
                big = true;
            }
        }
        for (uint64_t bm = __ballot(big); bm; bm &= bm - 1) {   // (wave-uniform)
            const int j = __ffsll((unsigned long long)bm) - 1;
            const int32_t opj = G.perm ? G.perm[oa + c + j] : oa + c + j;
            const int64_t e0 = ss_off[opj], e1 = ss_off[opj + 1];
            double bb = 0.0;
            for (int64_t e = e0 + lane; e < e1; e += WAVE) {
                const int32_t pp = ss_par[e];
                bb += (double)pw[pp] * sp(pp);
            }
            bb = wave_sum(bb);
            if (lane == j) ssv = G.alpha * (bb / Ms);
        }
        if (on) {
            if (G.lastfin)   // (write-through: the graph's last block reads it with sc1 loads)
                __hip_atomic_store(gpw((unsigned long long*)G.fx_ssv) + o, (unsigned long long)__double_as_longlong(ssv),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else
                G.fx_ssv[ssv_off + o] = ssv;
        }
    }
}

// The last k_tr_a block of a graph finishes the iteration itself (small graphs: window batches),
// so an iteration is ONE launch instead of k_tr_a + k_fx_b.  Every block writes its partial row
// and its call-graph terms write-through (sc1, hipMalloc'd pool memory), every wave waits for its
// stores (vmcnt(0)), and behind a workgroup barrier one lane takes a ticket from the graph's
// counter (an agent-scope add, returned); the block whose ticket completes the iteration's count is
// the consumer: it reads every row and does k_fx_b's work for every op -- the same exact limb sums,
// the same call-graph term (a lane per op of <= 8 parents, a wave per op of more: wave_sum's
// butterfly) and the same finish: bitwise k_fx_b's results.  Two forms of the hand-off
// (MI355X_MICROARCH.md, inter-workgroup visibility):
//  * a launch of at most one block per CU (<= num_cus blocks, the dynamic LDS padded past half a
//    CU's 160 KB so no two blocks share a CU: single windows) is the hand-off table's row 1 in
//    every cell -- one lane per storing workgroup adds to ONE unsharded counter, the last adder
//    told by the returned value, the other waves behind a barrier it joins, hipMalloc, one
//    workgroup per CU, 8-B sc1 stores and sc1 loads: no acquire (lf_acq 0);
//  * any other launch (batches: several workgroups per CU) takes the guide's general consumer
//    form: ONE agent acquire on the adding lane, its own vmcnt(0) wait, a workgroup barrier, then
//    the loads (lf_acq 1).  Only the finishing block pays it.
template <int NT>
__device__ __forceinline__ void tr_last_finish(const GDev& G, int it, double d, double Ms,
                                            GLB unsigned long long* Mnext) {
    constexpr int NW = NT / WAVE;
    __shared__ int s_last;
    const int32_t tid = (int32_t)threadIdx.x, lane = tid & (WAVE - 1), wv = tid / WAVE;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's row stores are out
    __syncthreads();
    if (tid == 0) {
        const unsigned long long t = __hip_atomic_fetch_add(gpw(G.mslot) + 6 * MSH + 1, 1ull, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
        const bool last = t + 1 == (unsigned long long)G.n_fa * (unsigned long long)(it + 1);
        if (last && G.lf_acq) {   // consumer: agent acquire (this CU's L1 invalidated), waited before the barrier
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    const int32_t N = G.N, nb = G.n_fa, nxt = (it & 1) ^ 1;
    const GLB unsigned long long* rows = gp((const unsigned long long*)G.fx_part);
    const GLB double* sp_cur = gp(G.spb[it & 1]);
    const GLB int64_t* ss_off = gp(G.ss_off);
    const GLB int32_t* ss_par = gp(G.ss_par);
    const GLB float* pw = gp(G.pw);
    const GLB float* u_o = gp(G.u_o);
    const double iscale = G.dscale ? G.dscale[1] : G.fx_iscale;
    for (int32_t ob = wv * WAVE; ob < N; ob += NW * WAVE) {   // lane = op
        const int32_t o = ob + lane;
        const bool on = o < N;
        unsigned long long lo = 0ull, hi = 0ull;
        // 16 rows per batch, every load in flight before the sums (indices clamped; repeats not added)
        const int32_t oc = on ? o : N - 1;
        for (int32_t b0 = 0; b0 < nb; b0 += 16) {
            unsigned long long v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                v[k] = __hip_atomic_load(rows + (size_t)min(b0 + k, nb - 1) * N + oc, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (b0 + k < nb) {
                    lo += v[k] & 0xffffffffull;
                    hi += v[k] >> 32;
                }
        }
        double ssv = 0.0;
        bool big = false;
        if (on && G.ssv_pre) {   // every block computed its share of the terms (tr_ssv_share): one load
            ssv = __longlong_as_double((long long)__hip_atomic_load(gp((const unsigned long long*)G.fx_ssv) + o,
                                                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        } else if (on) {
            const int64_t e0 = ss_off[o], e1 = ss_off[o + 1];
            if (e1 - e0 <= 8) {
                int32_t pp[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) pp[k] = e0 + k < e1 ? ss_par[e0 + k] : -1;
                double t[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) t[k] = pp[k] >= 0 ? (double)pw[pp[k]] * sp_cur[pp[k]] : 0.0;
                const double bb = ((t[0] + t[4]) + (t[2] + t[6])) + ((t[1] + t[5]) + (t[3] + t[7]));
                ssv = G.alpha * (bb / Ms);
            } else {
                big = true;
            }
        }
        for (uint64_t bm = __ballot(big); bm; bm &= bm - 1) {   // (wave-uniform)
            const int j = __ffsll((unsigned long long)bm) - 1;
            const int32_t oj = ob + j;
            const int64_t e0 = ss_off[oj], e1 = ss_off[oj + 1];
            double bb = 0.0;
            for (int64_t e = e0 + lane; e < e1; e += WAVE) {
                const int32_t pp = ss_par[e];
                bb += (double)pw[pp] * sp_cur[pp];
            }
            bb = wave_sum(bb);
            if (lane == j) ssv = G.alpha * (bb / Ms);
        }
        if (on) {
            const double sum = ((double)hi * 4294967296.0 + (double)lo) * iscale;
            const double v = d * (sum + ssv);   // pagerank.py:122-124
            G.spb[nxt][o] = v;
            G.sub[nxt][o] = (double)u_o[o] * v;
            atomicMax((unsigned long long*)&Mnext[o % MSH], d2bits(v));
        }
    }
}

#ifndef MR_TR_WPE512
#define MR_TR_WPE512 8   // minimum waves per SIMD asked of the plain 512-thread k_tr_a (A/B builds: 1)
#endif
template <class Q, int SUM, int NT, int EXT>
__global__ void __launch_bounds__(NT, NT == 512 && EXT == 0 && SUM != WV_SU_HOT ? MR_TR_WPE512 : 1) k_tr_a(const GDev* __restrict__ gs, int32_t ng, int32_t split, double d,
                                             double alpha, int it, int32_t unused) {
    constexpr bool SUL = SUM == WV_SU_ALL, HOT = SUM == WV_SU_HOT;
    constexpr int NW = NT / WAVE;
    extern __shared__ __attribute__((aligned(16))) unsigned char lraw[];
    __shared__ double red[NW];
    __shared__ double msh[2];
    const GDev& G = gs[fx_graph(gs, ng, split, 2)];
    const int32_t lb = (int32_t)blockIdx.x - G.blk0f;
    const int cur = it & 1, nxt = cur ^ 1, k3 = it % 3;
    const int32_t N = G.NA;   // (wide graphs: the hot ops)
    const int32_t tid = (int32_t)threadIdx.x;
    // pf (window batches, 512-thread variant): k_fx_b's finish of the previous iteration runs here,
    // in every block of the graph (below), so an iteration is one launch
    const bool pf = NT == 512 && SUL && EXT == 0 && G.pf;
    constexpr bool W32 = (EXT & 8) != 0;   // (fp32 wide graphs: float su, warm labels in LDS)
    using SU = TrSu<Q, EXT>;
    const TrLds L_(N, SUM, pf, W32);
    const int32_t NH = HOT ? G.n_hot : 0;   // <= L_.n_hot (the host sizes both alike), >= 64
    const GLB double* sug = gp(G.sub[cur]);   // ids >= N are pads (su 0)
    SU* su_l = (SU*)(lraw + L_.su);
    double* sp_l = (double*)(lraw + L_.sp);   // (pf) s_it itself, for the call-graph terms
    unsigned long long* lacc = (unsigned long long*)(lraw + L_.lacc);
    GLB unsigned long long* mslot = gpw(G.mslot);
    GLB unsigned long long* Mcur = mslot + (size_t)2 * MSH * k3;
    GLB unsigned long long* Mnext = mslot + (size_t)2 * MSH * ((k3 + 1) % 3);
    if (lb == 0 && tid < 2 * MSH) mslot[(size_t)2 * MSH * ((k3 + 2) % 3) + tid] = 0ull;
    double pf_max = -__builtin_huge_val();
    if (pf && it > 0) {
        // s_it[o] = d (S_o 2^-SC + alpha (P_ss s_{it-1})[o] / M_s(it-1)) from the previous launch's
        // partial rows and call-graph terms (buffers (it - 1) & 1): k_fx_b's exact limb sums and its
        // expression, so bitwise k_fx_b's values; every block of the graph computes all N of them
        // (a few rows each) -- block 0 also publishes s_it and M_s(it) for the final k_fx_b
        const int pb = (it - 1) & 1;
        const GLB unsigned long long* rows = gp((const unsigned long long*)G.fx_part) + (size_t)pb * G.pf_stride;
        const GLB double* ssvp = gp(G.fx_ssv) + (size_t)pb * N;
        const GLB float* u_o = gp(G.u_o);
        const double iscale = G.dscale ? G.dscale[1] : G.fx_iscale;
        const int32_t nb = G.n_fa;
        GLB double* spo = gpw(G.spb[cur]);
        for (int32_t o = tid; o < N + TR_PAD; o += NT) {
            if (o < N) {
                unsigned long long lo = 0ull, hi = 0ull;
                for (int32_t b = 0; b < nb; ++b) {
                    const unsigned long long v = rows[(size_t)b * N + o];
                    lo += v & 0xffffffffull;
                    hi += v >> 32;
                }
                const double sum = ((double)hi * 4294967296.0 + (double)lo) * iscale;
                const double v = d * (sum + ssvp[o]);   // pagerank.py:122-124
                sp_l[o] = v;
                su_l[o] = (double)u_o[o] * v;
                pf_max = nmax(pf_max, v);
                if (lb == 0) {
                    spo[o] = v;
                    atomicMax((unsigned long long*)&Mcur[o % MSH], d2bits(v));
                }
            } else {
                su_l[o] = 0.0;
                sp_l[o] = 0.0;
            }
        }
    } else if (W32) {   // hot ops, 64 zero pads, then the warm labels N .. ns_warm - 1
        const int32_t nw = G.ns_warm - N;
        for (int32_t o = tid; o < N + TR_PAD + nw; o += NT)
            su_l[o] = (SU)(o < N ? sug[o] : o < N + TR_PAD ? 0.0 : sug[o - TR_PAD]);
    } else if (SUL) {
        for (int32_t o = tid; o < N + TR_PAD; o += NT) su_l[o] = o < N ? sug[o] : 0.0;
        if (pf)
            for (int32_t o = tid; o < N + TR_PAD; o += NT) sp_l[o] = o < N ? G.spb[cur][o] : 0.0;
    }
    for (int32_t o = tid; o < N + TR_PAD; o += NT) lacc[o] = 0ull;
    if (HOT)
        for (int32_t o = tid; o < NH; o += NT) su_l[o] = sug[o];
    __shared__ int s_ssv;   // the call-graph term chunks taken (G.ssv_pre)
    if (tid < WAVE) {
        const double ms = wave_max(bits2d(Mcur[tid]));
        const double mr = wave_max(bits2d(Mcur[MSH + tid]));
        if (tid == 0) {
            msh[0] = ms;
            msh[1] = mr;
            s_ssv = 0;
        }
    }
    __syncthreads();   // accumulator and maxima ready
    if (pf && it > 0) {   // M_s(it): the maximum of the s_it just computed (block_max synchronises)
        const double m = block_max(pf_max, red);
        if (tid == 0) msh[0] = m;
        __syncthreads();
    }
    // hot ops (large graphs: the 1024-thread variant only) -- the mask sums of this iteration's su
    constexpr bool HOTT = SUL && NT == 1024;
    double* hs = (double*)(lraw + L_.hs);
    if (HOTT && L_.hot_ok && G.nhr) {
        tr_hot_sums(G, su_l, hs, tid);
        __syncthreads();
    }
    const double xsc = (G.dscale ? G.dscale[0] : G.fx_scale) / msh[1], Ms = msh[0];
    const double rmax_w = tr_walk<Q, SUM, NT, EXT, HOTT>(G, lb, cur, nxt, N, NH, d, Ms, xsc, su_l, lacc, hs);
    // the call-graph terms of this block's share of the columns, by the waves done walking
    if (G.ssv_pre) tr_ssv_share(G, lb, cur, Ms, &s_ssv, tid & (WAVE - 1), pf ? sp_l : nullptr, pf ? (int64_t)cur * N : 0);
    __syncthreads();
    GLB unsigned long long* prow = gpw(G.fx_part) + (pf ? (size_t)cur * G.pf_stride : 0) + (size_t)lb * N;
    if constexpr (NT == 512) {   // (window-graph variant only: the large graphs' kernel stays as it is)
        if (G.lastfin) {
            for (int32_t o = tid; o < N; o += NT)   // write-through: the last block reads them with sc1 loads
                __hip_atomic_store(prow + o, lacc[o], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const double rmax = block_max(rmax_w, red);
            if (tid == 0 && rmax >= 0.0) atomicMax((unsigned long long*)&Mnext[MSH + blockIdx.x % MSH], d2bits(rmax));
            tr_last_finish<NT>(G, it, d, Ms, Mnext);
            return;
        }
    }
    if (G.row_wt)   // write-through (sc1): the boundary to k_fx_b has no dirty lines to write back
        for (int32_t o = tid; o < N; o += NT)
            __hip_atomic_store(prow + o, lacc[o], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        for (int32_t o = tid; o < N; o += NT) prow[o] = lacc[o];
    const double rmax = block_max(rmax_w, red);
    if (tid == 0 && rmax >= 0.0)   // -inf: a block without traces (an empty shard's placeholder)
        atomicMax((unsigned long long*)&Mnext[MSH + blockIdx.x % MSH], d2bits(rmax));
}

// Column sums of the partial rows: a block per chunk of FB_OPS consecutive ops (lane = op, so
// every row read is one coalesced 512-B segment), its FB_W waves splitting the rows; the waves'
// limb sums meet in LDS (integers: order-free).  mode 0: whole graph; sharded graphs split it
// around the limb all-reduce: mode 1 writes this rank's limbs (lo, hi) per op to fx_limb, mode 2
// finishes from the reduced limbs.
// FB_W waves per block: 16 for graphs with many partial rows (a large graph alone: ~1k rows per
// op), 4 when every graph of the launch has few (batched window graphs: tens of rows) -- the block
// is then latency-bound (ss term, rows, LDS meet: a chain of dependent loads), and 4-wave blocks
// put the whole grid on the chip in one round instead of several.
constexpr int FB_W = 16, FB_W_SMALL = 4, FB_SMALL_ROWS = 256;
// ops per k_fx_b block: a lane reads op (lane % ops) of every (64/ops)-th row of its wave's share,
// so a row read stays one 128-B line per op group while small graphs still spread over many CUs
// A batch of many small graphs (C2 / C3 window groups: thousands of 16-op blocks, several rounds
// of the chip) takes 64 ops per block instead: lane = op, one row group per wave -- the same
// integer limb sums and call-graph terms, so bitwise the same results.  MR_FB_OPS: force 16 / 32 /
// 64 (read per call: tests)
static int fb_ops(int32_t N, bool many) {
    const char* e = getenv("MR_FB_OPS");
    const int force = e ? atoi(e) : 0;
    if (force == 16 || force == 32 || force == 64) return force;
    // (> 8192 ops: 64 measured ahead of 32 -- C4 140.0 -> 137.8 us per iteration, its rank-0-of-8
    // share 43.6 -> 41.5 us, C5 2.97 -> 2.94 ms; profiles/r05/r05q_fb_ops64_ab.txt)
    return N <= 8192 ? (many ? 64 : 16) : 64;
}
constexpr int64_t FB_MANY_BLOCKS = 1024;   // 16-op blocks of a launch from which "many" holds
constexpr int64_t LASTFIN_WORDS = 32768;
constexpr int32_t PF_NMAX = 1024;   // pf launches: ops per graph (three N-word LDS arrays per block)
constexpr int64_t PF_ROWS = 32;     // pf launches: partial rows per graph every block of it sums (C3 windows: up to 19)
#ifndef MR_LF_ONE_CU_LDS
#define MR_LF_ONE_CU_LDS (80 * 1024 + 1024)   // (A/B builds: 0 = every last-block launch takes the acquire)
#endif
constexpr size_t LF_ONE_CU_LDS = MR_LF_ONE_CU_LDS;   // > half of a CU's 160 KB: one block per CU   // k_tr_a's last-block finish: partial-row words it reads (256 KB)
// px.peers (sharded graphs on the peer path, one graph per launch): the exchange is fused in --
// mode 1 pushes the block's limbs (and block 0 this rank's r' maximum) into every rank's slot for
// this rank and stores the round number in the block's flag there; mode 2 block b waits for flag
// (src, b) of every source (px.spin; else k_peer_bwait waited before the launch) and sums the R
// slots in rank order.  Bitwise the all-reduce path: the same integers summed.
template <int FB_W>
__global__ void __launch_bounds__(WAVE * FB_W) k_fx_b(const GDev* __restrict__ gs, int32_t ng, int32_t split,
                                                     double d, int it, int mode, const MrPeerX px) {
    __shared__ unsigned long long slo[FB_W * WAVE], shi[FB_W * WAVE];
    __shared__ double lssv[WAVE];
    __shared__ int s_ok;
    const GDev& G = gs[fx_graph(gs, ng, split, 3)];
    const bool pxo = px.peers != nullptr;   // (uniform)
    const GLB unsigned long long* preg = (const GLB unsigned long long*)px.region;
    const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    const int32_t OPB = G.fb_ops, GR = WAVE / OPB;
    const int32_t ol = lane % OPB, grp = lane / OPB;
    // o: the column (the fused kernel's op label); op: the graph's op (perm: relabelled graphs)
    const int32_t o0 = ((int32_t)blockIdx.x - G.blk0fb) * OPB;
    const int32_t o = o0 + ol;
    const int32_t N = G.N, nb = G.n_fa;
    const bool on = o < N;
    const int k3c = it % 3;
    // the op's rows: k_tr_a's (stride NA), or on a wide graph its cold range's (stride cold_rw).
    // The first batch of 16 rows per lane is issued before the call-graph term below, so the two
    // chains of dependent loads overlap (window graphs: tens of rows, one batch covers them)
    const int32_t stride = FB_W * GR;
    const GLB unsigned long long* col = gp((const unsigned long long*)G.fx_part);
    int32_t nbl = 0;
    size_t rs = 1;
    if (on && mode != 2) {
        if (o < G.NA) {   // (pf graphs: the final iteration's rows, buffer it & 1)
            col = gp((const unsigned long long*)G.fx_part) + (G.pf ? (size_t)(it & 1) * G.pf_stride : 0) + o;
            nbl = nb;
            rs = (size_t)G.NA;
        } else {
            const int32_t oc = o - G.NA, r = oc / G.cold_rw, rb0 = G.cold_rowbase[r];
            nbl = G.cold_rowbase[r + 1] - rb0;
            col = gp(G.cold_part) + (size_t)rb0 * G.cold_rw + (oc - r * G.cold_rw);
            rs = (size_t)G.cold_rw;
        }
    }
    const int32_t rfirst = w * GR + grp;
    unsigned long long v0[16];
    if (nbl > 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) v0[k] = col[(size_t)min(rfirst + k * stride, nbl - 1) * rs];
    }
    // the call-graph term alpha (P_ss s_k)[op] / M_s(k) (pagerank.py:122-124) of the block's ops: a
    // wave per op, its lanes striding the op's parents, one fixed-order wave sum (a hub op with
    // thousands of parents costs one wave, not one thread).  (Not in mode 1: its sums only.)
    // ssv_pre: k_tr_a computed them (tr_ssv_share) -- one coalesced load
    if (mode != 1 && G.ssv_pre) {
        if (threadIdx.x < (unsigned)OPB)
            lssv[threadIdx.x] = o0 + (int32_t)threadIdx.x < N ? G.fx_ssv[(G.pf ? (size_t)(it & 1) * N : 0) + o0 + threadIdx.x] : 0.0;
    } else if (mode != 1) {
        const double Ms = wave_max(bits2d(G.mslot[(size_t)2 * MSH * k3c + lane]));
        const GLB double* sp_cur = gp(G.spb[it & 1]);
        const GLB int64_t* ss_off = gp(G.ss_off);
        const GLB int32_t* ss_par = gp(G.ss_par);
        const GLB float* pw = gp(G.pw);
        // the wave's ops j = w, w + FB_W, ..: one lane each for ops of <= 8 parents -- the lane
        // forms the wave sum's value itself (the butterfly of wave_sum over 64 slots with the
        // terms in slots 0..7 and zeros elsewhere: adding +0.0 is exact, so only the pairs
        // (l, l+4), (l, l+2), (0, 1) round) -- all the wave's ops in one chain of loads instead
        // of one chain per op; ops with more parents take the wave path after them
        const int32_t nj = (OPB - w + FB_W - 1) / FB_W;
        bool big = false;
        if (lane < nj) {
            const int32_t j = w + lane * FB_W, oj = o0 + j;
            if (oj < N) {
                const int32_t opj = G.perm ? G.perm[oj] : oj;
                const int64_t e0 = ss_off[opj], e1 = ss_off[opj + 1];
                if (e1 - e0 <= 8) {
                    int32_t pp[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) pp[k] = e0 + k < e1 ? ss_par[e0 + k] : -1;
                    double t[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) t[k] = pp[k] >= 0 ? (double)pw[pp[k]] * sp_cur[pp[k]] : 0.0;
                    const double bb = ((t[0] + t[4]) + (t[2] + t[6])) + ((t[1] + t[5]) + (t[3] + t[7]));
                    lssv[j] = G.alpha * (bb / Ms);
                } else {
                    big = true;
                }
            }
        }
        for (uint64_t bm = __ballot(big); bm; bm &= bm - 1) {   // (wave-uniform)
            const int32_t j = w + (int32_t)(__ffsll((unsigned long long)bm) - 1) * FB_W, oj = o0 + j;
            const int32_t opj = G.perm ? G.perm[oj] : oj;
            const int64_t e0 = ss_off[opj], e1 = ss_off[opj + 1];
            double bb = 0.0;
            for (int64_t e = e0 + lane; e < e1; e += WAVE) {
                const int32_t pp = ss_par[e];
                bb += (double)pw[pp] * sp_cur[pp];
            }
            bb = wave_sum(bb);
            if (lane == 0) lssv[j] = G.alpha * (bb / Ms);
        }
    }
    // the finishing lanes' operands, loaded before the rows so both latencies overlap
    const bool fin = w == 0 && lane < OPB && on;
    const int32_t op = fin && G.perm ? G.perm[o] : o;
    const float uo = fin ? G.u_o[op] : 0.0f;
    const int32_t bidx = (int32_t)blockIdx.x - G.blk0fb;
    const size_t par = (size_t)(px.seq & 1) * (size_t)px.R;   // this round's slots: [par + src] x W words
    if (bidx == 0 && w == 1 && mode) {   // r' maxima riding on the limb sum
        unsigned long long* Mn = G.mslot + (size_t)2 * MSH * ((it % 3 + 1) % 3);
        if (!pxo) {
            if (mode == 1) rmax_put(G, Mn, G.fx_limb + 2 * (size_t)N, lane);
            else rmax_take_bits(G.fx_limb + 2 * (size_t)N, G.nranks, Mn, lane);
        } else if (mode == 1) {   // this rank's maximum into word 2N + rank of its slot on every rank
            const double m = wave_max(bits2d(Mn[MSH + lane]));
            if (lane < px.R)
                __hip_atomic_store((GLB unsigned long long*)px.peers[lane] + px.slots + (par + px.rank) * px.W +
                                       2 * (size_t)N + px.rank,
                                   d2bits(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if (pxo && mode == 2) {
        if (px.spin && threadIdx.x == 0) {   // flag (src, bidx) of every source: this round's words are in
            s_ok = 1;
            const unsigned long long need = px.seq + 1, t0 = __builtin_amdgcn_s_memrealtime();
            for (int r = 0; r < px.R && s_ok; ++r)
                while (__hip_atomic_load(preg + px.bflags + (int64_t)r * px.nbf + bidx, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM) < need) {
                    __builtin_amdgcn_s_sleep(2);
                    // a round that already timed out (this call's error word): stop at once instead
                    // of spinning the full timeout again in every later iteration
                    if (__builtin_amdgcn_s_memrealtime() - t0 > px.timeout ||
                        __hip_atomic_load(preg + px.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0ull) {
                        s_ok = 0;
                        __hip_atomic_store((GLB unsigned long long*)px.region + px.err, 1ull, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
                        break;
                    }
                }
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
        } else if (!px.spin && threadIdx.x == 0) {
            s_ok = 1;
        }
        __syncthreads();
        if (!s_ok) return;   // (the error word reports it; the host raises MR_ERR_COMM)
        if (bidx == 0 && w == 1) {   // every rank's r' maximum: word 2N + src of slot src
            unsigned long long b = 0ull;
            for (int j = lane; j < px.R; j += WAVE)
                b = max(b, __hip_atomic_load(preg + px.slots + (par + j) * px.W + 2 * (size_t)N + j, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM));
            const double m = wave_max(bits2d(b));
            if (lane == 0) atomicMax(&G.mslot[(size_t)2 * MSH * ((it % 3 + 1) % 3) + MSH], d2bits(m));
        }
    }
    unsigned long long lo = 0ull, hi = 0ull;
    if (nbl > 0) {
        // the first batch (loaded above), then batches of 16 rows per lane, every load in flight
        // before the sums (indices clamped: the repeats are cache hits and are not added)
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (rfirst + k * stride < nbl) {
                lo += v0[k] & 0xffffffffull;
                hi += v0[k] >> 32;
            }
        for (int32_t r0 = rfirst + 16 * stride; r0 < nbl; r0 += 16 * stride) {
            unsigned long long v[16];
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = col[(size_t)min(r0 + k * stride, nbl - 1) * rs];
#pragma unroll
            for (int k = 0; k < 16; ++k)
                if (r0 + k * stride < nbl) {
                    lo += v[k] & 0xffffffffull;
                    hi += v[k] >> 32;
                }
        }
    }
    // the wave's row groups of one op meet by lane shuffles, the waves through LDS (integers:
    // order-free)
    for (int m = WAVE / 2; m >= OPB; m >>= 1) {
        lo += (unsigned long long)__shfl_xor((long long)lo, m);
        hi += (unsigned long long)__shfl_xor((long long)hi, m);
    }
    if (lane < OPB) {
        slo[w * WAVE + lane] = lo;
        shi[w * WAVE + lane] = hi;
    }
    __syncthreads();
    if (pxo && mode == 1) {   // push the block's limbs to every rank, then the block's flag there
        if (fin) {
            lo = hi = 0ull;
            for (int k = 0; k < FB_W; ++k) {
                lo += slo[k * WAVE + lane];
                hi += shi[k * WAVE + lane];
            }
            for (int r = 0; r < px.R; ++r) {
                GLB unsigned long long* dst = (GLB unsigned long long*)px.peers[r] + px.slots + (par + px.rank) * px.W;
                __hip_atomic_store(dst + 2 * op, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(dst + 2 * op + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (every wave: the r' word of wave 1 too)
        __syncthreads();
        if ((int32_t)threadIdx.x < px.R && !px.mute) {
            __atomic_thread_fence(__ATOMIC_RELEASE);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store((GLB unsigned long long*)px.peers[threadIdx.x] + px.bflags + (int64_t)px.rank * px.nbf + bidx,
                               (unsigned long long)(px.seq + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    if (!fin) return;
    lo = hi = 0ull;
    for (int k = 0; k < FB_W; ++k) {
        lo += slo[k * WAVE + lane];
        hi += shi[k * WAVE + lane];
    }
    if (mode == 1) {
        G.fx_limb[2 * op] = lo;
        G.fx_limb[2 * op + 1] = hi;
        return;
    }
    if (mode == 2 && pxo) {   // the R slots in rank order (integers: the all-reduce's sum)
        lo = hi = 0ull;
        for (int r = 0; r < px.R; ++r) {
            const GLB unsigned long long* sl = preg + px.slots + (par + r) * px.W;
            lo += __hip_atomic_load(sl + 2 * op, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            hi += __hip_atomic_load(sl + 2 * op + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    } else if (mode == 2) {
        lo = G.fx_limb[2 * op];
        hi = G.fx_limb[2 * op + 1];
    }
    const int nxt = (it & 1) ^ 1, k3 = it % 3;
    unsigned long long* Mnext = G.mslot + (size_t)2 * MSH * ((k3 + 1) % 3);
    const double ssv = lssv[lane];   // (written before the barrier above)
    // hi, lo < 2^53 (fewer than 2^21 rows over all ranks): both conversions exact, one rounding
    const double sum = ((double)hi * 4294967296.0 + (double)lo) * (o < G.NA ? (G.dscale ? G.dscale[1] : G.fx_iscale) : G.cx_iscale);
    const double v = d * (sum + ssv);      // pagerank.py:122-124
    G.spb[nxt][op] = v;
    const double su = (double)uo * v;
    if (G.su32) {   // (fp32 wide graphs: rounded to float, kept both ways)
        const float f = (float)su;
        G.sub[nxt][o] = (double)f;
        G.suf[nxt][o] = f;
    } else {
        G.sub[nxt][o] = su;   // su in the kernel's labels
    }
    atomicMax(&Mnext[op % MSH], d2bits(v));
}

// ---- wide fused graphs, per iteration, before k_tr_a
// cold half of each trace's su sum (pagerank.py:125), in position order: k_tr_a adds it to the
// lane's hot sum before the division by M_s(k)
// (over the listed wave tiles only: the long tiles of the general walk and the short tiles with
// more than two cold chunks -- the short-tile walk gathers the rest itself)
__global__ void k_cold_trace(const int32_t* __restrict__ coff, const int32_t* __restrict__ cops,
                             const double* __restrict__ su, const int32_t* __restrict__ tiles, int32_t ntl, int32_t T,
                             double* __restrict__ cacc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)ntl * WAVE) return;
    const int32_t p = tiles[i / WAVE] * WAVE + (int32_t)(i % WAVE);
    if (p >= T) return;
    const int32_t a = coff[p], b = coff[p + 1];
    double acc = 0.0;
    int32_t j = a;
    for (; j + 4 <= b; j += 4) {
        const int32_t o0 = cops[j], o1 = cops[j + 1], o2 = cops[j + 2], o3 = cops[j + 3];
        const double v0 = su[o0], v1 = su[o1], v2 = su[o2], v3 = su[o3];
        acc += v0;
        acc += v1;
        acc += v2;
        acc += v3;
    }
    for (; j < b; ++j) acc += su[cops[j]];
    cacc[p] = acc;
}
// cold half of P_sr r (pagerank.py:122-124): a block per slice of one range's (position, op)
// pairs, X = rint(q_k[p] / M_r(k) * 2^SCc) added into the range's LDS accumulator; the block's row
// goes out whole (k_fx_b sums a range's rows like k_tr_a's).  SCc leaves no overflow: an op gets
// at most one add per position of the slice (SCc = 64 - bits(widest slice span)).
template <class Q>
__global__ void __launch_bounds__(WIDE_CT) k_cold_ops(const int64_t* __restrict__ cb_beg, const int32_t* __restrict__ cp_pos,
                                                     const uint16_t* __restrict__ cp_op, const void* qv,
                                                     const unsigned long long* mslot, int it, double cx_scale,
                                                     int32_t RW, unsigned long long* __restrict__ cold_part) {
    extern __shared__ unsigned long long cacc_l[];
    __shared__ double mr;
    const Q* __restrict__ q = (const Q*)qv;
    const int k3 = it % 3;
    for (int32_t i = threadIdx.x; i < RW; i += WIDE_CT) cacc_l[i] = 0ull;
    if (threadIdx.x < WAVE) {
        const double m = wave_max(bits2d(mslot[(size_t)2 * MSH * k3 + MSH + threadIdx.x]));
        if (threadIdx.x == 0) mr = m;
    }
    __syncthreads();
    const double xsc = cx_scale / mr;
    const int64_t b = cb_beg[blockIdx.x], e = cb_beg[blockIdx.x + 1];
    int64_t i = b + threadIdx.x;
    for (; i + 3 * WIDE_CT < e; i += 4 * WIDE_CT) {   // four pairs in flight per thread
        int32_t p[4];
        uint16_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            p[j] = cp_pos[i + j * WIDE_CT];
            o[j] = cp_op[i + j * WIDE_CT];
        }
        double v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (double)q[p[j]];
#pragma unroll
        for (int j = 0; j < 4; ++j) atomicAdd(&cacc_l[o[j]], (unsigned long long)__double2ull_rn(v[j] * xsc));
    }
    for (; i < e; i += WIDE_CT) atomicAdd(&cacc_l[cp_op[i]], (unsigned long long)__double2ull_rn((double)q[cp_pos[i]] * xsc));
    __syncthreads();
    unsigned long long* row = cold_part + (size_t)blockIdx.x * RW;
    for (int32_t o = threadIdx.x; o < RW; o += WIDE_CT) row[o] = cacc_l[o];
}

// result = s/max(s) (pagerank.py:126,129); weight = result * sum(result) / N (:93-107)
__global__ void __launch_bounds__(1024) k_weights(const double* sp, const unsigned long long* mslot, int k3,
                                                  int32_t N, int exact, double* sn, double* weight, double* scal) {
    __shared__ double red[1024 / WAVE];
    __shared__ double tot;
    double ms = -__builtin_huge_val();
    for (int i = threadIdx.x; i < MSH; i += blockDim.x) ms = nmax(ms, bits2d(mslot[(size_t)2 * MSH * k3 + i]));
    const double Ms = block_max(ms, red);
    double m = -__builtin_huge_val();
    for (int32_t o = threadIdx.x; o < N; o += blockDim.x) {
        double v = sp[o] / Ms;
        sn[o] = v;
        m = nmax(m, v);
    }
    m = block_max(m, red);
    for (int32_t o = threadIdx.x; o < N; o += blockDim.x) sn[o] = sn[o] / m;
    __syncthreads();
    if (exact) {
        if (threadIdx.x == 0) {
            double s = 0.0;
            for (int32_t o = 0; o < N; ++o) s += sn[o];
            tot = s;
        }
        __syncthreads();
    } else {
        int32_t per = (N + blockDim.x - 1) / blockDim.x;
        int32_t a = threadIdx.x * per, b = min(a + per, N);
        double s = 0.0;
        for (int32_t o = a; o < b; ++o) s += sn[o];
        s = block_sum(s, red);
        if (threadIdx.x == 0) tot = s;
        __syncthreads();
    }
    const double total = tot;
    for (int32_t o = threadIdx.x; o < N; o += blockDim.x) weight[o] = sn[o] * total / (double)N;
    if (threadIdx.x == 0) scal[4] = total;
}
// k_weights for every graph of a batch (block g: graph g) plus a gather of each graph's four error
// words into one buffer, so the call's single read-back is one pinned copy
__global__ void __launch_bounds__(1024) k_weights_batch(const GDev* __restrict__ gs, int iters, int exact,
                                                        int32_t* flags_out) {
    const GDev& G = gs[blockIdx.x];
    if (threadIdx.x < 4) flags_out[4 * blockIdx.x + threadIdx.x] = G.flag[threadIdx.x];
    __shared__ double red[1024 / WAVE];
    __shared__ double tot;
    const double* sp = G.spb[iters & 1];
    const int k3 = iters % 3;
    const int32_t N = G.N;
    double* sn = G.sn;
    double ms = -__builtin_huge_val();
    for (int i = threadIdx.x; i < MSH; i += blockDim.x) ms = nmax(ms, bits2d(G.mslot[(size_t)2 * MSH * k3 + i]));
    const double Ms = block_max(ms, red);
    double m = -__builtin_huge_val();
    for (int32_t o = threadIdx.x; o < N; o += blockDim.x) {
        double v = sp[o] / Ms;
        sn[o] = v;
        m = nmax(m, v);
    }
    m = block_max(m, red);
    for (int32_t o = threadIdx.x; o < N; o += blockDim.x) sn[o] = sn[o] / m;
    __syncthreads();
    if (exact) {
        if (threadIdx.x == 0) {
            double s = 0.0;
            for (int32_t o = 0; o < N; ++o) s += sn[o];
            tot = s;
        }
        __syncthreads();
    } else {
        int32_t per = (N + blockDim.x - 1) / blockDim.x;
        int32_t a = threadIdx.x * per, b = min(a + per, N);
        double s = 0.0;
        for (int32_t o = a; o < b; ++o) s += sn[o];
        s = block_sum(s, red);
        if (threadIdx.x == 0) tot = s;
        __syncthreads();
    }
    const double total = tot;
    for (int32_t o = threadIdx.x; o < N; o += blockDim.x) G.weight[o] = sn[o] * total / (double)N;
    if (threadIdx.x == 0) G.scal[4] = total;
}
// ---------------------------------------------------------------- trace-sharded graphs
// local call edges (child, parent) as sort keys c << nb | p
__global__ void k_sh_edge_keys(const int64_t* ss_off, const int32_t* ss_par, int32_t N, int nb, uint64_t* key) {
    const int32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= N) return;
    for (int64_t e = ss_off[c]; e < ss_off[c + 1]; ++e) key[e] = ((uint64_t)c << nb) | (uint32_t)ss_par[e];
}
__global__ void k_sh_pad(uint64_t* key, int64_t from, int64_t to, uint64_t pad) {
    const int64_t i = from + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < to) key[i] = pad;
}
// heads of distinct real keys in the sorted union (pads sort last and are dropped)
__global__ void k_sh_edge_heads(const uint64_t* key, int64_t n, uint64_t pad, int32_t* head) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) head[i] = key[i] != pad && (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}
__global__ void k_sh_edge_out(const uint64_t* key, const int32_t* head, const int64_t* pos, int64_t n, int nb,
                              int32_t* ss_par, int32_t* ccount) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !head[i]) return;
    ss_par[pos[i]] = (int32_t)(key[i] & ((1ull << nb) - 1ull));
    atomicAdd(&ccount[(int32_t)(key[i] >> nb)], 1);
}
// this rank's kind classes as (key, check hash of the representative, count); empty slots skipped
__global__ void k_sh_kind_list(const unsigned long long* hk, const KCnt* cr, const uint64_t* hchk, int64_t cap, const int32_t* flag,
                               const int64_t* pos, uint64_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap || !flag[i]) return;
    const int64_t p = pos[i];
    out[3 * p] = hk[i];
    out[3 * p + 1] = hchk[i];   // k_kind_insert<true>: the representative's check hash
    out[3 * p + 2] = cr[i].cnt;
}
__global__ void k_sh_kind_flags(const unsigned long long* hk, int64_t cap, int32_t* flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cap) flag[i] = hk[i] != 0ull;
}
// all ranks' lists into one table: counts summed per key; a key whose check hash differs
// between ranks is a 64-bit collision across ranks -> flag
__global__ void k_sh_kind_merge(const uint64_t* in, int64_t n, uint64_t* gk, uint64_t* gh, unsigned long long* gc,
                                uint64_t mask, int32_t* flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t k = in[3 * i];
    if (!k) return;
    uint64_t s = mix64(k) & mask;
    for (;;) {
        const unsigned long long old = atomicCAS((unsigned long long*)&gk[s], 0ull, (unsigned long long)k);
        if (old == 0ull) {
            gh[s] = in[3 * i + 1];   // first writer; later writers compare after the table settles
            break;
        }
        if (old == k) break;
        s = (s + 1) & mask;
    }
    atomicAdd(&gc[s], (unsigned long long)in[3 * i + 2]);
}
__global__ void k_sh_kind_check(const uint64_t* in, int64_t n, const uint64_t* gk, const uint64_t* gh, uint64_t mask,
                                int32_t* flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !in[3 * i]) return;
    const uint64_t k = in[3 * i];
    uint64_t s = mix64(k) & mask;
    while (gk[s] != k) s = (s + 1) & mask;
    if (gh[s] != in[3 * i + 1]) atomicOr(flag, 1);
}
// ---- the kind-class exchange partitioned by key (peer regions): a class key is OWNED by rank
// owner(key); every rank sends its (key, check hash, count) records to their owners, each owner
// sums the counts of the keys it owns and returns every record's total to its sender
__device__ __forceinline__ int kind_owner(uint64_t key, int R) { return (int)((mix64(key ^ 0x5bd1e995ull) >> 33) % (uint64_t)R); }
__global__ void k_kx_count(const uint64_t* rec, int64_t n, int R, unsigned long long* cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) atomicAdd(&cnt[kind_owner(rec[3 * i], R)], 1ull);
}
// records by owner: record i -> send slot spos[i] (order inside an owner's run arbitrary: the
// owner's sums and the returned totals do not depend on it)
__global__ void k_kx_place(const uint64_t* rec, int64_t n, int R, unsigned long long* cursor, uint64_t* send,
                           int64_t* spos) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t p = (int64_t)atomicAdd(&cursor[kind_owner(rec[3 * i], R)], 1ull);
    send[3 * p] = rec[3 * i];
    send[3 * p + 1] = rec[3 * i + 1];
    send[3 * p + 2] = rec[3 * i + 2];
    spos[i] = p;
}
// the owner's totals back to the senders: received record j came from rank s (roff: first record of
// each source) and goes to slot soff_at_s + (j - roff[s]) of s's area B
__global__ void k_kx_return(const uint64_t* in, int64_t n, const uint64_t* gk, const unsigned long long* gc, uint64_t mask,
                            const int64_t* roff, const int64_t* dbase, int R, unsigned long long* const* areas) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t k = in[3 * j];
    uint64_t s = mix64(k) & mask;
    while (gk[s] != k) s = (s + 1) & mask;
    int src = 0;
    while (src + 1 < R && roff[src + 1] <= j) ++src;
    __hip_atomic_store((__attribute__((address_space(1))) unsigned long long*)areas[src] + dbase[src] + (j - roff[src]),
                       gc[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// kind[t] = the returned total of its class's record
__global__ void k_kx_apply(const unsigned long long* hk, const int32_t* slot_of, const int32_t* flag, const int64_t* pos,
                           const int64_t* spos, const unsigned long long* ret, int32_t T, double* kind) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const int32_t sl = slot_of[t];
    (void)hk;
    (void)flag;
    kind[t] = (double)ret[spos[pos[sl]]];
}
// kind[t] = the class size over all ranks
__global__ void k_sh_kind_apply(const unsigned long long* hk, const int32_t* slot_of, int32_t T, const uint64_t* gk,
                                const unsigned long long* gc, uint64_t mask, double* kind) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const uint64_t k = hk[slot_of[t]];
    uint64_t s = mix64(k) & mask;
    while (gk[s] != k) s = (s + 1) & mask;
    kind[t] = (double)gc[s];
}
}  // namespace

// ------------------------------------------------------------------------------ host side
// MR_DEBUG=1: check every launch (names the failing kernel instead of a later sticky error)
static const bool g_debug = getenv("MR_DEBUG") != nullptr;
#define MR_DEBUG_CHECK(ctx, name)                                                                          \
    do {                                                                                                   \
        if (g_debug) {                                                                                     \
            hipError_t e_ = hipGetLastError();                                                             \
            if (e_ == hipSuccess) e_ = hipStreamSynchronize((ctx)->stream);                                \
            if (e_ != hipSuccess) return mr_fail((ctx), MR_ERR_HIP, "%s: %s", name, hipGetErrorString(e_)); \
        }                                                                                                  \
    } while (0)

void mr_prof_begin(mr_ctx* ctx);
void mr_prof_end(mr_ctx* ctx, double bytes, int64_t iters = 1);

using TrA = void (*)(const GDev*, int32_t, int32_t, double, double, int, int32_t);
// ext: some graph of the launch carries kind multiplicities (bit 0: mw_tp) or a cold side (bit 1:
// wide graphs) -- only the short-tile walk of the su-in-LDS mode distinguishes them
static TrA tr_kernel(bool fp32, int mode, int NT, int ext = 0) {
    static const TrA tab[2][3][2] = {
        {{k_tr_a<double, 0, 512, 0>, k_tr_a<double, 0, 1024, 0>},
         {k_tr_a<double, 1, 512, 0>, k_tr_a<double, 1, 1024, 0>},
         {k_tr_a<double, 2, 512, 0>, k_tr_a<double, 2, 1024, 0>}},
        {{k_tr_a<float, 0, 512, 0>, k_tr_a<float, 0, 1024, 0>},
         {k_tr_a<float, 1, 512, 0>, k_tr_a<float, 1, 1024, 0>},
         {k_tr_a<float, 2, 512, 0>, k_tr_a<float, 2, 1024, 0>}}};
    static const TrA tab_ext[4][2][2] = {
        {{k_tr_a<double, 1, 512, 1>, k_tr_a<double, 1, 1024, 1>}, {k_tr_a<float, 1, 512, 1>, k_tr_a<float, 1, 1024, 1>}},
        {{k_tr_a<double, 1, 512, 2>, k_tr_a<double, 1, 1024, 2>}, {k_tr_a<float, 1, 512, 2>, k_tr_a<float, 1, 1024, 2>}},
        {{k_tr_a<double, 1, 512, 3>, k_tr_a<double, 1, 1024, 3>}, {k_tr_a<float, 1, 512, 3>, k_tr_a<float, 1, 1024, 3>}},
        {{k_tr_a<double, 1, 512, 4>, k_tr_a<double, 1, 1024, 4>}, {k_tr_a<float, 1, 512, 4>, k_tr_a<float, 1, 1024, 4>}}};
    // ext 10: fp32 wide graphs with float su and warm labels in LDS
    if (ext == 10 && fp32 && mode == WV_SU_ALL) return NT == 1024 ? k_tr_a<float, 1, 1024, 10> : k_tr_a<float, 1, 512, 10>;
    // ext 4: run-merged window graphs (trun; never beside multiplicities or cold sums)
    if (ext == 4 && mode == WV_SU_ALL) return tab_ext[3][fp32 ? 1 : 0][NT == 1024 ? 1 : 0];
    if ((ext & 3) && mode == WV_SU_ALL) return tab_ext[(ext & 3) - 1][fp32 ? 1 : 0][NT == 1024 ? 1 : 0];
    return tab[fp32 ? 1 : 0][mode][NT == 1024 ? 1 : 0];
}
static int num_cus() {
    static const int ncu = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            v = 256;
        return std::max(v, 1);
    }();
    return ncu;
}

// ops of the fused kernel's walk: a wide graph's hot ops, else all
static int32_t kern_n(const mr_graph* g) { return g->wide ? g->NA : g->N; }

// Launch plan of the fused iteration (k_tr_a) for a batch of graphs (one kernel variant per launch).
struct FxPlan {
    int NT = 1024;      // block size (16 waves; 512 when the graphs are small)
    int mode = WV_SU_ALL;   // su in LDS for every fused graph of the batch / hot ops / none
    bool sul = true;    // mode == WV_SU_ALL
    bool pf = false;    // window batches: the next launch finishes an iteration (k_tr_a's pf prologue)
    bool w32 = false;   // fp32 wide graphs only: float su and warm labels in LDS (k_tr_a EXT & 8)
};
static FxPlan fx_plan(mr_graph* const* gs, int ng) {
    FxPlan P;
    int32_t nmax = 0;
    int64_t tmax = 0;
    for (int i = 0; i < ng; ++i)
        if (gs[i]->fused) {
            nmax = std::max(nmax, kern_n(gs[i]));
            tmax = std::max<int64_t>(tmax, gs[i]->T);
        }
    // 1024-thread blocks when the largest graph has a wave tile for every wave of the chip (and
    // always for graphs with register-accumulated hot ops: only that variant carries them)
    P.NT = cdiv(tmax, WAVE) >= (int64_t)num_cus() * 16 ? 1024 : 512;
    for (int i = 0; i < ng; ++i)
        if (gs[i]->fused && gs[i]->nhr) P.NT = 1024;
    bool relabeled = false;
    for (int i = 0; i < ng; ++i) relabeled = relabeled || (gs[i]->fused && gs[i]->relabeled);
    P.sul = TrLds(nmax, WV_SU_ALL).su_lds;
    P.mode = P.sul ? WV_SU_ALL : relabeled ? WV_SU_HOT : WV_SU_GLOBAL;
    if (P.mode == WV_SU_HOT)   // every graph of the launch must be relabelled (hot ops = low labels)
        for (int i = 0; i < ng; ++i)
            if (gs[i]->fused && !gs[i]->relabeled) P.mode = WV_SU_GLOBAL;
    if (P.mode == WV_SU_HOT && TrLds(nmax, WV_SU_HOT).n_hot < 64) P.mode = WV_SU_GLOBAL;
    return P;
}
static int32_t plan_n_hot(int32_t N, const FxPlan& P) {
    return P.mode == WV_SU_HOT ? TrLds(N, WV_SU_HOT).n_hot : 0;
}
static size_t plan_lds(int32_t N, const FxPlan& P) { return TrLds(N, P.mode, P.pf, P.w32).total; }

// resident blocks of the plan's kernel on the chip (occupancy by LDS image and VGPRs)
static int64_t plan_resident(int32_t N, const FxPlan& P) {
    const size_t lds = plan_lds(N, P);
    // (cached per (mode, block size, LDS bytes): a window group asks for each of its 256 graphs)
    static std::mutex mu;
    static std::map<std::tuple<int, int, size_t>, int> cache;
    const auto key = std::make_tuple(P.mode, P.NT, lds);
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return (int64_t)num_cus() * it->second;
    }
    const TrA kfn = tr_kernel(false, P.mode, P.NT, 0);
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)kfn, P.NT, lds) != hipSuccess || n < 1)
        n = std::max<int>(1, (int)(WV_LDS_MAX / std::max<size_t>(lds, 1)));
    std::lock_guard<std::mutex> lk(mu);
    cache[key] = n;
    return (int64_t)num_cus() * n;
}

// k_tr_a: blocks of one graph and the cut of its tiles into contiguous per-wave runs of about
// equal cost (chunks + 2 per tile: a tile's q/r words weigh about two chunks).  Cached per
// graph for the wave count; at most 1023 tiles (65472 traces) per block.
// wsum: wave tiles of all fused graphs of the launch.  A graph of a batch gets its share of the
// resident blocks in proportion to its tiles: a small graph of a batch then runs a few blocks with
// several tiles per wave instead of one block per tile set -- the per-block fixed cost (LDS image,
// the N-word partial row written here and re-read by k_fx_b) falls with the block count while the
// batch still fills the chip.
// a tile's fixed cost in chunks for the per-wave cut: its q / r words and r' (about two chunks),
// plus the hot-op accumulators and mask sum on hot-op layouts (3: with 2 the waves of short hot
// tiles became a tail, C4 188 us per iteration)
static double tr_tile_weight(const mr_graph* g) { return g->nhr ? 3.0 : 2.0; }
// window graphs (layout order, ranked in batches whose groups cut them differently): the fixed-point
// scale from the graph's trace count -- a bound for any block of any cut -- instead of the cut's
// largest block (tr_cut_body); 0 for other graphs (the finest scale of their cut)
static int32_t tr_scfix(const mr_graph* g) {
    return g->lo ? 64 - bits_for((uint64_t)std::min<int64_t>(std::max<int32_t>(g->T, 1), 1023 * WAVE)) : 0;
}
static int tr_split(mr_ctx* ctx, mr_graph* g, const FxPlan& P, int64_t wsum, int64_t* nfa,
                    std::vector<CutArg>* defer = nullptr, int64_t force_nb = 0) {
    const int64_t W = g->n_wt, NW = P.NT / WAVE;
    const int64_t resident = plan_resident(kern_n(g), P);
    int64_t nb = std::max<int64_t>({std::min<int64_t>(resident, cdiv(W, NW)), cdiv(W, 1023), 1});
    if (const char* fe = getenv("MR_TR_BLOCKS"))   // (A/B knob, read per call) blocks of a lone graph
        if (force_nb <= 0 && wsum <= W && atoi(fe) > 0) force_nb = atoi(fe);
    if (force_nb > 0) {   // (at most 1023 wave tiles per block still)
        nb = std::max<int64_t>(force_nb, cdiv(W, 1023));
    } else {
        if (wsum > W) {
            const int64_t share = (int64_t)std::ceil((double)resident * (double)W / (double)wsum);
            nb = std::min(nb, share);
        }
        // at least two tiles per wave: a launch of few tiles (one window's graphs) otherwise runs a
        // block per 8 tiles, each paying its LDS image and an N-word partial row for them (C2 single
        // window: 365 blocks of one tile per wave 0.85 ms, ~180 blocks 0.78 ms; batches and whole
        // graphs run many tiles per wave and do not reach the cap)
        nb = std::max<int64_t>({std::min<int64_t>(nb, cdiv(W, 2 * NW)), cdiv(W, 1023), 1});
    }
    // on the device (k_tr_cut: no host round trip) unless a block's traces must be weighed by
    // their kinds' multiplicities (kind-compressed graphs) or the cut table exceeds its LDS
    if (g->tile_mult_h.empty() && nb * NW <= TC_MAX) {
        const int64_t nw = nb * NW;
        if (!(g->wtile.p && g->wtile_nw == nw && g->wtile_msum < 0)) {
            MR_TRY(g->wtile.alloc(ctx, (size_t)nw + 1));
            MR_TRY(g->dscale.alloc(ctx, 2));
            if (defer) {   // launched with the batch's other cuts (k_tr_cut_b)
                defer->push_back(CutArg{g->coff.p, g->wtile.p, g->dscale.p, (int32_t)W, (int32_t)nw, (int32_t)NW,
                                        (float)tr_tile_weight(g), tr_scfix(g)});
            } else {
                hipLaunchKernelGGL(k_tr_cut, dim3(1), dim3(TC_T), 0, ctx->stream, g->coff.p, (int32_t)W, (int32_t)nw,
                                   (int32_t)NW, g->wtile.p, g->dscale.p, tr_tile_weight(g), tr_scfix(g));
                MR_TRY_HIP(ctx, hipGetLastError());
            }
            g->wtile_nw = (int32_t)nw;
            g->wtile_msum = -1;   // the scale is on the device
        }
        *nfa = nb;
        return MR_OK;
    }
    if (g->coff_h.size() != (size_t)W + 1) {
        g->coff_h.assign((size_t)W + 1, 0);
        MR_TRY(g->coff.download(ctx, g->coff_h.data(), (size_t)W + 1));
        MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    }
    const std::vector<int32_t>& co = g->coff_h;
    for (;;) {
        const int64_t nw = nb * NW;
        if (g->wtile.p && g->wtile_nw == nw && g->wtile_msum >= 0) break;
        std::vector<int32_t> cut((size_t)nw + 1);
        const double tw = tr_tile_weight(g);
        const double total = W ? (double)co[(size_t)W] + tw * (double)W : 0.0;
        int64_t k = 0;
        for (int64_t i = 0; i <= nw; ++i) {   // first tile whose cost prefix reaches the target
            const double target = total * (double)i / (double)nw;
            while (k < W && (double)co[(size_t)k] + tw * (double)k < target) ++k;
            cut[(size_t)i] = (int32_t)k;
        }
        cut[(size_t)nw] = (int32_t)W;
        int32_t tpb = 0;
        int64_t msum = 0;   // traces a block stands for (kind-compressed graphs: with multiplicity)
        for (int64_t b = 0; b < nb; ++b) {
            const int32_t k0 = cut[(size_t)(b * NW)], k1 = cut[(size_t)((b + 1) * NW)];
            tpb = std::max(tpb, k1 - k0);
            int64_t m = (int64_t)(k1 - k0) * WAVE;
            if (!g->tile_mult_h.empty()) {
                m = 0;
                for (int32_t k = k0; k < k1; ++k) m += g->tile_mult_h[(size_t)k];
            }
            msum = std::max(msum, m);
        }
        if (tpb > 1023) {
            nb += resident;
            continue;
        }
        g->wtile_msum = msum;
        MR_TRY(g->wtile.upload(ctx, cut.data(), cut.size()));
        MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));   // (the host vector leaves scope)
        g->wtile_nw = (int32_t)nw;
        g->wtile_tpb = tpb;
        break;
    }
    *nfa = nb;
    return MR_OK;
}

// k_tr_a blocks of every graph of a batch launch: ONE resident set of blocks, split by the graphs'
// wave tiles so that the largest per-block share is as small as it can be -- each graph first gets
// floor(resident x its tiles / all tiles) blocks (at least one, at least its 1023-tile cap, at most
// one per two tiles per wave), then the remaining blocks go one at a time to the graph whose blocks
// carry the most tiles.  (Rounding each graph's share UP put 1152 blocks on the 1024 resident slots
// of a C2 group -- 128 windows' 13k- and 187k-trace graphs, 7.5 and 0.5 blocks of share each: a
// second round of blocks behind the first.)  Empty: the single-graph rule of tr_split.
#ifndef MR_TR_TPW
#define MR_TR_TPW 2   // batch launches: at least this many wave tiles per wave of a graph's blocks
#endif
static std::vector<int64_t> batch_blocks(mr_graph* const* gs, int ng, const FxPlan& P, int64_t wsum) {
    std::vector<int64_t> nb;
    int nf = 0;
    for (int i = 0; i < ng; ++i) nf += gs[i]->fused ? 1 : 0;
    if (nf < 2 || wsum <= 0) return nb;
    int64_t R = INT64_MAX;
    for (int i = 0; i < ng; ++i)
        if (gs[i]->fused) R = std::min(R, plan_resident(kern_n(gs[i]), P));
    // (two or three blocks per resident slot measured 2-3 % faster per iteration inside the pipeline
    // and within the wall-time spread, profiles/r06/r06i_oversub_ab.txt: one set kept)
#ifdef MR_AB_RFRAC   // (A/B builds: a fraction of the resident slots, leaving room for the builds' blocks)
    R = std::max<int64_t>(1, (int64_t)((double)R * MR_AB_RFRAC));
#endif
    const int64_t NW = P.NT / WAVE;
    nb.assign((size_t)ng, 0);
    std::vector<int64_t> cap((size_t)ng, 0);
    int64_t used = 0;
    for (int i = 0; i < ng; ++i) {
        if (!gs[i]->fused) continue;
        const int64_t W = gs[i]->n_wt, lo = std::max<int64_t>(cdiv(W, 1023), 1);
        cap[(size_t)i] = std::max<int64_t>(lo, cdiv(W, (int64_t)MR_TR_TPW * NW));
        nb[(size_t)i] = std::min(cap[(size_t)i], std::max(lo, (int64_t)((double)R * (double)W / (double)wsum)));
        used += nb[(size_t)i];
    }
    std::priority_queue<std::pair<double, int>> q;   // (tiles per block, graph)
    for (int i = 0; i < ng; ++i)
        if (gs[i]->fused && nb[(size_t)i] < cap[(size_t)i])
            q.push({(double)gs[i]->n_wt / (double)nb[(size_t)i], i});
    while (used < R && !q.empty()) {
        const int i = q.top().second;
        q.pop();
        ++nb[(size_t)i];
        ++used;
        if (nb[(size_t)i] < cap[(size_t)i]) q.push({(double)gs[i]->n_wt / (double)nb[(size_t)i], i});
    }
    return nb;
}
static int fused_blocks(mr_ctx* ctx, mr_graph* g, const FxPlan& P, int64_t wsum, int64_t* nfa,
                        std::vector<CutArg>* defer = nullptr, int64_t force_nb = 0) {
    return tr_split(ctx, g, P, wsum, nfa, defer, force_nb);
}

// k_tr_a's layout of a fused graph (after w_t and the kernel's ids rs16 / rsp): traces sorted by
// op count, tiles of 64 positions, ids lane-interleaved in chunks of 4.  One host round trip (the
// chunk count sizes the id array; the chunk offsets stay on the host for the per-wave cut).
// off / ids: the trace-major incidence the kernel walks (rs_off with rs16 / rsp, or a wide graph's
// hot entries), N: the kernel's op count (pads N + lane)
// hot ops stripped from the id chunks (register-accumulated in k_tr_a): MR_TR_HOT ops (default
// HOT_MAX, 0 = none) covering at least 1/8 of the traces, on graphs of >= MR_TR_HOT_MIN traces
// (default 2^20: window graphs keep their layout) whose su fits in LDS
static int hot_strip(mr_ctx* ctx, mr_graph* g, const int64_t*& off, const uint16_t*& src, int32_t N, int64_t& nent,
                     DBuf<int64_t>& roff, DBuf<uint16_t>& rids, DBuf<uint8_t>& mask) {
    // (read per preparation: tests flip them)
    const char* eh = getenv("MR_TR_HOT");
    const char* em = getenv("MR_TR_HOT_MIN");
    const int hcap = g->wide ? HOT_MAX_WIDE : HOT_MAX;   // (the wide variant carries fewer accumulators)
    const int hmax = eh ? std::min(std::max(atoi(eh), 0), hcap) : hcap;
    const int64_t tmin = em ? (int64_t)atoll(em) : TR_LARGE;
    g->nhr = 0;
    g->hmask.reset();
    const int32_t T = g->T;
    if (hmax == 0 || (int64_t)T < tmin || N < 1 || N > 16384 || !TrLds(N, WV_SU_ALL).hot_ok) return MR_OK;
    hipStream_t st = ctx->stream;
    std::vector<int32_t> cov((size_t)N);
    if (!g->wide && g->cov.p) {   // the kernel's ids are the graph's: its coverage (prepare / build) serves
        MR_TRY(g->cov.download(ctx, cov.data(), (size_t)N));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    } else {   // (wide graphs: the hot half's relabelled ids)
        DBuf<int32_t> dc;
        MR_TRY(dc.zero(ctx, (size_t)N));
        if (nent)
            hipLaunchKernelGGL(k_cov_hist, dim3(cdiv(nent, 256 * 64)), dim3(256), (size_t)N * sizeof(int32_t), st, src,
                               nent, N, dc.p);
        MR_TRY(dc.download(ctx, cov.data(), (size_t)N));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    }
    std::vector<int32_t> ord((size_t)N);
    for (int32_t o = 0; o < N; ++o) ord[(size_t)o] = o;
    std::stable_sort(ord.begin(), ord.end(), [&](int32_t a, int32_t b) { return cov[(size_t)a] > cov[(size_t)b]; });
    std::vector<int8_t> hidx((size_t)N, (int8_t)-1);
    int nh = 0;
    for (; nh < hmax && nh < N && (int64_t)cov[(size_t)ord[(size_t)nh]] * 8 >= (int64_t)T; ++nh) {
        hidx[(size_t)ord[(size_t)nh]] = (int8_t)nh;
        g->hop[nh] = ord[(size_t)nh];
    }
    // worth its pass only when the hot ops carry a quarter of the entries: the C4 graph's top 8
    // carry 26 % (iteration 154 -> 145 us); the span-built C4 graph's 23 % (op 0 in every trace, then
    // seven at 30 %) gained nothing measurable per iteration while the strip added ~1 ms to its
    // build (c4 --from-spans, A/B in the commit log)
    // (MR_TR_HOT_FRAC: that share, default 0.25; tests force the layout with 0)
    const char* ef = getenv("MR_TR_HOT_FRAC");
    const double fmin = ef ? atof(ef) : 0.25;
    int64_t hsum = 0;
    for (int h = 0; h < nh; ++h) hsum += cov[(size_t)g->hop[h]];
    if (nh == 0 || (double)hsum < fmin * (double)nent) return MR_OK;
    DBuf<int8_t> dh;
    DBuf<int32_t> rlen;
    DBuf<int64_t> tmp;
    MR_TRY(dh.upload(ctx, hidx.data(), hidx.size()));
    MR_TRY(rlen.alloc(ctx, (size_t)T));
    MR_TRY(mask.alloc(ctx, (size_t)T));
    MR_TRY(roff.alloc(ctx, (size_t)T + 1));
    MR_TRY(tmp.alloc(ctx, (size_t)scan_tmp_elems(T)));
    hipLaunchKernelGGL(k_hot_count, dim3(cdiv(T, 256)), dim3(256), (size_t)N, st, off, src, T, dh.p, N, rlen.p, mask.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, rlen.p, roff.p, T, tmp.p));
    // (sized by the full entry count: no read-back; nent stays an upper bound for the layout)
    MR_TRY(rids.alloc(ctx, (size_t)std::max<int64_t>(nent, 1) + 8));
    hipLaunchKernelGGL(k_hot_fill, dim3(cdiv(T, 256)), dim3(256), (size_t)N, st, off, src, T, dh.p, N, mask.p, roff.p, rids.p);
    MR_TRY_HIP(ctx, hipGetLastError());
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // (the host hidx leaves scope)
    g->nhr = nh;
    off = roff.p;
    src = rids.p;
    return MR_OK;
}

static int tr_layout(mr_ctx* ctx, mr_graph* g, const int64_t* off, const uint16_t* src, int32_t N, int64_t nent,
                     int32_t* zeroed, const int32_t* skey = nullptr) {
    hipStream_t st = ctx->stream;
    const int32_t T = g->T;
    DBuf<int64_t> roff;
    DBuf<uint16_t> rids;
    DBuf<uint8_t> hm;
    MR_TRY(hot_strip(ctx, g, off, src, N, nent, roff, rids, hm));
    const int32_t W = cdiv(T, WAVE);
    g->n_wt = W;
    g->wtile_nw = 0;
    const int32_t nbin = N + 1;   // trace lengths 1..N (distinct ops)
    // zeroed: 2 * nbin words the caller cleared (histogram, slot counters), else cleared here
    const bool lscan = nbin <= TP_LSCAN;
    DBuf<int32_t> hz;
    DBuf<int64_t> boff, c64, tmp;
    if (!zeroed) {
        MR_TRY(hz.zero(ctx, 2 * (size_t)nbin));
        zeroed = hz.p;
    }
    int32_t* hist = zeroed;
    int32_t* taken = zeroed + nbin;
    MR_TRY(c64.alloc(ctx, (size_t)W + 1));
    MR_TRY(g->tperm.alloc(ctx, (size_t)std::max(T, 1)));
    MR_TRY(g->w_tp.alloc(ctx, (size_t)std::max(T, 1)));
    g->tpos_ok = false;
    MR_TRY(g->coff.alloc(ctx, (size_t)W + 1));
    // (length, secondary key): a stable radix sort, equal keys in trace order -- for wide graphs (the
    // cold count as secondary key) and kind-compressed ones, whose fixed-point scale depends on
    // the tiles' multiplicity sums (the counting sort below orders equal lengths run-dependently)
    if (T && (skey || g->kinds_given)) {
        DBuf<uint64_t> key;
        DBuf<uint32_t> val;
        MR_TRY(key.alloc(ctx, (size_t)T));
        MR_TRY(val.alloc(ctx, (size_t)T));
        hipLaunchKernelGGL(k_tr_skey, dim3(cdiv(T, 256)), dim3(256), 0, st, off, skey, T, key.p, val.p);
        {
            SortScratch ws;
            MR_TRY(mr_radix_sort(ctx, key.p, val.p, T, bits_for((uint64_t)N) + 4, ws));
        }
        hipLaunchKernelGGL(k_tr_perm_w, dim3(cdiv(T, 256)), dim3(256), 0, st, val.p, g->w_t.p, T, g->tperm.p, g->w_tp.p);
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    } else if (T) {
        const bool big = (int64_t)T >= (int64_t)num_cus() * TRB * TR_PER_SMALL * 4;
        const int per = big ? TR_PER_BIG : TR_PER_SMALL;
        const int nb = cdiv(T, (int64_t)TRB * per);
        hipLaunchKernelGGL(big ? k_tr_hist<TR_PER_BIG> : k_tr_hist<TR_PER_SMALL>, dim3(nb), dim3(TRB),
                           (size_t)nbin * sizeof(int32_t), st, off, T, nbin, hist);
        if (!lscan) {
            MR_TRY(boff.alloc(ctx, (size_t)nbin + 1));
            MR_TRY(tmp.alloc(ctx, (size_t)scan_tmp_elems(nbin)));
            MR_TRY(mr_exclusive_scan_i32(ctx, hist, boff.p, nbin, tmp.p));
        }
        hipLaunchKernelGGL(big ? k_tr_place<TR_PER_BIG> : k_tr_place<TR_PER_SMALL>, dim3(nb), dim3(TRB),
                           2 * (size_t)nbin * sizeof(int32_t), st, off, T, nbin,
                           lscan ? (const int64_t*)nullptr : boff.p, hist, taken, g->w_t.p, g->tperm.p, g->w_tp.p);
    }
    {   // chunk counts per wave tile, their prefix and its int32 copy: one launch
        const int64_t nt = std::max<int64_t>(cdiv((int64_t)W, TS_TILE), 1);
        unsigned long long* dst = nullptr;
        uint64_t epoch = 0;
        MR_TRY(mr_dl_status(ctx, nt, &dst, &epoch));
        hipLaunchKernelGGL(k_tr_chunk_scan, dim3((unsigned)nt), dim3(TS_T), 0, st, g->tperm.p, off, T, W, c64.p,
                           g->coff.p, dst, epoch);
    }
    // the id array at an upper bound of the chunk count (no host round trip): tile k holds
    // ceil(maxlen_k / 4) chunks, and with lengths ascending maxlen_k <= every
    // length of tile k + 1, so sum_k maxlen_k <= nent / 64 + 2 N
    g->coff_h.clear();
    const int64_t nch = 2 * (int64_t)W + (nent / WAVE + 2 * (int64_t)N) / 4 + 2;
    MR_TRY(g->tids.alloc(ctx, (size_t)std::max<int64_t>(nch, 1) * WAVE * 4));
    if (W)
        hipLaunchKernelGGL(k_tr_fill, dim3(cdiv((int64_t)W * WAVE, 256)), dim3(256), 0, st, g->tperm.p, off, src,
                           c64.p, T, N, W, g->tids.p);
    if (g->nhr) {   // the hot-op bits in position order
        MR_TRY(g->hmask.alloc(ctx, (size_t)T));
        hipLaunchKernelGGL(k_hot_perm, dim3(cdiv(T, 256)), dim3(256), 0, st, g->tperm.p, hm.p, T, g->hmask.p);
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // (the stripped lists leave scope)
    }
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;   // (scratch returns to the stream-ordered pool)
}

// A wide fused graph (N > FX_NMAX): ops relabelled by coverage, hot entries (labels < NA) laid
// out for k_tr_a, cold entries per position for k_cold_trace and grouped by op range for
// k_cold_ops with the blocks of each range (about WIDE_CB over all ranges, by pair count).
static int wide_prepare(mr_ctx* ctx, mr_graph* g) {
    hipStream_t st = ctx->stream;
    const int32_t N = g->N, T = g->T, NA = WIDE_NA;
    const int64_t nnz = g->nnz_sr;
    g->wide = true;
    g->NA = NA;
    g->rsp.reset();
    // ---- coverage, then labels by descending coverage (perm[new] = old)
    if (!g->cov_ready) MR_TRY_HIP(ctx, hipMemsetAsync(g->cov.p, 0, (size_t)N * sizeof(int32_t), st));
    if (nnz && !g->cov_ready)
        hipLaunchKernelGGL(k_cov_hist_w, dim3(cdiv(nnz, (int64_t)256 * 256)), dim3(256),
                           (size_t)std::min(N, WIDE_HIST) * sizeof(int32_t), st, g->rs_ops.p, nnz, N, g->cov.p);
    const int nbo = bits_for((uint64_t)(N - 1));
    DBuf<uint64_t> key;
    DBuf<int32_t> inv;
    MR_TRY(key.alloc(ctx, (size_t)N));
    MR_TRY(inv.alloc(ctx, (size_t)N));
    MR_TRY(g->perm.alloc(ctx, (size_t)N));
    hipLaunchKernelGGL(k_relabel_keys_w, dim3(cdiv(N, 256)), dim3(256), 0, st, g->cov.p, N, nbo, key.p);
    {
        SortScratch ws;
        MR_TRY(mr_radix_sort(ctx, key.p, nullptr, N, nbo + 32, ws));
    }
    hipLaunchKernelGGL(k_relabel_perm_w, dim3(cdiv(N, 256)), dim3(256), 0, st, key.p, N, (1ull << nbo) - 1ull, g->perm.p,
                       inv.p);
    g->relabeled = true;
    // ---- hot entries per trace (u16, node order; a trace without any walks the pad id NA)
    DBuf<int32_t> nh, nc;
    DBuf<int64_t> tmp;
    MR_TRY(nh.alloc(ctx, (size_t)T));
    MR_TRY(nc.alloc(ctx, (size_t)T));
    MR_TRY(g->hot_off.alloc(ctx, (size_t)T + 1));
    MR_TRY(tmp.alloc(ctx, (size_t)scan_tmp_elems(std::max<int64_t>(T, 1))));
    hipLaunchKernelGGL(k_wide_count, dim3(cdiv(T, 256)), dim3(256), 0, st, g->rs_off.p, g->rs_ops.p, inv.p, T, NA, nh.p,
                       nc.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, nh.p, g->hot_off.p, T, tmp.p));
    int64_t n_hot = 0;
    MR_TRY_HIP(ctx, hipMemcpyAsync(&n_hot, g->hot_off.p + T, sizeof n_hot, hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    MR_TRY(g->hot16.alloc(ctx, (size_t)n_hot + 8));
    hipLaunchKernelGGL(k_wide_hot, dim3(cdiv(T, 256)), dim3(256), 0, st, g->rs_off.p, g->rs_ops.p, inv.p, T, NA,
                       g->hot_off.p, g->hot16.p);
    MR_TRY(tr_layout(ctx, g, g->hot_off.p, g->hot16.p, NA, n_hot, nullptr, nc.p));   // tperm, w_tp, tids, coff
    // ---- cold entries in position order
    DBuf<int32_t> cnt;
    DBuf<int64_t> coff64;
    MR_TRY(cnt.alloc(ctx, (size_t)T));
    MR_TRY(coff64.alloc(ctx, (size_t)T + 1));
    hipLaunchKernelGGL(k_wide_cold_cnt, dim3(cdiv(T, 256)), dim3(256), 0, st, g->tperm.p, nc.p, T, cnt.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, cnt.p, coff64.p, T, tmp.p));
    int64_t n_cold = 0;
    MR_TRY_HIP(ctx, hipMemcpyAsync(&n_cold, coff64.p + T, sizeof n_cold, hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    g->n_cold = n_cold;
    MR_TRY(g->cold_off_p.alloc(ctx, (size_t)T + 1));
    hipLaunchKernelGGL(k_tr_coff, dim3(cdiv((int64_t)T + 1, 256)), dim3(256), 0, st, coff64.p, T, g->cold_off_p.p);
    const int32_t W = g->n_wt;
    // ---- cold tiles of the short-tile walk (after cold_ops_p, below) and the long-tile start
    DBuf<int32_t> ccnt;
    DBuf<int64_t> cc64;
    MR_TRY(ccnt.alloc(ctx, (size_t)std::max(W, 1)));
    MR_TRY(cc64.alloc(ctx, (size_t)W + 1));
    MR_TRY(g->ccoff.alloc(ctx, (size_t)W + 1));
    const int32_t R = (int32_t)cdiv((int64_t)N - NA, WIDE_RW_MAX);
    const int32_t RW = (int32_t)(cdiv(cdiv((int64_t)N - NA, R), WAVE) * WAVE);
    g->n_ranges = R;
    g->cold_rw = RW;
    MR_TRY(g->cold_ops_p.alloc(ctx, (size_t)n_cold + 1));
    MR_TRY(g->cp_pos.alloc(ctx, (size_t)n_cold + 1));
    MR_TRY(g->cp_op.alloc(ctx, (size_t)n_cold + 1));
    DBuf<int64_t> rb;
    MR_TRY(rb.zero(ctx, (size_t)R + 1));
    {
        DBuf<uint64_t> ck;
        MR_TRY(ck.alloc(ctx, (size_t)n_cold + 1));
        if (T && !g->tpos_ok) {   // (the inverse of this layout's tperm; the preference reuses it)
            MR_TRY(g->tpos.alloc(ctx, (size_t)T));
            hipLaunchKernelGGL(k_inv_perm, dim3(cdiv(T, 256)), dim3(256), 0, st, g->tperm.p, T, g->tpos.p);
            g->tpos_ok = true;
        }
        if (T)
            hipLaunchKernelGGL(k_wide_cold_fill_t, dim3(cdiv(T, 256)), dim3(256), 0, st, g->tpos.p, g->rs_off.p,
                               g->rs_ops.p, inv.p, T, NA, RW, coff64.p, g->cold_ops_p.p, ck.p);
        SortScratch ws;
        MR_TRY(mr_radix_sort(ctx, ck.p, nullptr, n_cold, 8, ws));   // stable: positions stay ascending
        if (n_cold) {
            hipLaunchKernelGGL(k_wide_bounds, dim3(cdiv(n_cold, 256)), dim3(256), 0, st, ck.p, n_cold, R, rb.p);
            hipLaunchKernelGGL(k_wide_unpack, dim3(cdiv(n_cold, 256)), dim3(256), 0, st, ck.p, n_cold, g->cp_pos.p,
                               g->cp_op.p);
        }
    }
    if (W) {
        hipLaunchKernelGGL(k_ctile_cnt, dim3(cdiv(W, 256)), dim3(256), 0, st, g->cold_off_p.p, T, W, ccnt.p);
        DBuf<int64_t> tmp2;
        MR_TRY(tmp2.alloc(ctx, (size_t)scan_tmp_elems(W)));
        MR_TRY(mr_exclusive_scan_i32(ctx, ccnt.p, cc64.p, W, tmp2.p));
        hipLaunchKernelGGL(k_tr_coff, dim3(cdiv((int64_t)W + 1, 256)), dim3(256), 0, st, cc64.p, W, g->ccoff.p);
        int64_t nch = 0;
        MR_TRY_HIP(ctx, hipMemcpyAsync(&nch, cc64.p + W, sizeof nch, hipMemcpyDeviceToHost, st));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
        MR_TRY(g->ctids.alloc(ctx, (size_t)std::max<int64_t>(nch, 1) * WAVE * 2));
        hipLaunchKernelGGL(k_ctile_fill, dim3(cdiv((int64_t)W * WAVE, 256)), dim3(256), 0, st, g->cold_off_p.p,
                           g->cold_ops_p.p, cc64.p, T, N, W, g->ctids.p);
        // long tiles (more hot chunks than the short walk's last tier) and short tiles with more
        // than two cold chunks keep k_cold_trace's sums: the list of those tiles
        std::vector<int32_t> co((size_t)W + 1), cn((size_t)W), tl;
        MR_TRY(g->coff.download(ctx, co.data(), co.size()));
        MR_TRY(ccnt.download(ctx, cn.data(), cn.size()));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
        for (int32_t k = 0; k < W; ++k)
            if (co[(size_t)k + 1] - co[(size_t)k] > std::min(TR_TIERS_EXT, TR_TIERS_W32) || cn[(size_t)k] > 2) tl.push_back(k);
        g->n_ctl = (int32_t)tl.size();
        MR_TRY(g->ctl.alloc(ctx, std::max<size_t>(tl.size(), 1)));
        if (!tl.empty()) MR_TRY(g->ctl.upload(ctx, tl.data(), tl.size()));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // (the host list leaves scope)
    } else {
        MR_TRY_HIP(ctx, hipMemsetAsync(g->ccoff.p, 0, sizeof(int32_t), st));
        g->n_ctl = 0;
    }
    std::vector<int64_t> rbh((size_t)R + 1);
    MR_TRY(rb.download(ctx, rbh.data(), rbh.size()));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    // ---- k_cold_ops blocks: each range's pairs in equal slices, blocks proportional to its pairs
    std::vector<int32_t> rowbase((size_t)R + 1);
    std::vector<int64_t> beg;
    for (int32_t r = 0; r < R; ++r) {
        const int64_t pr = rbh[(size_t)r + 1] - rbh[(size_t)r];
        const int64_t nbr = std::max<int64_t>(1, (int64_t)std::llround((double)WIDE_CB * (double)pr / (double)std::max<int64_t>(n_cold, 1)));
        rowbase[(size_t)r] = (int32_t)beg.size();
        for (int64_t j = 0; j < nbr; ++j) beg.push_back(rbh[(size_t)r] + pr * j / nbr);
    }
    rowbase[(size_t)R] = (int32_t)beg.size();
    beg.push_back(rbh[(size_t)R]);
    g->n_cb = (int32_t)beg.size() - 1;
    MR_TRY(g->cb_beg.upload(ctx, beg.data(), beg.size()));
    MR_TRY(g->cold_rowbase.upload(ctx, rowbase.data(), rowbase.size()));
    MR_TRY(g->cold_part.alloc(ctx, (size_t)g->n_cb * (size_t)RW));
    MR_TRY(g->cold_acc.alloc(ctx, (size_t)T));
    DBuf<unsigned long long> span;
    MR_TRY(span.zero(ctx, 1));
    hipLaunchKernelGGL(k_wide_span, dim3(cdiv(g->n_cb, 256)), dim3(256), 0, st, g->cb_beg.p, g->n_cb, g->cp_pos.p, span.p);
    unsigned long long sp = 0;
    MR_TRY(span.download(ctx, &sp, 1));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // (also: the host vectors leave scope)
    g->cold_span = std::max<uint64_t>(sp, 1);
    g->n_tiles = 0;
    g->n_pairs = 0;
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}

// Derived per-graph arrays: fp32 reciprocals, u16 ids, and the P_sr tiles.  One host round trip
// (the number of (tile, op) pairs sizes the pair arrays).
// mr_graph_prepare of several graphs built from spans (a window's two): one launch per step when
// all are small fused graphs whose su stays in LDS (no relabelling, one-block histogram scan),
// else one prepare each.  keep: the descriptors' host copy, alive until the stream has used it.
int mr_graph_prepare_batch(mr_ctx* ctx, mr_graph* const* gs, int n, std::vector<unsigned char>& keep) {
    const bool off = getenv("MR_NO_PREP_BATCH") != nullptr;   // A/B knob (read per call: tests flip it)
    bool ok = !off && n >= 2 && getenv("MR_NO_FUSED") == nullptr;
    for (int i = 0; i < n && ok; ++i) {
        const mr_graph* g = gs[i];
        ok = g->rs_is_sr && g->traces_nonempty && !g->force_tile && g->cov_ready && g->N > 0 && g->T > 0 &&
             g->N <= FX_NMAX && g->N + 1 <= TP_LSCAN && g->nnz_rs == g->nnz_sr && g->nnz_sr < (1ll << 31) &&
             TrLds(g->N, WV_SU_ALL).su_lds &&
             (int64_t)g->T < (int64_t)num_cus() * TRB * TR_PER_SMALL * 4;
    }
    if (!ok) {
        for (int i = 0; i < n; ++i) MR_TRY(mr_graph_prepare(ctx, gs[i]));
        return MR_OK;
    }
    for (int i = 0; i < n; ++i) {   // (the batched layout keeps every op in the id chunks)
        gs[i]->nhr = 0;
        gs[i]->hmask.reset();
    }
    hipStream_t st = ctx->stream;
    keep.assign((size_t)n * sizeof(PDev), 0);
    PDev* hp = reinterpret_cast<PDev*>(keep.data());
    std::vector<DBuf<int32_t>> trz((size_t)n);
    std::vector<DBuf<int64_t>> c64((size_t)n);
    int32_t bgc = 0, bth = 0, bcs = 0, bfl = 0, nbin_max = 0;
    int64_t st_words = 0;
    for (int i = 0; i < n; ++i) {
        mr_graph* g = gs[i];
        const int32_t N = g->N, T = g->T, W = cdiv(T, WAVE);
        const int64_t nnz = g->nnz_sr;
        MR_TRY(g->w_t.alloc(ctx, (size_t)T));
        MR_TRY(g->u_o.alloc(ctx, (size_t)N));
        MR_TRY(g->pw.alloc(ctx, (size_t)N));
        MR_TRY(g->rs16.alloc(ctx, (size_t)nnz + 8));
        const int32_t nz = 2 * (N + 1);
        MR_TRY(trz[(size_t)i].alloc(ctx, (size_t)nz));
        MR_TRY(c64[(size_t)i].alloc(ctx, (size_t)W + 1));
        MR_TRY(g->tperm.alloc(ctx, (size_t)std::max(T, 1)));
        MR_TRY(g->tpos.alloc(ctx, (size_t)std::max(T, 1)));
        g->tpos_ok = true;   // (k_tr_place_b writes the inverse beside tperm)
        MR_TRY(g->w_tp.alloc(ctx, (size_t)std::max(T, 1)));
        MR_TRY(g->coff.alloc(ctx, (size_t)W + 1));
        const int64_t nch = 2 * (int64_t)W + (nnz / WAVE + 2 * (int64_t)N) / 4 + 2;   // as tr_layout
        MR_TRY(g->tids.alloc(ctx, (size_t)std::max<int64_t>(nch, 1) * WAVE * 4));
        g->relabeled = false;
        g->wide = false;
        g->NA = N;
        g->fused = true;
        g->perm.reset();
        g->rsp.reset();
        g->n_wt = W;
        g->wtile_nw = 0;
        g->coff_h.clear();
        g->n_tiles = 0;
        g->n_pairs = 0;
        PDev& v = hp[i];
        v.T = T;
        v.N = N;
        v.nbin = N + 1;
        v.W = W;
        v.nz = nz;
        v.nnz = nnz;
        v.n_cs = (int32_t)std::max<int64_t>(cdiv((int64_t)W, TS_TILE), 1);
        v.st_off = st_words;
        st_words += v.n_cs;
        v.len_t = g->len_t.p;
        v.len_o = g->len_o.p;
        v.nchild = g->nchild.p;
        v.rs_ops = g->rs_ops.p;
        v.rs_off = g->rs_off.p;
        v.w_t = g->w_t.p;
        v.u_o = g->u_o.p;
        v.pw = g->pw.p;
        v.w_tp = g->w_tp.p;
        v.rs16 = g->rs16.p;
        v.tids = g->tids.p;
        v.trz = trz[(size_t)i].p;
        v.tperm = g->tperm.p;
        v.tpos = g->tpos.p;
        v.coff = g->coff.p;
        v.c64 = c64[(size_t)i].p;
        v.b_gc = bgc;
        bgc += cdiv(std::max<int64_t>({(int64_t)T, (int64_t)N, cdiv(nnz, 4), (int64_t)nz}), 256);
        v.b_th = bth;
        bth += cdiv(T, (int64_t)TRB * TR_PER_SMALL);
        v.b_cs = bcs;
        bcs += v.n_cs;
        v.b_fill = bfl;
        bfl += cdiv((int64_t)W * WAVE, 256);
        nbin_max = std::max(nbin_max, N + 1);
    }
    DBuf<PDev> dpd;
    MR_TRY(dpd.upload(ctx, hp, (size_t)n));
    unsigned long long* dst = nullptr;
    uint64_t epoch = 0;
    MR_TRY(mr_dl_status(ctx, st_words, &dst, &epoch));
    hipLaunchKernelGGL(k_graph_consts_b, dim3(bgc), dim3(256), 0, st, dpd.p, n);
    hipLaunchKernelGGL(k_tr_hist_b, dim3(bth), dim3(TRB), (size_t)nbin_max * sizeof(int32_t), st, dpd.p, n);
    hipLaunchKernelGGL(k_tr_place_b, dim3(bth), dim3(TRB), 2 * (size_t)nbin_max * sizeof(int32_t), st, dpd.p, n);
    hipLaunchKernelGGL(k_tr_chunk_scan_b, dim3(bcs), dim3(TS_T), 0, st, dpd.p, n, dst, epoch);
    hipLaunchKernelGGL(k_tr_fill_b, dim3(bfl), dim3(256), 0, st, dpd.p, n);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;   // (scratch returns to the stream-ordered pool)
}

int mr_graph_prepare(mr_ctx* ctx, mr_graph* g) {
    hipStream_t st = ctx->stream;
    const int32_t N = g->N, T = g->T;
    const int64_t nnz = g->nnz_sr;
    if (nnz >= (1ll << 31)) return mr_fail(ctx, MR_ERR_ARG, "more than 2^31 (trace, op) pairs on one device: shard the traces");
    MR_TRY(g->w_t.alloc(ctx, (size_t)T));
    MR_TRY(g->u_o.alloc(ctx, (size_t)N));
    MR_TRY(g->pw.alloc(ctx, (size_t)N));
    if (!g->cov_ready) MR_TRY(g->cov.alloc(ctx, (size_t)N));
    const bool u16 = N <= 65536 && g->nnz_rs;
    if (u16) MR_TRY(g->rs16.alloc(ctx, (size_t)g->nnz_rs + 8));
    // the fused layout's histogram and slot counters, cleared by the same launch
    DBuf<int32_t> trz;
    const int32_t nz = N <= FX_NMAX ? 2 * (N + 1) : 0;
    if (nz) MR_TRY(trz.alloc(ctx, (size_t)nz));
    const int64_t nc = std::max<int64_t>({(int64_t)T, (int64_t)N, u16 ? cdiv(g->nnz_rs, 4) : 0, (int64_t)nz});
    if (nc)
        hipLaunchKernelGGL(k_graph_consts, dim3(cdiv(nc, 256)), dim3(256), 0, st, g->len_t.p, g->w_t.p, T, g->len_o.p,
                           g->nchild.p, g->u_o.p, g->pw.p, N, g->rs_ops.p, u16 ? g->nnz_rs : 0,
                           u16 ? g->rs16.p : (uint16_t*)nullptr, trz.p, nz);
    g->relabeled = false;   // (set below for fused graphs that need it)
    g->wide = false;
    g->NA = N;
    static const bool no_fused = getenv("MR_NO_FUSED") != nullptr;   // A/B knob: force the tile path
    static const bool no_wide = getenv("MR_NO_WIDE") != nullptr;     // A/B knob: N > FX_NMAX on the tile path
    const bool fusable = !no_fused && !g->force_tile && g->rs_is_sr && g->traces_nonempty;
    if (fusable && !no_wide && N > FX_NMAX && (int64_t)N <= (int64_t)WIDE_NA + (int64_t)WIDE_RMAX * WIDE_RW_MAX) {
        g->fused = true;
        return wide_prepare(ctx, g);
    }
    g->fused = fusable && N <= FX_NMAX;
    if (g->fused) {   // no P_sr tiles: the fused iteration reads the trace-major ids only
        if (!g->cov_ready) MR_TRY_HIP(ctx, hipMemsetAsync(g->cov.p, 0, (size_t)std::max(N, 1) * sizeof(int32_t), st));
        if (nnz && N && !g->cov_ready)
            hipLaunchKernelGGL(k_cov_hist, dim3(cdiv(nnz, 256 * 64)), dim3(256), (size_t)N * sizeof(int32_t), st,
                               g->rs16.p, nnz, N, g->cov.p);
        // su does not fit in LDS beside the accumulators: relabel ops by descending coverage so
        // k_tr_a stages the su of the most covered ops (ops [0, n_hot)) and gathers the rest.
        // The kinds keep rs16 (original labels, the same hash on every rank); only the
        // iteration's id stream (rsp), su and the partial rows use the new labels.
        g->relabeled = !TrLds(N, WV_SU_ALL).su_lds;
        if (g->relabeled) {
            DBuf<uint64_t> key;
            DBuf<int32_t> inv;
            MR_TRY(key.alloc(ctx, (size_t)N));
            MR_TRY(inv.alloc(ctx, (size_t)N));
            MR_TRY(g->perm.alloc(ctx, (size_t)N));
            MR_TRY(g->rsp.alloc(ctx, (size_t)nnz + 8));
            hipLaunchKernelGGL(k_relabel_keys, dim3(cdiv(N, 256)), dim3(256), 0, st, g->cov.p, N, key.p);
            SortScratch ws;
            MR_TRY(mr_radix_sort(ctx, key.p, nullptr, N, 46, ws));
            hipLaunchKernelGGL(k_relabel_perm, dim3(cdiv(N, 256)), dim3(256), 0, st, key.p, N, g->perm.p, inv.p);
            if (nnz) hipLaunchKernelGGL(k_relabel_ids, dim3(cdiv(nnz, 256)), dim3(256), 0, st, g->rs16.p, nnz, inv.p, g->rsp.p);
        } else {
            g->perm.reset();
            g->rsp.reset();
        }
        MR_TRY(tr_layout(ctx, g, g->rs_off.p, g->relabeled ? g->rsp.p : g->rs16.p, N, nnz, trz.p));
        g->n_tiles = 0;
        g->n_pairs = 0;
        MR_TRY_HIP(ctx, hipGetLastError());
        return MR_OK;
    }
    // tiles: ~256 of them when T allows, 256..4096 traces each
    int ts = TSHIFT_MIN;
    while (ts < TSHIFT_MAX && ((int64_t)T >> ts) > 256) ++ts;
    g->tshift = ts;
    g->n_tiles = T ? cdiv(T, (int64_t)1 << ts) : 0;
    const int32_t NTL = g->n_tiles;
    const int nb = std::max(1, bits_for((uint64_t)std::max(N - 1, 0)));
    const int64_t* off = g->rs_is_sr ? g->rs_off.p : g->srt_off.p;
    const int32_t* ops = g->rs_is_sr ? g->rs_ops.p : g->srt_ops.p;
    MR_TRY(g->tl_ltr.alloc(ctx, (size_t)nnz));
    MR_TRY(g->tile_pr0.alloc(ctx, (size_t)NTL + 1));
    MR_TRY(g->tile_lp0.alloc(ctx, (size_t)NTL + 1));
    MR_TRY(g->op_pr_off.alloc(ctx, (size_t)N + 1));
    int64_t np = 0;
    DBuf<int32_t> pr_tile;
    {
        DBuf<uint64_t> key;
        DBuf<uint32_t> val;
        DBuf<int32_t> head;
        DBuf<int64_t> hpos, tmp;
        MR_TRY(key.alloc(ctx, (size_t)nnz));
        MR_TRY(val.alloc(ctx, (size_t)nnz));
        MR_TRY(head.alloc(ctx, (size_t)nnz));
        MR_TRY(hpos.alloc(ctx, (size_t)nnz + 1));
        MR_TRY(tmp.alloc(ctx, (size_t)scan_tmp_elems(std::max<int64_t>(nnz, 1))));
        if (T) hipLaunchKernelGGL(k_tile_keys, dim3(cdiv(T, 256)), dim3(256), 0, st, off, ops, T, ts, nb, key.p, val.p);
        SortScratch ws;
        MR_TRY(mr_radix_sort(ctx, key.p, val.p, nnz, nb + bits_for((uint64_t)std::max(NTL - 1, 0)), ws));
        if (nnz) hipLaunchKernelGGL(k_key_heads, dim3(cdiv(nnz, 256)), dim3(256), 0, st, key.p, nnz, head.p);
        MR_TRY(mr_exclusive_scan_i32(ctx, head.p, hpos.p, nnz, tmp.p));
        MR_TRY_HIP(ctx, hipMemcpyAsync(&np, hpos.p + nnz, sizeof np, hipMemcpyDeviceToHost, st));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
        g->n_pairs = np;
        MR_TRY(g->pr_op.alloc(ctx, (size_t)np));
        MR_TRY(g->pr_beg.alloc(ctx, (size_t)np + 1));
        MR_TRY(pr_tile.alloc(ctx, (size_t)np));
        if (nnz)
            hipLaunchKernelGGL(k_tile_pairs, dim3(cdiv(nnz, 256)), dim3(256), 0, st, key.p, val.p, head.p, hpos.p, nnz, nb,
                               g->tl_ltr.p, g->pr_op.p, g->pr_beg.p, pr_tile.p);
        else
            MR_TRY_HIP(ctx, hipMemsetAsync(g->pr_beg.p, 0, sizeof(int64_t), st));
    }
    hipLaunchKernelGGL(k_lower_bound<int32_t>, dim3(cdiv(NTL + 1, 256)), dim3(256), 0, st, pr_tile.p, np,
                       (const int64_t*)nullptr, NTL, g->tile_pr0.p);
    // long pairs (> LONG_PAIR entries) get a whole wave; listed per tile
    MR_TRY(g->lp.alloc(ctx, (size_t)std::max<int64_t>(np, 1)));
    {
        DBuf<int32_t> lflag, lp_tile;
        DBuf<int64_t> lpos, tmp;
        MR_TRY(lflag.alloc(ctx, (size_t)np));
        MR_TRY(lpos.alloc(ctx, (size_t)np + 1));
        MR_TRY(lp_tile.alloc(ctx, (size_t)std::max<int64_t>(np, 1)));
        MR_TRY(tmp.alloc(ctx, (size_t)scan_tmp_elems(std::max<int64_t>(np, 1))));
        if (np) hipLaunchKernelGGL(k_long_flags, dim3(cdiv(np, 256)), dim3(256), 0, st, g->pr_beg.p, np, lflag.p);
        MR_TRY(mr_exclusive_scan_i32(ctx, lflag.p, lpos.p, np, tmp.p));
        if (np)
            hipLaunchKernelGGL(k_long_list, dim3(cdiv(np, 256)), dim3(256), 0, st, lflag.p, lpos.p, pr_tile.p, np, g->lp.p,
                               lp_tile.p);
        hipLaunchKernelGGL(k_lower_bound<int32_t>, dim3(cdiv(NTL + 1, 256)), dim3(256), 0, st, lp_tile.p, (int64_t)0,
                           lpos.p + np, NTL, g->tile_lp0.p);
    }
    // op-major order of the pairs (tile order within an op): the s' reduction order
    MR_TRY(g->op_pr.alloc(ctx, (size_t)np));
    {
        DBuf<uint64_t> key;
        DBuf<uint32_t> val;
        DBuf<int32_t> okey;
        MR_TRY(key.alloc(ctx, (size_t)np));
        MR_TRY(val.alloc(ctx, (size_t)np));
        MR_TRY(okey.alloc(ctx, (size_t)np));
        if (np) hipLaunchKernelGGL(k_pair_op_keys, dim3(cdiv(np, 256)), dim3(256), 0, st, g->pr_op.p, np, key.p, val.p);
        SortScratch ws;
        MR_TRY(mr_radix_sort(ctx, key.p, val.p, np, nb, ws));
        if (np) hipLaunchKernelGGL(k_op_pairs, dim3(cdiv(np, 256)), dim3(256), 0, st, key.p, val.p, np, g->op_pr.p, okey.p);
        hipLaunchKernelGGL(k_lower_bound<int32_t>, dim3(cdiv(N + 1, 256)), dim3(256), 0, st, okey.p, np,
                           (const int64_t*)nullptr, N, g->op_pr_off.p);
    }
    if (N) hipLaunchKernelGGL(k_cov, dim3(cdiv(N, 256)), dim3(256), 0, st, g->op_pr_off.p, g->op_pr.p, g->pr_beg.p, N, g->cov.p);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;   // scratch returns to the stream-ordered pool: no sync needed
}


// kinds, preference vector and iteration state of one graph (everything before the iterations)
static int shard_kinds(mr_ctx* ctx, mr_graph* g, uint64_t cap);
static int graph_kinds(mr_ctx* ctx, mr_graph* g, bool chk, bool ktab, uint64_t cap, uint64_t seed, uint64_t hmask);

// (plan-independent: a window's graphs are set up on the stream that built them, before the
// batch's plan exists -- mr_pagerank_presetup)
static int lo_setup_one(mr_ctx* ctx, mr_graph* g, int anomaly, double d, bool fp32);
static int pagerank_setup(mr_ctx* ctx, mr_graph* g, int anomaly, double d, bool fp32, uint32_t flags, bool sharded,
                          uint64_t seed, uint64_t hmask) {
    if (g->lo) return lo_setup_one(ctx, g, anomaly, d, fp32);   // (exact kind classes: no seed to vary)
    hipStream_t st = ctx->stream;
    const int32_t N = g->N, T = g->T;
    // Kinds through a global hash table (k_kind_insert) while it stays cache-resident, and for one
    // shard of a multi-rank graph (the cross-rank merge needs its classes and a check hash per
    // class); larger graphs by partition (k_kind_rec .. k_kind_final: no table of random atomics)
    const bool chk = sharded && ctx->nranks > 1;
    uint64_t cap = 1;
    while (cap < 2ull * (uint64_t)T) cap <<= 1;
    const char* kpe = getenv("MR_KIND_PART_MIN");   // test knob (read per call): traces from which the partition path runs
    const int64_t kp_min = kpe ? (int64_t)atoll(kpe) : KIND_PART_MIN_DEFAULT;
    const bool ktab = chk || (int64_t)T < kp_min;
    if (!ktab) cap = 0;
    const int32_t n_pr = g->n_pr;
    const int nbp = cdiv(n_pr > 0 ? n_pr : 1, TB);
    MR_TRY(g->kind.alloc(ctx, (size_t)T));
    MR_TRY(g->pref.alloc(ctx, (size_t)T));
    MR_TRY(g->c_t.alloc(ctx, (size_t)T));
    MR_TRY(g->flag.alloc(ctx, 8));
    MR_TRY(g->scal.alloc(ctx, 8));
    MR_TRY(g->ppart.alloc(ctx, 2 * (size_t)nbp));
    if (ktab) {
        MR_TRY(g->ht_key.alloc(ctx, cap));
        MR_TRY(g->ht_cr.alloc(ctx, cap));
        MR_TRY(g->slot_of.alloc(ctx, (size_t)T));
    }
    MR_TRY(g->mslot.alloc(ctx, MSLOT_WORDS));
    MR_TRY(g->sn.alloc(ctx, (size_t)N));
    MR_TRY(g->spb[0].alloc(ctx, (size_t)N));
    MR_TRY(g->spb[1].alloc(ctx, (size_t)N));
    MR_TRY(g->sub[0].alloc(ctx, (size_t)N + TR_PAD));   // [N, N + TR_PAD) = 0: the fused walks' pad slots
    MR_TRY(g->sub[1].alloc(ctx, (size_t)N + TR_PAD));
    if (fp32 && g->wide) {
        MR_TRY(g->suf[0].alloc(ctx, (size_t)N + TR_PAD));
        MR_TRY(g->suf[1].alloc(ctx, (size_t)N + TR_PAD));
    }
    MR_TRY(g->weight.alloc(ctx, (size_t)N));
    const bool tr = g->fused;
    if (tr) MR_TRY(g->c_tp.alloc(ctx, (size_t)std::max(T, 1)));
    if (g->fused) MR_TRY(g->fx_ssv.alloc(ctx, (size_t)N));
    else MR_TRY(g->part.alloc(ctx, (size_t)std::max<int64_t>(g->n_pairs, 1)));
    for (int i = 0; i < 2; ++i) {
        if (fp32) MR_TRY(g->q32[i].alloc(ctx, (size_t)T + 1));   // [T]: k_tr_a's pad slot
        else MR_TRY(g->q64[i].alloc(ctx, (size_t)T + 1));
    }
    // one launch clears every per-call word (instead of a memset per buffer) and sets the iteration
    // state up (k_iter_init's part: it depends on nothing the kinds / preference compute)
    hipLaunchKernelGGL(k_pr_reset_init,
                       dim3(cdiv(std::max<int64_t>({(int64_t)T, (int64_t)cap, (int64_t)N + TR_PAD, MSLOT_WORDS, 16}), 256)),
                       dim3(256), 0, st, T, (int64_t)cap, N, g->pref.p, g->c_t.p, g->ht_key.p, g->ht_cr.p,
                       g->flag.p, g->scal.p, tr ? g->w_tp.p : g->w_t.p, tr ? g->mw_tp.p : nullptr, g->u_o.p,
                       g->T_all > 0 ? g->T_all : (int64_t)T, g->spb[0].p, g->sub[0].p, g->sub[1].p, g->q64[0].p,
                       g->q32[0].p, (int)fp32, g->mslot.p, g->relabeled ? (const int32_t*)g->perm.p : nullptr,
                       (int)(fp32 && g->wide), g->suf[0].p, g->suf[1].p);
    MR_DEBUG_CHECK(ctx, "k_pr_reset_init");
    // ---- kinds (a kind-compressed graph carries its class sizes: kinds_given)
    if (!g->kinds_given) MR_TRY(graph_kinds(ctx, g, chk, ktab, cap, seed, hmask));
    if (chk) MR_TRY(shard_kinds(ctx, g, cap));   // class sizes over all ranks (one rank: already global)
    // ---- preference
    const int32_t* prt = g->pr_identity ? nullptr : g->pr_trace.p;
    const int32_t* prl = g->pr_identity ? nullptr : g->pr_len.p;
    // also with n_pr == 0 (an empty shard): the one block writes the zero partials the sums read
    hipLaunchKernelGGL(k_pref_partial, dim3(nbp), dim3(TB), 0, st, g->kind.p, prt, prl, g->len_t.p, n_pr,
                       g->mult.p, g->ppart.p, g->flag.p);
    if ((flags & MR_PR_EXACT_SUMS) && !sharded && !g->mult.p)
        hipLaunchKernelGGL(k_pref_total_exact, dim3(1), dim3(64), 0, st, g->kind.p, prt, prl, g->len_t.p, n_pr,
                           g->scal.p);
    else
        hipLaunchKernelGGL(k_pref_total, dim3(1), dim3(1024), 0, st, g->ppart.p, nbp, g->scal.p);
    MR_DEBUG_CHECK(ctx, "k_pref");
    if (sharded) MR_TRY(mr_coll_allreduce(ctx, g->scal.p + 2, 2, MR_DT_F64, 0));   // sum(1/k), sum(1/len)
    const float cd = (float)(1.0 - d);
    // k_tr_a graphs whose pr_trace is operation_trace: c_t in position order from the same launch
    const bool fuse_gather = tr && !prt && !prl && n_pr == T;
    // large graphs: trace order, c_tp scattered through the inverse permutation (built once per layout)
    const char* pte = getenv("MR_PREF_T_MIN");   // (tests, A/B; read per call) traces from which the trace-order form runs
    const int64_t pref_t_min = pte ? (int64_t)atoll(pte) : (int64_t)1 << 20;
    if (fuse_gather && T > 0 && (int64_t)T >= pref_t_min) {
        if (!g->tpos_ok) {
            MR_TRY(g->tpos.alloc(ctx, (size_t)T));
            hipLaunchKernelGGL(k_inv_perm, dim3(cdiv(T, 256)), dim3(256), 0, st, g->tperm.p, T, g->tpos.p);
            g->tpos_ok = true;
        }
        hipLaunchKernelGGL(k_pref_apply_t, dim3(cdiv(T, 256)), dim3(256), 0, st, g->kind.p, g->len_t.p, T, g->scal.p,
                           anomaly, cd, g->phi, g->pref.p, g->tpos.p, g->c_tp.p);
        MR_DEBUG_CHECK(ctx, "k_pref_apply_t");
        return MR_OK;
    }
    if (n_pr > 0)
        hipLaunchKernelGGL(k_pref_apply, dim3(nbp), dim3(TB), 0, st, g->kind.p, prt, prl, g->len_t.p, n_pr,
                           g->scal.p, anomaly, cd, g->phi, g->pref.p, g->c_t.p, fuse_gather ? (const int32_t*)g->tperm.p : nullptr,
                           fuse_gather ? g->c_tp.p : nullptr);
    MR_DEBUG_CHECK(ctx, "k_pref_apply");
    if (tr && T && !fuse_gather)
        hipLaunchKernelGGL(k_tr_gather, dim3(cdiv(T, 256)), dim3(256), 0, st, g->c_t.p, g->tperm.p, T, g->c_tp.p);
    return MR_OK;
}

// Can pagerank_setup of g run inside a batched set-up?  The window graphs' case: a whole graph on
// one rank, kinds through the hash table with u16 ids, pr_trace = operation_trace, k_tr_a layout.
static bool setup_batchable(const mr_graph* g, uint32_t flags) {
    const char* kpe = getenv("MR_KIND_PART_MIN");
    const int64_t kp_min = kpe ? (int64_t)atoll(kpe) : KIND_PART_MIN_DEFAULT;
    return g->T > 0 && (int64_t)g->T < kp_min && !g->kinds_given && !g->mult.p && g->rs_is_sr && g->rs16.p &&
           g->pr_identity && g->n_pr == g->T && g->fused && g->tperm.p && g->w_tp.p && !g->mw_tp.p &&
           !(flags & MR_PR_EXACT_SUMS) && g->T_all == 0;
}

// pagerank_setup of several graphs (all setup_batchable) in six launches
// hs / dsd: the descriptors (host and device), owned by the caller until its stream work is done
static int pagerank_setup_batch(mr_ctx* ctx, mr_graph* const* gs, const int* anomaly, int ng, double d, bool fp32,
                                uint64_t seed, uint64_t hmask, std::vector<unsigned char>& keep, DBuf<SDev>& dsd) {
    hipStream_t st = ctx->stream;
    keep.assign((size_t)ng * sizeof(SDev), 0);
    SDev* hs = reinterpret_cast<SDev*>(keep.data());
    int32_t br = 0, bk = 0, bv = 0, bp = 0;
    for (int i = 0; i < ng; ++i) {
        mr_graph* g = gs[i];
        const int32_t N = g->N, T = g->T;
        uint64_t cap = 1;
        while (cap < 2ull * (uint64_t)T) cap <<= 1;
        const int nbp = cdiv(T, TB);
        MR_TRY(g->kind.alloc(ctx, (size_t)T));
        MR_TRY(g->pref.alloc(ctx, (size_t)T));
        MR_TRY(g->c_t.alloc(ctx, (size_t)T));
        MR_TRY(g->flag.alloc(ctx, 8));
        MR_TRY(g->scal.alloc(ctx, 8));
        MR_TRY(g->ppart.alloc(ctx, 2 * (size_t)nbp));
        MR_TRY(g->ht_key.alloc(ctx, cap));
        MR_TRY(g->ht_cr.alloc(ctx, cap));
        MR_TRY(g->slot_of.alloc(ctx, (size_t)T));
        MR_TRY(g->mslot.alloc(ctx, MSLOT_WORDS));
        MR_TRY(g->sn.alloc(ctx, (size_t)N));
        MR_TRY(g->spb[0].alloc(ctx, (size_t)N));
        MR_TRY(g->spb[1].alloc(ctx, (size_t)N));
        MR_TRY(g->sub[0].alloc(ctx, (size_t)N + TR_PAD));
        MR_TRY(g->sub[1].alloc(ctx, (size_t)N + TR_PAD));
        MR_TRY(g->weight.alloc(ctx, (size_t)N));
        MR_TRY(g->c_tp.alloc(ctx, (size_t)std::max(T, 1)));
        MR_TRY(g->fx_ssv.alloc(ctx, (size_t)N));
        for (int j = 0; j < 2; ++j) {
            if (fp32) MR_TRY(g->q32[j].alloc(ctx, (size_t)T + 1));
            else MR_TRY(g->q64[j].alloc(ctx, (size_t)T + 1));
        }
        SDev& v = hs[i];
        v.T = T;
        v.N = N;
        v.anomaly = anomaly[i];
        v.fp32 = fp32 ? 1 : 0;
        v.cap = (int64_t)cap;
        v.T_all = T;
        v.cd = (float)(1.0 - d);
        v.phi = g->phi;
        v.pref = g->pref.p;
        v.c_t = g->c_t.p;
        v.c_tp = g->c_tp.p;
        v.tperm = g->tperm.p;
        if (!g->tpos_ok) {   // (graphs prepared one at a time: the inverse of tperm, once per layout)
            MR_TRY(g->tpos.alloc(ctx, (size_t)std::max(T, 1)));
            if (T) hipLaunchKernelGGL(k_inv_perm, dim3(cdiv(T, 256)), dim3(256), 0, st, g->tperm.p, T, g->tpos.p);
            g->tpos_ok = true;
        }
        v.tpos = g->tpos.p;
        v.hk = g->ht_key.p;
        v.cr = g->ht_cr.p;
        v.slot_of = g->slot_of.p;
        v.flag = g->flag.p;
        v.kind = g->kind.p;
        v.scal = g->scal.p;
        v.ppart = g->ppart.p;
        v.w_t = g->w_t.p;
        v.w_tq = g->w_tp.p;
        v.u_o = g->u_o.p;
        v.sp0 = g->spb[0].p;
        v.su0 = g->sub[0].p;
        v.su1 = g->sub[1].p;
        v.q64 = g->q64[0].p;
        v.q32 = g->q32[0].p;
        v.mslot = g->mslot.p;
        v.perm = g->relabeled ? g->perm.p : nullptr;
        v.off = g->rs_off.p;
        v.o16 = g->rs16.p;
        v.len_t = g->len_t.p;
        v.b_reset = br;
        br += cdiv(std::max<int64_t>({(int64_t)T, (int64_t)cap, (int64_t)N + TR_PAD, MSLOT_WORDS, 16}), 256);
        v.b_kins = bk;
        bk += cdiv(T, KB);
        v.b_kver = bv;
        bv += cdiv(T, 256);
        v.b_pref = bp;
        bp += nbp;
    }
    MR_TRY(dsd.upload(ctx, hs, (size_t)ng));
    hipLaunchKernelGGL(k_reset_init_b, dim3(br), dim3(256), 0, st, dsd.p, ng);
    hipLaunchKernelGGL(k_kind_insert_b, dim3(bk), dim3(KB), 0, st, dsd.p, ng, seed, hmask);
    hipLaunchKernelGGL(k_kind_verify_b, dim3(bv), dim3(256), 0, st, dsd.p, ng);
    hipLaunchKernelGGL(k_pref_partial_b, dim3(bp), dim3(TB), 0, st, dsd.p, ng);
    hipLaunchKernelGGL(k_pref_total_b, dim3(ng), dim3(1024), 0, st, dsd.p);
    hipLaunchKernelGGL(k_pref_apply_b, dim3(bp), dim3(TB), 0, st, dsd.p, ng);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}

// Kinds of g (pagerank.py:54-66) into g->kind, the class representative of each trace into
// g->krep when that is allocated; a 64-bit key collision sets flag word 0.
static int graph_kinds(mr_ctx* ctx, mr_graph* g, bool chk, bool ktab, uint64_t cap, uint64_t seed, uint64_t hmask) {
    hipStream_t st = ctx->stream;
    const int32_t T = g->T;
    const int64_t* koff = g->rs_is_sr ? g->rs_off.p : g->srt_off.p;
    const int32_t* kops = g->rs_is_sr ? g->rs_ops.p : g->srt_ops.p;
    static const bool walk = getenv("MR_KIND_WALK") != nullptr;   // A/B knob: per-thread int32 walk
    const bool u16 = !walk && g->rs_is_sr && g->rs16.p != nullptr;   // rs16 = u16 copy of rs_ops
    if (ktab) {
        if (chk) MR_TRY(g->ht_chk.alloc(ctx, cap));
        auto kins = chk ? (u16 ? k_kind_insert<true, 2> : walk ? k_kind_insert<true, 0> : k_kind_insert<true, 4>)
                        : (u16 ? k_kind_insert<false, 2> : walk ? k_kind_insert<false, 0> : k_kind_insert<false, 4>);
        if (T)
            hipLaunchKernelGGL(kins, dim3(cdiv(T, KB)), dim3(KB), 0, st, koff, kops, (const uint16_t*)g->rs16.p, g->w_t.p,
                               T, g->ht_key.p, g->ht_cr.p, g->slot_of.p, (uint64_t)(cap - 1), seed,
                               chk ? g->ht_chk.p : (uint64_t*)nullptr, hmask);
        MR_DEBUG_CHECK(ctx, "k_kind_insert");
        if (T && u16)
            hipLaunchKernelGGL(k_kind_verify<uint16_t>, dim3(cdiv(T, 256)), dim3(256), 0, st, koff,
                               (const uint16_t*)g->rs16.p, g->w_t.p, T, g->ht_cr.p, g->slot_of.p, g->kind.p, g->flag.p,
                               g->krep.p);
        else if (T)
            hipLaunchKernelGGL(k_kind_verify<int32_t>, dim3(cdiv(T, 256)), dim3(256), 0, st, koff, kops, g->w_t.p, T,
                               g->ht_cr.p, g->slot_of.p, g->kind.p, g->flag.p, g->krep.p);
        MR_DEBUG_CHECK(ctx, "k_kind_verify");
    } else if (T) {
        // partitions P = 2^pb >= T / KP_MEAN by the hash's top bits (records <= T)
        const int pb = bits_for((uint64_t)(cdiv(T, KP_MEAN) - 1));
        const int64_t P = (int64_t)1 << pb;
        const int32_t nb = cdiv(T, KB);
        const size_t R = (size_t)nb * KB;
        DBuf<KRec> rec, e;
        DBuf<int32_t> nrec, rec_of, rpos, hist;
        DBuf<uint32_t> eslot;
        DBuf<int64_t> pstart, tmp;
        DBuf<unsigned long long> cur;
        MR_TRY(rec.alloc(ctx, R));
        MR_TRY(e.alloc(ctx, (size_t)T));
        MR_TRY(nrec.alloc(ctx, (size_t)nb));
        MR_TRY(rec_of.alloc(ctx, (size_t)T));
        MR_TRY(pstart.alloc(ctx, (size_t)P + 1));
        // The two-pass grouping (k_kp1_*, k_kp2; no device atomic per record) at every size: its
        // records carry their block-order slot (eslot), k_kind_part writes each class back there and
        // k_kind_final reads it in block order -- one random 8-B write per record, where the
        // per-record cursor scatter (k_kind_rscatter: a returning atomic and a random 16-B write per
        // record, then a random read per trace; 7.4 ms of C5's 100M records) took three.
        // MR_KIND_GROUP=cursor (A/B, read per call) forces the cursor form.
        const char* kge = getenv("MR_KIND_GROUP");
        const bool cursor = kge && !strcmp(kge, "cursor");
        auto krec = u16 ? k_kind_rec<2> : walk ? k_kind_rec<0> : k_kind_rec<4>;
        if (cursor) {
            MR_TRY(rpos.alloc(ctx, R));
            MR_TRY(hist.zero(ctx, (size_t)P));
            MR_TRY(cur.alloc(ctx, (size_t)P));
            MR_TRY(tmp.alloc(ctx, (size_t)scan_tmp_elems(P)));
            hipLaunchKernelGGL(krec, dim3(nb), dim3(KB), 0, st, koff, kops, (const uint16_t*)g->rs16.p, g->w_t.p, T,
                               seed, hmask, pb, rec.p, nrec.p, rec_of.p, hist.p);
            MR_TRY(mr_exclusive_scan_i32(ctx, hist.p, pstart.p, P, tmp.p));
            MR_TRY_HIP(ctx, hipMemcpyAsync(cur.p, pstart.p, (size_t)P * sizeof(int64_t), hipMemcpyDeviceToDevice, st));
            hipLaunchKernelGGL(k_kind_rscatter, dim3(cdiv((int64_t)R, 256)), dim3(256), 0, st, rec.p, nrec.p,
                               (int32_t)std::min<size_t>(R, 0x7fffffff), pb, cur.p, e.p, rpos.p);
        } else {
            const int b1 = std::min(pb, KP1_B), nbk = 1 << b1, nf = 1 << (pb - b1);
            const int32_t ntile = (int32_t)cdiv((int64_t)R, KT);
            const int64_t nc = (int64_t)nbk * ntile;
            DBuf<int32_t> tcnt;
            DBuf<int64_t> toff;
            DBuf<KRec> r1;
            DBuf<uint32_t> s1;
            MR_TRY(tcnt.alloc(ctx, (size_t)nc));
            MR_TRY(toff.alloc(ctx, (size_t)nc + 1));
            MR_TRY(tmp.alloc(ctx, (size_t)scan_tmp_elems(nc)));
            MR_TRY(r1.alloc(ctx, (size_t)T));
            MR_TRY(s1.alloc(ctx, (size_t)T));
            hipLaunchKernelGGL(krec, dim3(nb), dim3(KB), 0, st, koff, kops, (const uint16_t*)g->rs16.p, g->w_t.p, T,
                               seed, hmask, pb, rec.p, nrec.p, rec_of.p, (int32_t*)nullptr);
            hipLaunchKernelGGL(k_kp1_count, dim3(ntile), dim3(KT_T), 0, st, rec.p, nrec.p, (int64_t)R, b1, ntile, tcnt.p);
            MR_TRY(mr_exclusive_scan_i32(ctx, tcnt.p, toff.p, nc, tmp.p));
            hipLaunchKernelGGL(k_kp1_scatter, dim3(ntile), dim3(KT_T), 0, st, rec.p, nrec.p, (int64_t)R, b1, ntile,
                               toff.p, r1.p, s1.p);
            const size_t lds2 = (size_t)KP2_T * sizeof(int64_t) + (size_t)nf * sizeof(uint32_t);
            MR_TRY(eslot.alloc(ctx, (size_t)T));
            hipLaunchKernelGGL(k_kp2, dim3(nbk), dim3(KP2_T), lds2, st, r1.p, s1.p, toff.p, pb, b1, ntile, e.p, eslot.p,
                               pstart.p);
            MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // (the level-1 buffers leave scope)
        }
        hipLaunchKernelGGL(k_kind_part, dim3((uint32_t)P), dim3(KP_B), 0, st, pstart.p, e.p, g->flag.p,
                           cursor ? nullptr : eslot.p, rec.p);
        // the classes: through rpos into e (cursor form) or in block order in rec (two-pass form)
        const int32_t* rp = cursor ? rpos.p : nullptr;
        const KRec* cls = cursor ? e.p : rec.p;
        if (u16)
            hipLaunchKernelGGL(k_kind_final<uint16_t>, dim3(cdiv(T, 256)), dim3(256), 0, st, rec_of.p, rp, cls, koff,
                               (const uint16_t*)g->rs16.p, g->w_t.p, T, g->kind.p, g->flag.p, g->krep.p);
        else
            hipLaunchKernelGGL(k_kind_final<int32_t>, dim3(cdiv(T, 256)), dim3(256), 0, st, rec_of.p, rp, cls, koff,
                               kops, g->w_t.p, T, g->kind.p, g->flag.p, g->krep.p);
        MR_DEBUG_CHECK(ctx, "k_kind_part");
    }
    return MR_OK;
}

// algorithmic bytes of one iteration of one graph: op ids once, offsets, the
// r/v/len_t streams, call edges and three N-vectors; o = 4-byte offsets below 2^31 nonzeros
static double iter_bytes(const mr_graph* g, bool fp32) {
    const double w = fp32 ? 4.0 : 8.0, o = g->nnz_sr < (1ll << 31) ? 4.0 : 8.0;
    return 4.0 * (double)g->nnz_sr + o * ((double)g->T + 1) + 4.0 * w * (double)g->T + (8.0 + w) * (double)g->E +
           3.0 * w * (double)g->N;
}

// one attempt with kind-hash seed `seed`; *collided reports a 64-bit key collision found by the
// exact verification (k_kind_verify / k_sh_kind_check), after which the caller retries
// MR_PR_HOST_TIMING: host wall time of pagerank_attempt's phases (no syncs added; diagnostics only)
struct HostMarks {
    bool on = getenv("MR_PR_HOST_TIMING") != nullptr;
    int ng;
    std::vector<std::pair<const char*, std::chrono::steady_clock::time_point>> m;
    explicit HostMarks(int n) : ng(n) { mark("start"); }
    void mark(const char* name) {
        if (on) m.emplace_back(name, std::chrono::steady_clock::now());
    }
    ~HostMarks() {
        if (m.size() < 2) return;
        fprintf(stderr, "[pagerank host ng=%d]", ng);
        for (size_t i = 1; i < m.size(); ++i)
            fprintf(stderr, " %s %.1f", m[i].first, std::chrono::duration<double, std::micro>(m[i].second - m[i - 1].second).count());
        fprintf(stderr, " us\n");
    }
};
struct PrAsync {   // (mr_internal.h) what an enqueued batch's kernels still read, and its error words
    std::vector<unsigned char> setup_h;
    DBuf<SDev> setup_d;
    std::vector<GDev> hv;
    DBuf<GDev> dv;
    DBuf<int32_t> fl;
    hipEvent_t ev = nullptr;
    int32_t* hflag = nullptr;   // pinned, 4 per graph
    std::vector<int> anomaly;
    int ng = 0;
    bool defer = false;         // the words' copy waits for mr_pagerank_async_commit
    bool committed = false;     // the words' copy and the event are enqueued
    ~PrAsync() {
        if (ev) (void)hipEventDestroy(ev);
    }
};
static int pagerank_attempt(mr_ctx* ctx, mr_graph* const* gs, const int* anomaly, int ng, double d, double alpha,
                            int iters, int precision, uint32_t flags, bool sharded, uint64_t seed, uint64_t hmask,
                            bool* collided, PrAsync* as = nullptr) {
    *collided = false;
    HostMarks hm(ng);
    if (!ctx || ng <= 0 || !gs || !anomaly) return mr_fail(ctx, MR_ERR_ARG, "mr_pagerank: bad arguments");
    if (iters < 0) return mr_fail(ctx, MR_ERR_ARG, "iters < 0");
    for (int i = 0; i < ng; ++i) {
        if (!gs[i] || gs[i]->ctx != ctx) return mr_fail(ctx, MR_ERR_STATE, "mr_pagerank: bad handles");
        // np.amax of an empty vector (pagerank.py:126-127); a shard tests the whole graph's traces,
        // so a rank whose shard is empty still joins every collective of the call
        const int64_t T = sharded ? gs[i]->T_all : (int64_t)gs[i]->T;
        if (gs[i]->N == 0 || T == 0)
            return mr_fail(ctx, MR_ERR_VALUE, "zero-size array to reduction operation maximum which has no identity");
    }
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const bool fp32 = precision == MR_FP32;
    FxPlan plan = fx_plan(gs, ng);
    std::vector<unsigned char> setup_h;   // (batched set-up descriptors: alive until the call's final sync)
    DBuf<SDev> setup_d;
    {   // set-up of every graph not set up ahead (mr_pagerank_presetup): batched when they allow it
        std::vector<mr_graph*> need;
        std::vector<int> need_a;
        bool batch = !sharded && getenv("MR_NO_SETUP_BATCH") == nullptr;
        for (int i = 0; i < ng; ++i) {
            mr_graph* g = gs[i];
            const bool pre = g->pre_ok && g->pre_anomaly == anomaly[i] && g->pre_d == d && g->pre_phi == g->phi && g->pre_fp32 == fp32 &&
                             g->pre_flags == flags && g->pre_seed == seed && g->pre_hmask == hmask && !sharded;
            g->pre_ok = false;   // the iteration state is consumed by this call
            if (pre) continue;
            need.push_back(g);
            need_a.push_back(anomaly[i]);
            batch = batch && setup_batchable(g, flags);
        }
        if (batch && need.size() >= 2) {
            MR_TRY(pagerank_setup_batch(ctx, need.data(), need_a.data(), (int)need.size(), d, fp32, seed, hmask,
                                        setup_h, setup_d));
        } else {
            for (size_t j = 0; j < need.size(); ++j)
                MR_TRY(pagerank_setup(ctx, need[j], need_a[j], d, fp32, flags, sharded, seed, hmask));
        }
    }
    hm.mark("setup");
    {   // window batches: the next launch's blocks finish an iteration (k_tr_a pf), no k_fx_b between
        // launches -- every graph fused and plain (no multiplicities, cold sums, merged runs, hot
        // ops or relabelling), N <= PF_NMAX (three N-word LDS arrays, four blocks per CU).
        // MR_TR_PF=0 (read per call; A/B and tests): k_fx_b every iteration
        const char* pe = getenv("MR_TR_PF");
        plan.pf = !(pe && atoi(pe) == 0) && !sharded && ng >= 2 && plan.NT == 512 && plan.mode == WV_SU_ALL;
        for (int i = 0; i < ng && plan.pf; ++i) {
            const mr_graph* g = gs[i];
            plan.pf = g->fused && !g->wide && !g->relabeled && !g->nhr && !g->mw_tp.p && kern_n(g) <= PF_NMAX &&
                      !(g->lo && g->lo_merged == 1);
        }
    }
    {   // fp32 wide graphs: su as floats in k_tr_a's LDS, the freed half holding the next ~10k
        // ("warm") labels' su, so their cold entries read LDS instead of L2 (k_tr_a EXT & 8);
        // every fused graph of the launch wide and plain (no multiplicities)
#ifndef MR_AB_NO_W32
        plan.w32 = fp32 && plan.mode == WV_SU_ALL && !plan.pf;
#endif
        bool anyf = false;
        for (int i = 0; i < ng && plan.w32; ++i)
            if (gs[i]->fused) {
                anyf = true;
                plan.w32 = gs[i]->wide && !gs[i]->mw_tp.p && !gs[i]->trun.p;
            }
        plan.w32 = plan.w32 && anyf;
    }
    int64_t wsum = 0;   // wave tiles of the launch's fused graphs (k_tr_a's block budget)
    for (int i = 0; i < ng; ++i)
        if (gs[i]->fused) wsum += gs[i]->n_wt;
    std::vector<CutArg> cuts;   // the graphs' per-wave cuts, launched together
    const std::vector<int64_t> nbs = batch_blocks(gs, ng, plan, wsum);
    for (int i = 0; i < ng; ++i) {
        mr_graph* g = gs[i];
        if (g->fused) {   // the plan's blocks: partial rows and (k_tr_a) the per-wave cut
            int64_t nfa = 0;
            MR_TRY(fused_blocks(ctx, g, plan, wsum, &nfa, &cuts, nbs.empty() ? 0 : nbs[(size_t)i]));
            // (pf: rows and call-graph terms double-buffered, iteration it & 1)
            MR_TRY(g->fx_part.alloc(ctx, (size_t)(plan.pf ? 2 : 1) * std::max<int64_t>(nfa, 1) * (size_t)kern_n(g)));
            if (plan.pf) MR_TRY(g->fx_ssv.alloc(ctx, 2 * (size_t)g->N));
        }
    }
    hm.mark("blocks");
    for (size_t c0 = 0; c0 < cuts.size(); c0 += TC_BATCH) {
        CutBatch cb;
        const size_t n = std::min<size_t>(TC_BATCH, cuts.size() - c0);
        for (size_t j = 0; j < n; ++j) cb.a[j] = cuts[c0 + j];
        hipLaunchKernelGGL(k_tr_cut_b, dim3((unsigned)n), dim3(TC_T), 0, st, cb);
        MR_TRY_HIP(ctx, hipGetLastError());
    }
    // a sharded wide graph: the widest cold slice span over the ranks (one scale for every rank)
    uint64_t cold_span_all = 1;
    for (int i = 0; i < ng; ++i)
        if (gs[i]->wide) cold_span_all = std::max(cold_span_all, gs[i]->cold_span);
    if (sharded && mr_coll_ready(ctx)) {
        DBuf<uint64_t> csp;
        MR_TRY(csp.upload(ctx, &cold_span_all, 1));
        MR_TRY(mr_coll_allreduce(ctx, csp.p, 1, MR_DT_U64, 1));
        MR_TRY(csp.download(ctx, &cold_span_all, 1));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    }
    // ---- batched power iteration: one k_iter_a + k_iter_b pair per iteration for every graph
    std::vector<GDev> hv((size_t)ng);
    int64_t fb16 = 0;   // k_fx_b blocks of the launch at 16 ops per block
    for (int i = 0; i < ng; ++i)
        if (gs[i]->fused) fb16 += cdiv(gs[i]->N, 16);
    const bool fb_many = fb16 > FB_MANY_BLOCKS;
    int32_t blocks_a = 0, blocks_b = 0, blocks_fa = 0, blocks_fb = 0;
    size_t lds = VCAP * sizeof(double), lds_f = 0;
    const char* lfe = getenv("MR_TR_LASTFIN");   // (A/B and tests, read per call) 0: k_fx_b for every graph
    const bool lastfin_on = !(lfe && atoi(lfe) == 0);
    const char* sve = getenv("MR_TR_SSV");   // (A/B and tests, read per call) 0: k_fx_b computes the call-graph terms
    const bool ssv_on = !(sve && atoi(sve) == 0);
    const char* lse = getenv("MR_TR_LFSSV");   // (A/B and tests, read per call)
    const bool lfssv_on = !(lse && atoi(lse) == 0);
    // (A/B, read per call) 0: plain partial-row stores.  Write-through measured C4 rank 0 of 8: 43.1
    // vs 44.6 us per iteration, C4 whole: within noise (two repeats each)
    const char* rwe = getenv("MR_TR_ROW_WT");
    const bool row_wt_on = !(rwe && atoi(rwe) == 0);
    double bytes = 0.0;
    for (int i = 0; i < ng; ++i) {
        mr_graph* g = gs[i];
        GDev& v = hv[(size_t)i];
        v.rs_off = g->rs_off.p;
        v.rs_ops = g->rs_ops.p;
        v.rs16 = g->rs16.p;
        v.rsw = g->relabeled ? g->rsp.p : g->rs16.p;
        v.perm = g->relabeled ? g->perm.p : nullptr;
        v.n_hot = plan_n_hot(kern_n(g), plan);
        v.tids = g->tids.p;
        v.coff = g->coff.p;
        v.wtile = g->wtile.p;
        v.c_tp = g->c_tp.p;
        v.w_tp = g->w_tp.p;
        v.mw_tp = g->mw_tp.p;
        v.hmask = g->nhr ? g->hmask.p : nullptr;
        v.trun = g->lo && g->lo_merged == 1 ? g->trun.p : nullptr;   // (set at prepare: the ids' rotation follows it)
        v.ctids = g->wide ? g->ctids.p : nullptr;
        v.ccoff = g->wide ? g->ccoff.p : nullptr;
        v.nhr = g->fused ? g->nhr : 0;
        for (int h = 0; h < 8; ++h) v.hop[h] = g->hop[h];
        v.c_t = g->c_t.p;
        v.w_t = g->w_t.p;
        v.u_o = g->u_o.p;
        v.pw = g->pw.p;
        v.ltr = g->tl_ltr.p;
        v.pr_beg = g->pr_beg.p;
        v.tile_pr0 = g->tile_pr0.p;
        v.lp = g->lp.p;
        v.tile_lp0 = g->tile_lp0.p;
        v.op_pr_off = g->op_pr_off.p;
        v.op_pr = g->op_pr.p;
        v.ss_off = g->ss_off.p;
        v.ss_par = g->ss_par.p;
        for (int j = 0; j < 2; ++j) {
            v.q[j] = fp32 ? (void*)g->q32[j].p : (void*)g->q64[j].p;
            v.sub[j] = g->sub[j].p;
            v.suf[j] = g->suf[j].p;
            v.spb[j] = g->spb[j].p;
        }
        v.part = g->part.p;
        v.mslot = g->mslot.p;
        v.sn = g->sn.p;
        v.weight = g->weight.p;
        v.scal = g->scal.p;
        v.flag = g->flag.p;
        v.fx_part = (unsigned long long*)g->fx_part.p;
        v.fx_ssv = g->fx_ssv.p;
        v.fx_limb = (unsigned long long*)g->fx_limb.p;
        v.op_sum = g->op_sum.p;
        v.rank = ctx->rank;
        v.nranks = ctx->nranks;
        // a shard without traces still runs one (empty) block: it clears the maxima slot and
        // writes a zero partial row, and the collectives after the launch need every rank
        int64_t nfa = 0;
        if (g->fused) MR_TRY(fused_blocks(ctx, g, plan, wsum, &nfa, nullptr, nbs.empty() ? 0 : nbs[(size_t)i]));
        nfa = g->fused ? std::max<int64_t>(nfa, sharded ? 1 : 0) : 0;
        // a row entry stays below 2^64 (traces per block < 2^(64-sc)).  Shards of one graph hold
        // different trace counts and their limbs are summed, so they share one scale, 2^48 (<= 65535
        // traces per block: wv_blocks / fx_blocks); window graphs take their cut-independent scale
        // (tr_scfix); a graph cut on the device carries its scale there (dscale)
        const int64_t tpb = g->fused ? g->wtile_msum : 0;
        const int sc = sharded ? 48 : tr_scfix(g) > 0 ? tr_scfix(g) : 64 - bits_for((uint64_t)std::max<int64_t>(tpb, 1));
        v.alpha = alpha;
        v.fx_scale = std::ldexp(1.0, sc);
        v.fx_iscale = std::ldexp(1.0, -sc);
        v.T = g->T;
        v.N = g->N;
        v.NA = kern_n(g);
        v.cold_rw = g->cold_rw;
        v.ns_warm = plan.w32 ? v.NA + std::min(TrLds(v.NA, WV_SU_ALL, false, true).n_warm, g->N - v.NA) : v.NA;
        v.su32 = fp32 && g->wide;
        v.cold_acc = g->wide ? g->cold_acc.p : nullptr;
        v.cold_part = (const unsigned long long*)g->cold_part.p;
        v.cold_rowbase = g->cold_rowbase.p;
        v.cx_scale = v.fx_scale;
        v.cx_iscale = v.fx_iscale;
        // the graph's scale on the device (k_tr_cut) unless the ranks share the fixed one
        v.dscale = (!sharded && g->fused && g->wtile_msum < 0) ? g->dscale.p : nullptr;
        if (g->wide) {
            // cold rows: at most cold_span adds per op and row; a sharded graph's ranks sum their
            // limbs per op, and an op hot on one rank may be cold on another: one scale for both
            // (the smaller), agreed over the ranks (cold_span_all)
            const int scc = 64 - bits_for(sharded ? cold_span_all : g->cold_span);
            if (sharded) {
                const int s1 = std::min(sc, scc);
                v.fx_scale = v.cx_scale = std::ldexp(1.0, s1);
                v.fx_iscale = v.cx_iscale = std::ldexp(1.0, -s1);
            } else {
                v.cx_scale = std::ldexp(1.0, scc);
                v.cx_iscale = std::ldexp(1.0, -scc);
            }
        }
        v.blk0f = blocks_fa;
        v.n_fa = (int32_t)nfa;
        blocks_fa += v.n_fa;
        v.blk0fb = blocks_fb;
        v.fb_ops = fb_ops(g->N, fb_many);
        // the last k_tr_a block finishes small graphs itself (window batches: one launch per
        // iteration); its sc1 row reads stay short: at most LASTFIN_WORDS row words
        // (ops <= threads: the finishing block takes every op in one round -- C3's 500-op windows;
        // C2's 1000-op windows measured -1.5 % with it, C3 +6.5 % windows/s, -7 % single window)
        v.lastfin = lastfin_on && plan.NT == 512 && !sharded && g->fused && !g->wide && !g->relabeled &&
                    plan.mode == WV_SU_ALL && nfa >= 1 && g->N <= plan.NT && nfa * (int64_t)g->N <= LASTFIN_WORDS;
        v.n_fb = g->fused && !v.lastfin ? cdiv(g->N, v.fb_ops) : 0;
        // the call-graph terms in k_tr_a (large graphs: k_fx_b's chains of dependent loads leave its
        // critical path; not for wide graphs: k_fx_b's columns past NA).  Last-block graphs: every
        // block writes its share write-through and the last block reads the terms with one load per
        // op instead of the ss_off -> ss_par -> pw / s_k chain (MR_TR_LFSSV=0: the chain; read per call)
        v.ssv_pre = ssv_on && nfa >= 1 && !g->wide && ((v.n_fb > 0 && g->N >= 2048) || (v.lastfin && lfssv_on));
        v.pf = plan.pf && !v.lastfin && nfa <= PF_ROWS;
        v.pf_stride = nfa * (int64_t)kern_n(g);
        if (v.pf) v.ssv_pre = 1;   // (the next launch's prologue reads the terms: one load per op)
        v.row_wt = row_wt_on && g->N >= 2048;
        blocks_fb += v.n_fb;
        v.blk0 = blocks_a;
        v.blk0b = blocks_b;
        bytes += iter_bytes(g, fp32);
        if (g->fused) {
            continue;   // no tile-path blocks (n_tb = n_tiles = n_ob = 0)
        }
        v.n_tb = std::max(cdiv(g->T, TB), sharded ? 1 : 0);   // (empty shard: see nfa)
        v.n_tiles = g->n_tiles;
        v.tshift = g->tshift;
        v.lds_su = g->N <= LDS_NODES;
        blocks_a += v.n_tb + v.n_tiles;
        v.n_ob = cdiv(g->N, TB / WAVE);
        blocks_b += v.n_ob;
        if (v.lds_su) lds = std::max(lds, ((size_t)g->N + VCAP) * sizeof(double));
        lds = std::max(lds, ((size_t)1 << g->tshift) * (fp32 ? sizeof(float) : sizeof(double)));
    }
    const int32_t split_fa = ng == 2 ? hv[1].blk0f : 0, split_fb = ng == 2 ? hv[1].blk0fb : 0;
    for (int i = 0; i < ng; ++i)
        if (gs[i]->fused) lds_f = std::max(lds_f, plan_lds(kern_n(gs[i]), plan));
    {   // last-block graphs: a launch that fits one block per CU runs so (LDS past half a CU), and its
        // finishing blocks skip the acquire (tr_last_finish); else they take it
        bool any_lf = false;
        for (int i = 0; i < ng; ++i) any_lf = any_lf || hv[(size_t)i].lastfin;
        const bool one_cu = LF_ONE_CU_LDS > 0 && any_lf && blocks_fa <= num_cus() && LF_ONE_CU_LDS <= WV_LDS_MAX;
        if (one_cu) lds_f = std::max(lds_f, LF_ONE_CU_LDS);
        for (int i = 0; i < ng; ++i) hv[(size_t)i].lf_acq = one_cu ? 0 : 1;
    }
    for (int i = 0; i < ng; ++i)   // hot-op layouts need every op's su in LDS (a batch with a much wider graph)
        if (gs[i]->fused && gs[i]->nhr && plan.mode != WV_SU_ALL)
            return mr_fail(ctx, MR_ERR_ARG, "pagerank batch: a hot-op layout (T >= MR_TR_HOT_MIN) with a graph of > %d ops",
                           (int)WIDE_NA);
    int any_ext = 0;   // kind multiplicities (1), cold sums (2) or merged runs (4) in some fused graph of the launch
    for (int i = 0; i < ng; ++i)
        if (gs[i]->fused)
            any_ext |= (hv[(size_t)i].mw_tp ? 1 : 0) | (hv[(size_t)i].cold_acc ? 2 : 0) | (hv[(size_t)i].trun ? 4 : 0);
    if ((any_ext & 4) && (any_ext & 3)) any_ext &= 3;   // (not built: such a launch walks every trace)
    for (int i = 0; i < ng; ++i)   // the wide variant carries HOT_MAX_WIDE hot accumulators
        if ((any_ext & 2) && gs[i]->fused && gs[i]->nhr > HOT_MAX_WIDE)
            return mr_fail(ctx, MR_ERR_ARG, "pagerank batch: a hot-op layout of %d ops beside a wide graph", gs[i]->nhr);
    bool launch_pf = plan.pf;   // every graph finishes in-kernel: no k_fx_b before the last iteration
    for (int i = 0; i < ng; ++i) launch_pf = launch_pf && (hv[(size_t)i].lastfin || hv[(size_t)i].pf);
    launch_pf = launch_pf && any_ext == 0;
    if (!launch_pf)
        for (int i = 0; i < ng; ++i) {
            if (hv[(size_t)i].pf) hv[(size_t)i].ssv_pre = ssv_on && !gs[i]->wide && gs[i]->N >= 2048;
            hv[(size_t)i].pf = 0;
        }
    const TrA tr_a = tr_kernel(fp32, plan.mode, plan.NT, any_ext == 2 && plan.w32 ? 10 : any_ext);
    DBuf<GDev> dv;
    hm.mark("descr");
    MR_TRY(dv.upload(ctx, hv.data(), hv.size()));
    // a sharded graph with no collective backend is one whole shard: the split launches around the
    // (no-op) all-reduces would compute the same integers / sums in two halves
    const bool coll = sharded && mr_coll_ready(ctx);
    // wide graphs: k_cold_ops (LDS-bound) runs on the side stream beside k_cold_trace (L2-gather
    // bound) and k_tr_a on the main stream; k_fx_b waits for both
    bool any_wide = false;
    for (int i = 0; i < ng; ++i) any_wide = any_wide || gs[i]->wide;
    // k_fx_b's block size: 4 waves when no graph of the launch has many partial rows
    bool fb_small = !any_wide;
    // (a large graph alone -- C4: 256 rows of 10k ops -- sums faster with 16-wave blocks: 137 -> 134 us)
    for (int i = 0; i < ng; ++i) fb_small = fb_small && hv[(size_t)i].n_fa <= FB_SMALL_ROWS && hv[(size_t)i].N <= 4096;
    hipStream_t sst = st;
#ifdef MR_AB_WIDE_SERIAL   // (A/B builds: k_cold_ops on the main stream)
    if (false) {
#else
    if (any_wide) {
#endif
        if (!ctx->side) {
            MR_TRY_HIP(ctx, hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
            for (hipEvent_t& e : ctx->side_ev) MR_TRY_HIP(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        sst = ctx->side;
    }
    // sharded fused graph on the peer path: the exchange inside k_fx_b (MR_PEER_SPLIT=1: the separate
    // push / reduce launches; relabelled graphs always -- the ranks' op labels differ, so a block's
    // columns on one rank are not the same ops on another)
    MrPeerX px{}, px_off{};
    bool px_on = false;
    if (coll && ng == 1 && gs[0]->fused && !gs[0]->wide && !gs[0]->relabeled && mr_peer_ready(ctx) &&
        !getenv("MR_PEER_SPLIT")) {
        const int prc = mr_peer_fx_prepare(ctx, 2 * (int64_t)gs[0]->N + ctx->nranks, (int32_t)blocks_fb, &px);
        if (prc == MR_OK) {
            px_on = true;
            // ranks sharing a device: mode-2 blocks spinning there would hold CUs a peer's 160-KB
            // k_tr_a blocks need -- one waiting block instead (MR_PEER_SPIN=0/1 forces it)
            const char* se = getenv("MR_PEER_SPIN");
            px.spin = se ? atoi(se) != 0 : !mr_peer_same_device(ctx);
        } else if (prc != MR_ERR_STATE) {
            return prc;
        }
    }
    hm.mark("pre-loop");
    for (int it = 0; it < iters; ++it) {
        mr_prof_begin(ctx);
        if (any_wide && sst != st) {
            MR_TRY_HIP(ctx, hipEventRecord(ctx->side_ev[0], st));   // this iteration's su and q are ready
            MR_TRY_HIP(ctx, hipStreamWaitEvent(sst, ctx->side_ev[0], 0));
        }
        for (int i = 0; i < ng; ++i) {   // wide graphs: the cold halves, before k_tr_a / k_fx_b
            mr_graph* g = gs[i];
            if (!g->wide) continue;
            const void* qc = fp32 ? (const void*)g->q32[it & 1].p : (const void*)g->q64[it & 1].p;
            const size_t lds_c = (size_t)g->cold_rw * sizeof(unsigned long long);
            if (fp32)
                hipLaunchKernelGGL(k_cold_ops<float>, dim3(g->n_cb), dim3(WIDE_CT), lds_c, sst, g->cb_beg.p, g->cp_pos.p,
                                   g->cp_op.p, qc, g->mslot.p, it, hv[(size_t)i].cx_scale, g->cold_rw,
                                   (unsigned long long*)g->cold_part.p);
            else
                hipLaunchKernelGGL(k_cold_ops<double>, dim3(g->n_cb), dim3(WIDE_CT), lds_c, sst, g->cb_beg.p, g->cp_pos.p,
                                   g->cp_op.p, qc, g->mslot.p, it, hv[(size_t)i].cx_scale, g->cold_rw,
                                   (unsigned long long*)g->cold_part.p);
            if (g->n_ctl)   // (the listed tiles only: the short-tile walk gathers the rest itself)
                hipLaunchKernelGGL(k_cold_trace, dim3(cdiv((int64_t)g->n_ctl * WAVE, 256)), dim3(256), 0, st,
                                   g->cold_off_p.p, g->cold_ops_p.p, g->sub[it & 1].p, g->ctl.p, g->n_ctl, g->T,
                                   g->cold_acc.p);
            MR_DEBUG_CHECK(ctx, "k_cold");
        }
        if (any_wide && sst != st) MR_TRY_HIP(ctx, hipEventRecord(ctx->side_ev[1], sst));
        if (blocks_fa) {
            hipLaunchKernelGGL(tr_a, dim3(blocks_fa), dim3(plan.NT), lds_f, st, dv.p, ng, split_fa, d, alpha, it, 0);
            MR_DEBUG_CHECK(ctx, "k_tr_a");
            if (any_wide && sst != st) MR_TRY_HIP(ctx, hipStreamWaitEvent(st, ctx->side_ev[1], 0));   // k_cold_ops done
            auto fx_b = [&](int mode, const MrPeerX& p) {
                if (fb_small)
                    hipLaunchKernelGGL(k_fx_b<FB_W_SMALL>, dim3(blocks_fb), dim3(WAVE * FB_W_SMALL), 0, st, dv.p, ng,
                                       split_fb, d, it, mode, p);
                else
                    hipLaunchKernelGGL(k_fx_b<FB_W>, dim3(blocks_fb), dim3(WAVE * FB_W), 0, st, dv.p, ng, split_fb, d,
                                       it, mode, p);
            };
            if (!coll) {
                // (none: every graph finished by its last k_tr_a block; pf launches: the next k_tr_a
                // finishes this iteration, k_fx_b only after the last one)
                if (blocks_fb && (!launch_pf || it == iters - 1)) fx_b(0, px_off);
            } else if (px_on) {   // the exchange fused into k_fx_b: push in mode 1, per-block waits in mode 2
                fx_b(1, px);
                if (!px.spin) MR_TRY(mr_peer_fx_wait(ctx, px, blocks_fb));
                fx_b(2, px);
                mr_peer_fx_round_done(ctx, &px);
            } else {   // ONE all-reduce: the P_sr r limbs and every rank's r' max (exact: integers)
                fx_b(1, px_off);
                const int64_t nw = 2 * (int64_t)gs[0]->N + ctx->nranks;
                const int prc = mr_peer_allreduce_u64(ctx, (unsigned long long*)gs[0]->fx_limb.p, nw);
                if (prc == MR_ERR_STATE) MR_TRY(mr_coll_allreduce(ctx, gs[0]->fx_limb.p, nw, MR_DT_U64, 0));
                else MR_TRY(prc);
                fx_b(2, px_off);
            }
            MR_DEBUG_CHECK(ctx, "k_fx_b");
        }
        if (blocks_a) {
            if (fp32) hipLaunchKernelGGL(k_iter_a<float>, dim3(blocks_a), dim3(TB), lds, st, dv.p, ng, d, it);
            else hipLaunchKernelGGL(k_iter_a<double>, dim3(blocks_a), dim3(TB), lds, st, dv.p, ng, d, it);
            MR_DEBUG_CHECK(ctx, "k_iter_a");
        }
        if (blocks_b) {
            if (!coll) {
                hipLaunchKernelGGL(k_iter_b, dim3(blocks_b), dim3(TB), 0, st, dv.p, ng, d, alpha, it, 0);
            } else {   // ONE all-reduce: the per-op P_sr r sums (fp64 SUM) and every rank's r' max
                hipLaunchKernelGGL(k_iter_b, dim3(blocks_b), dim3(TB), 0, st, dv.p, ng, d, alpha, it, 1);
                const int64_t nw = (int64_t)gs[0]->N + ctx->nranks;
                const int prc = mr_peer_allreduce_f64(ctx, gs[0]->op_sum.p, nw);
                if (prc == MR_ERR_STATE) MR_TRY(mr_coll_allreduce(ctx, gs[0]->op_sum.p, nw, MR_DT_F64, 0));
                else MR_TRY(prc);
                hipLaunchKernelGGL(k_iter_b, dim3(blocks_b), dim3(TB), 0, st, dv.p, ng, d, alpha, it, 2);
            }
            MR_DEBUG_CHECK(ctx, "k_iter_b");
        }
        mr_prof_end(ctx, bytes);
    }
    // weights of every graph and the gathered error words in one launch (the flags are final:
    // the kernels that raise them ran before the iterations; a sharded graph's words meet in a
    // MAX first, below, so it reads them after that)
    DBuf<int32_t> fl;
    MR_TRY(fl.alloc(ctx, (size_t)4 * ng));
    hm.mark("loop");
    hipLaunchKernelGGL(k_weights_batch, dim3(ng), dim3(1024), 0, st, dv.p, iters, (int)((flags & MR_PR_EXACT_SUMS) != 0),
                       fl.p);
    MR_DEBUG_CHECK(ctx, "k_weights");
    MR_TRY_HIP(ctx, hipGetLastError());
    if (coll && ctx->peer_on) MR_TRY(mr_peer_check(ctx, "peer all-reduce"));   // an error, not wrong sums
    // a shard's local collision must make every rank retry: the error words meet in a MAX
    if (coll) {
        MR_TRY(mr_coll_allreduce(ctx, gs[0]->flag.p, 4, MR_DT_I32, 1));
        MR_TRY_HIP(ctx, hipMemcpyAsync(fl.p, gs[0]->flag.p, 4 * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    }
    if (as) {   // enqueued only: the words go to the caller's pinned slot, the finish reads them
        as->setup_h = std::move(setup_h);
        as->setup_d.swap(setup_d);
        as->hv = std::move(hv);
        as->dv.swap(dv);
        as->fl.swap(fl);
        as->anomaly.assign(anomaly, anomaly + ng);
        as->ng = ng;
        return as->defer ? MR_OK : mr_pagerank_async_commit(ctx, as);
    }
    // the only host round trip of the call: error words raised by the kernels (one pinned read)
    std::vector<int32_t> hflag((size_t)4 * ng, 0);
    if ((size_t)4 * ng * sizeof(int32_t) <= MR_PIN_BYTES) {
        unsigned char* hp = nullptr;
        MR_TRY(mr_read_bytes(ctx, fl.p, (size_t)4 * ng * sizeof(int32_t), &hp));
        memcpy(hflag.data(), hp, hflag.size() * sizeof(int32_t));
    } else {
        MR_TRY(fl.download(ctx, hflag.data(), hflag.size()));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    }
    for (int i = 0; i < ng; ++i) {
        if (hflag[(size_t)4 * i] & 1) {
            *collided = true;
            return MR_OK;
        }
        if (hflag[(size_t)4 * i + 2] & 1) return mr_fail(ctx, MR_ERR_STATE, "trace kinds: a partition exceeded its table");
        if (anomaly[i] && (hflag[(size_t)4 * i + 1] & 1)) return mr_fail(ctx, MR_ERR_ZERODIV, "float division by zero");
    }
    return MR_OK;
}

// A 64-bit set-hash collision between two different trace kinds is caught by the exact
// verification; the whole call then reruns with the next seed (independent hash functions), so
// an input that collides under one seed is still ranked.  Seeds are a fixed sequence: every rank
// of a sharded graph takes the same one.
static uint64_t kind_seed(int a) {
    static const uint64_t seed0 = [] {   // MR_KIND_SEED: test knob (start the sequence elsewhere)
        const char* e = getenv("MR_KIND_SEED");
        return e ? (uint64_t)strtoull(e, nullptr, 0) : 0x5eed5eedull;
    }();
    return seed0 + 0x9E3779B97F4A7C15ull * (uint64_t)a;
}
// MR_KIND_TEST_COLLIDE: test knob -- the first attempt keeps 2 bits of every key, so distinct
// kinds collide and the verification + retry path runs
static uint64_t kind_hmask(int a) { return (a == 0 && getenv("MR_KIND_TEST_COLLIDE") != nullptr) ? 3ull : ~0ull; }

// A graph's kinds, preference and iteration state for its next mr_pagerank(_batch) call with
// these arguments, on THIS context's stream (the one that built it): mr_windows_batch sets up a
// window's graphs while the previous group's iterations run.  The next call on the graph skips
// its own setup when the arguments match (first kind-hash seed; a collision retries in full).
int mr_pagerank_presetup_n(mr_ctx* ctx, mr_graph* const* gs, const int* an, int n, double d, int precision,
                           std::vector<unsigned char>& keep) {
    const bool fp32 = precision == MR_FP32;
    bool batch = n >= 2 && getenv("MR_NO_SETUP_BATCH") == nullptr;
    for (int i = 0; i < n && batch; ++i) batch = gs[i]->N && gs[i]->T && setup_batchable(gs[i], 0);
    if (!batch) {
        for (int i = 0; i < n; ++i) MR_TRY(mr_pagerank_presetup(ctx, gs[i], an[i], d, precision, 0));
        return MR_OK;
    }
    DBuf<SDev> dsd;   // (returns to this context's pool: reused only by later work on this stream)
    MR_TRY(pagerank_setup_batch(ctx, gs, an, n, d, fp32, kind_seed(0), kind_hmask(0), keep, dsd));
    for (int i = 0; i < n; ++i) {
        mr_graph* g = gs[i];
        g->pre_ok = true;
        g->pre_anomaly = an[i];
        g->pre_d = d;
        g->pre_phi = g->phi;
        g->pre_fp32 = fp32;
        g->pre_flags = 0;
        g->pre_seed = kind_seed(0);
        g->pre_hmask = kind_hmask(0);
    }
    return MR_OK;
}

int mr_pagerank_presetup(mr_ctx* ctx, mr_graph* g, int anomaly, double d, int precision, uint32_t flags) {
    const bool fp32 = precision == MR_FP32;
    if (g->N == 0 || g->T == 0) return MR_OK;   // (the call itself raises)
    MR_TRY(pagerank_setup(ctx, g, anomaly, d, fp32, flags, false, kind_seed(0), kind_hmask(0)));
    g->pre_ok = true;
    g->pre_anomaly = anomaly;
    g->pre_d = d;
    g->pre_phi = g->phi;
    g->pre_fp32 = fp32;
    g->pre_flags = flags;
    g->pre_seed = kind_seed(0);
    g->pre_hmask = kind_hmask(0);
    return MR_OK;
}

// ---------------------------------------------------------------- window graphs in layout order
// the iteration state's buffers of a layout-order graph and its LDev set-up fields
static int lo_state(mr_ctx* ctx, mr_graph* g, int anomaly, double d, bool fp32, LDev& v) {
    const int32_t N = g->N, T = g->T;
    MR_TRY(g->flag.alloc(ctx, 8));
    MR_TRY(g->scal.alloc(ctx, 8));
    MR_TRY(g->mslot.alloc(ctx, MSLOT_WORDS));
    MR_TRY(g->sn.alloc(ctx, (size_t)N));
    MR_TRY(g->spb[0].alloc(ctx, (size_t)N));
    MR_TRY(g->spb[1].alloc(ctx, (size_t)N));
    MR_TRY(g->sub[0].alloc(ctx, (size_t)N + TR_PAD));
    MR_TRY(g->sub[1].alloc(ctx, (size_t)N + TR_PAD));
    MR_TRY(g->weight.alloc(ctx, (size_t)N));
    MR_TRY(g->fx_ssv.alloc(ctx, (size_t)N));
    MR_TRY(g->c_tp.alloc(ctx, (size_t)std::max(T, 1)));
    for (int j = 0; j < 2; ++j) {
        if (fp32) MR_TRY(g->q32[j].alloc(ctx, (size_t)T + 1));   // [T]: k_tr_a's pad slot
        else MR_TRY(g->q64[j].alloc(ctx, (size_t)T + 1));
    }
    v.T = T;
    v.N = N;
    v.anomaly = anomaly;
    v.fp32 = fp32 ? 1 : 0;
    v.cd = (float)(1.0 - d);
    v.phi = g->phi;
    v.v0 = 1.0 / (double)((int64_t)N + T);   // pagerank.py:118-119
    v.nbp = g->lo_nbp;
    v.w_tp = g->w_tp.p;
    v.c_tp = g->c_tp.p;
    v.kind = g->kind.p;
    v.lenp = g->lo_lenp.p;
    v.ppart = g->ppart.p;
    v.scal = g->scal.p;
    v.flag = g->flag.p;
    v.mslot = g->mslot.p;
    v.sp0 = g->spb[0].p;
    v.su0 = g->sub[0].p;
    v.su1 = g->sub[1].p;
    v.q64 = g->q64[0].p;
    v.q32 = g->q32[0].p;
    v.u_o = g->u_o.p;
    return MR_OK;
}
static void lo_mark_presetup(mr_graph* g, int anomaly, double d, bool fp32) {
    g->pre_ok = true;
    g->pre_anomaly = anomaly;
    g->pre_d = d;
    g->pre_phi = g->phi;
    g->pre_fp32 = fp32;
    g->pre_flags = 0;
    g->pre_seed = kind_seed(0);
    g->pre_hmask = kind_hmask(0);
}
// pagerank_setup of a layout-order graph (a call that did not take its presetup: a group rerun):
// its kind class sizes, span counts and preference partials by position are kept on the graph
static int lo_setup_one(mr_ctx* ctx, mr_graph* g, int anomaly, double d, bool fp32) {
    std::vector<unsigned char> keep(sizeof(LDev), 0);
    LDev& v = *reinterpret_cast<LDev*>(keep.data());
    MR_TRY(lo_state(ctx, g, anomaly, d, fp32, v));
    v.b_app = 0;
    DBuf<LDev> dl;
    MR_TRY(dl.upload(ctx, &v, 1));
    hipStream_t st = ctx->stream;
    hipLaunchKernelGGL(k_lo_total_b, dim3(1), dim3(1024), 0, st, dl.p);
    const int64_t na = std::max<int64_t>({(int64_t)g->T, (int64_t)g->N + TR_PAD, MSLOT_WORDS, 8});
    hipLaunchKernelGGL(k_lo_apply_b, dim3(cdiv(na, 256)), dim3(256), 0, st, dl.p, 1);
    MR_TRY_HIP(ctx, hipGetLastError());
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // (the host descriptor leaves scope)
    return MR_OK;
}

int mr_lo_prepare_batch(mr_ctx* ctx, mr_graph* const* gs, const mr_spans* const* sps, IxBuild* const* bs,
                        const int* anomaly, int n, double d, int precision, std::vector<unsigned char>& keep) {
    if (n <= 0) return MR_OK;
    const bool fp32 = precision == MR_FP32;
    hipStream_t st = ctx->stream;
    // a trace's ids rotated by its layout index mod length (spreads a shared first op over a tile's
    // id chunks, k_lo_fill_b).  MR_TR_MERGE=1 (read per call; the bench's run-merged side leg and
    // tests): runs of identical traces share their head's rotation and k_tr_a walks each run by its
    // head -- kind compression inside the walk, so never the default: the headline
    // walks every trace.  MR_TR_MERGE=2 (tests): the run rotations without the merged walk, so every
    // lane walks its own trace in its run head's order -- bitwise the merged walk
    const char* mge = getenv("MR_TR_MERGE");
    const int merge = mge ? std::min(std::max(atoi(mge), 0), 2) : 0;
    keep.assign((size_t)n * sizeof(LDev), 0);
    LDev* hv = reinterpret_cast<LDev*>(keep.data());
    std::vector<DBuf<int64_t>> c64((size_t)n);
    int32_t bcs = 0, bfl = 0, bap = 0;
    int64_t st_words = 0;
    for (int i = 0; i < n; ++i) {
        mr_graph* g = gs[i];
        const mr_spans* sp = sps[i];
        const IxBuild& b = *bs[i];
        const int32_t N = g->N, T = g->T, W = cdiv(T, WAVE);
        const int64_t nnz = g->nnz_sr;
        if (N <= 0 || T <= 0 || N > FX_NMAX || !TrLds(N, WV_SU_ALL).su_lds || nnz >= (1ll << 31))
            return mr_fail(ctx, MR_ERR_STATE, "mr_lo_prepare_batch: graph outside the layout-order limits");
        g->lo = true;
        g->rs_is_sr = true;
        g->pr_identity = true;
        g->n_pr = T;
        g->traces_nonempty = true;
        g->cov_ready = true;
        g->nhr = 0;
        g->hmask.reset();
        g->relabeled = false;
        g->wide = false;
        g->NA = N;
        g->fused = true;
        g->perm.reset();
        g->rsp.reset();
        g->n_wt = W;
        g->wtile_nw = 0;
        g->coff_h.clear();
        g->n_tiles = 0;
        g->n_pairs = 0;
        g->tpos_ok = false;
        g->lo_nbp = cdiv((int64_t)W * WAVE, 256);
        MR_TRY(g->w_tp.alloc(ctx, (size_t)T));
        MR_TRY(g->kind.alloc(ctx, (size_t)T));
        MR_TRY(g->lo_lenp.alloc(ctx, (size_t)T));
        g->lo_merged = merge;
        if (merge) MR_TRY(g->trun.alloc(ctx, (size_t)T));
        MR_TRY(g->ppart.alloc(ctx, 2 * (size_t)g->lo_nbp));
        MR_TRY(g->coff.alloc(ctx, (size_t)W + 1));
        MR_TRY(c64[(size_t)i].alloc(ctx, (size_t)W + 1));
        const int64_t nch = 2 * (int64_t)W + (nnz / WAVE + 2 * (int64_t)N) / 4 + 2;   // as tr_layout
        MR_TRY(g->tids.alloc(ctx, (size_t)std::max<int64_t>(nch, 1) * WAVE * 4));
        LDev& v = hv[i];
        MR_TRY(lo_state(ctx, g, anomaly[i], d, fp32, v));
        v.W = W;
        v.NP = sp->n_podops;
        v.n_cs = (int32_t)std::max<int64_t>(cdiv((int64_t)W, TS_TILE), 1);
        v.st_off = st_words;
        st_words += v.n_cs;
        v.b_cs = bcs;
        bcs += v.n_cs;
        v.b_fill = bfl;
        bfl += g->lo_nbp;
        v.b_app = bap;
        bap += cdiv(std::max<int64_t>({(int64_t)T, (int64_t)N + TR_PAD, MSLOT_WORDS, 8}), 256);
        v.pinv = b.pinv.p;
        v.lo_off = sp->lo_off.p;
        v.lo16 = sp->lo16.p;
        v.lo_len = sp->lo_len.p;
        v.lo_kid = sp->lo_kid.p;
        v.noc = b.node_of_code.p;
        v.kcnt = b.kcnt;
        v.c64 = c64[(size_t)i].p;
        v.coff = g->coff.p;
        v.tids = g->tids.p;
        v.trun = merge ? g->trun.p : nullptr;
        lo_mark_presetup(g, anomaly[i], d, fp32);
    }
    DBuf<LDev> dl;
    MR_TRY(dl.upload(ctx, hv, (size_t)n));
    unsigned long long* dst = nullptr;
    uint64_t epoch = 0;
    MR_TRY(mr_dl_status(ctx, st_words, &dst, &epoch));
    hipLaunchKernelGGL(k_lo_cs_b, dim3(bcs), dim3(TS_T), 0, st, dl.p, n, dst, epoch);
    hipLaunchKernelGGL(k_lo_fill_b, dim3(bfl), dim3(256), 0, st, dl.p, n);
    hipLaunchKernelGGL(k_lo_total_b, dim3(n), dim3(1024), 0, st, dl.p);
    hipLaunchKernelGGL(k_lo_apply_b, dim3(bap), dim3(256), 0, st, dl.p, n);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;   // (scratch returns to the stream-ordered pool)
}

int mr_pagerank_batch_impl(mr_ctx* ctx, mr_graph* const* gs, const int* anomaly, int ng, double d, double alpha,
                           int iters, int precision, uint32_t flags, bool sharded = false) {
    constexpr int ATTEMPTS = 4;
    for (int a = 0; a < ATTEMPTS; ++a) {
        bool collided = false;
        MR_TRY(pagerank_attempt(ctx, gs, anomaly, ng, d, alpha, iters, precision, flags, sharded, kind_seed(a),
                                kind_hmask(a), &collided));
        if (!collided) return MR_OK;
    }
    return mr_fail(ctx, MR_ERR_STATE, "trace-kind hash collision under %d seeds", ATTEMPTS);
}

// MR_PR_KIND_COMPRESS (§8(f) f4): kinds of g with each trace's class representative, then a graph
// of the K representatives (multiplicities carried in q and in the preference sums), ranked
// by the same fused iteration; its weights are g's.  Graphs off the fused path (or with
// pr_trace != operation_trace) rank uncompressed.
static int kind_compressed_pagerank(mr_ctx* ctx, mr_graph* g, int anomaly, double d, double alpha, int iters,
                                    int precision, uint32_t flags) {
    const uint32_t plain = flags & ~(uint32_t)MR_PR_KIND_COMPRESS;
    if (!ctx || !g || g->ctx != ctx) return mr_fail(ctx, MR_ERR_ARG, "mr_pagerank: bad arguments");
    const int32_t T = g->T, N = g->N;
    if (!g->fused || !g->rs_is_sr || !g->pr_identity || T == 0 || N == 0)
        return mr_pagerank_batch_impl(ctx, &g, &anomaly, 1, d, alpha, iters, precision, plain);
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    // the representatives' graph depends on g's structure only (built, never changed): a later call
    // ranks the kept one (its preference and iteration state are set up per call as usual).
    // MR_KC_NOCACHE: rebuild every call (read per call)
    auto rank_kc = [&](mr_graph* gcp) -> int {
        gcp->phi = g->phi;
        MR_TRY(mr_pagerank_batch_impl(ctx, &gcp, &anomaly, 1, d, alpha, iters, precision, plain));
        MR_TRY(g->weight.alloc(ctx, (size_t)N));
        MR_TRY(g->sn.alloc(ctx, (size_t)N));
        MR_TRY_HIP(ctx, hipMemcpyAsync(g->weight.p, gcp->weight.p, (size_t)N * 8, hipMemcpyDeviceToDevice, st));
        MR_TRY_HIP(ctx, hipMemcpyAsync(g->sn.p, gcp->sn.p, (size_t)N * 8, hipMemcpyDeviceToDevice, st));
        return MR_OK;
    };
    if (g->kc && getenv("MR_KC_NOCACHE") == nullptr) return rank_kc(g->kc.get());
    g->kc.reset();
    // ---- kinds with representatives (the seed sequence of mr_pagerank_batch_impl)
    uint64_t cap = 1;
    while (cap < 2ull * (uint64_t)T) cap <<= 1;
    const char* kpe = getenv("MR_KIND_PART_MIN");
    const bool ktab = (int64_t)T < (kpe ? (int64_t)atoll(kpe) : KIND_PART_MIN_DEFAULT);
    if (!ktab) cap = 0;
    MR_TRY(g->kind.alloc(ctx, (size_t)T));
    MR_TRY(g->krep.alloc(ctx, (size_t)T));
    MR_TRY(g->pref.alloc(ctx, (size_t)T));
    MR_TRY(g->c_t.alloc(ctx, (size_t)T));
    MR_TRY(g->flag.alloc(ctx, 8));
    MR_TRY(g->scal.alloc(ctx, 8));
    if (ktab) {
        MR_TRY(g->ht_key.alloc(ctx, cap));
        MR_TRY(g->ht_cr.alloc(ctx, cap));
        MR_TRY(g->slot_of.alloc(ctx, (size_t)T));
    }
    bool ok = false;
    for (int a = 0; a < 4 && !ok; ++a) {
        hipLaunchKernelGGL(k_pr_reset, dim3(cdiv(std::max<int64_t>({(int64_t)T, (int64_t)cap, 16}), 256)), dim3(256), 0,
                           st, T, (int64_t)cap, N, g->pref.p, g->c_t.p, g->ht_key.p, g->ht_cr.p, g->flag.p, g->scal.p);
        MR_TRY(graph_kinds(ctx, g, false, ktab, cap, kind_seed(a), kind_hmask(a)));
        int32_t hf[4];
        MR_TRY(g->flag.download(ctx, hf, 4));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
        if (hf[2] & 1) return mr_fail(ctx, MR_ERR_STATE, "trace kinds: a partition exceeded its table");
        ok = !(hf[0] & 1);
    }
    if (!ok) return mr_fail(ctx, MR_ERR_STATE, "trace-kind hash collision under 4 seeds");
    // ---- the representatives' graph
    DBuf<int32_t> fl, rep, cnt;
    DBuf<int64_t> pos, tmp;
    MR_TRY(fl.alloc(ctx, (size_t)T));
    MR_TRY(pos.alloc(ctx, (size_t)T + 1));
    MR_TRY(tmp.alloc(ctx, (size_t)scan_tmp_elems(T)));
    hipLaunchKernelGGL(k_kc_flags, dim3(cdiv(T, 256)), dim3(256), 0, st, g->krep.p, T, fl.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, fl.p, pos.p, T, tmp.p));
    int64_t K = 0;
    MR_TRY_HIP(ctx, hipMemcpyAsync(&K, pos.p + T, sizeof K, hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    std::unique_ptr<mr_graph> gc(new mr_graph());
    gc->ctx = ctx;
    gc->N = N;
    gc->T = (int32_t)K;
    gc->T_all = T;   // v0 = 1 / (N + T) over every trace (pagerank.py:118-119)
    gc->E = g->E;
    MR_TRY(rep.alloc(ctx, (size_t)K));
    MR_TRY(cnt.alloc(ctx, (size_t)K));
    MR_TRY(gc->len_t.alloc(ctx, (size_t)K));
    MR_TRY(gc->mult.alloc(ctx, (size_t)K));
    hipLaunchKernelGGL(k_kc_reps, dim3(cdiv(T, 256)), dim3(256), 0, st, fl.p, pos.p, T, g->rs_off.p, g->len_t.p,
                       g->kind.p, rep.p, gc->len_t.p, gc->mult.p, cnt.p);
    MR_TRY(gc->rs_off.alloc(ctx, (size_t)K + 1));
    MR_TRY(tmp.alloc(ctx, (size_t)scan_tmp_elems(K)));
    MR_TRY(mr_exclusive_scan_i32(ctx, cnt.p, gc->rs_off.p, K, tmp.p));
    int64_t nnz = 0;
    MR_TRY_HIP(ctx, hipMemcpyAsync(&nnz, gc->rs_off.p + K, sizeof nnz, hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    MR_TRY(gc->rs_ops.alloc(ctx, (size_t)nnz));
    hipLaunchKernelGGL(k_kc_ops, dim3(cdiv(K, 256)), dim3(256), 0, st, rep.p, gc->rs_off.p, (int32_t)K, g->rs_off.p,
                       g->rs_ops.p, gc->rs_ops.p);
    MR_TRY(gc->len_o.alloc(ctx, (size_t)N));
    MR_TRY(gc->nchild.alloc(ctx, (size_t)N));
    MR_TRY(gc->ss_off.alloc(ctx, (size_t)N + 1));
    MR_TRY(gc->ss_par.alloc(ctx, (size_t)std::max<int64_t>(g->E, 1)));
    MR_TRY_HIP(ctx, hipMemcpyAsync(gc->len_o.p, g->len_o.p, (size_t)N * 4, hipMemcpyDeviceToDevice, st));
    MR_TRY_HIP(ctx, hipMemcpyAsync(gc->nchild.p, g->nchild.p, (size_t)N * 4, hipMemcpyDeviceToDevice, st));
    MR_TRY_HIP(ctx, hipMemcpyAsync(gc->ss_off.p, g->ss_off.p, ((size_t)N + 1) * 8, hipMemcpyDeviceToDevice, st));
    if (g->E) MR_TRY_HIP(ctx, hipMemcpyAsync(gc->ss_par.p, g->ss_par.p, (size_t)g->E * 4, hipMemcpyDeviceToDevice, st));
    gc->rs_is_sr = true;
    gc->pr_identity = true;
    gc->n_pr = (int32_t)K;
    gc->nnz_sr = gc->nnz_rs = nnz;
    gc->kinds_given = true;   // (before the prepare: its layout is then the stable sort)
    MR_TRY(mr_graph_prepare(ctx, gc.get()));
    if (!gc->fused)
        return mr_pagerank_batch_impl(ctx, &g, &anomaly, 1, d, alpha, iters, precision, plain);
    MR_TRY(gc->mw_tp.alloc(ctx, (size_t)K));
    hipLaunchKernelGGL(k_kc_mw, dim3(cdiv(K, 256)), dim3(256), 0, st, gc->tperm.p, gc->w_tp.p, gc->mult.p, (int32_t)K,
                       gc->mw_tp.p);
    DBuf<int64_t> tm;
    MR_TRY(tm.alloc(ctx, (size_t)std::max(gc->n_wt, 1)));
    hipLaunchKernelGGL(k_kc_tile_mult, dim3(cdiv(gc->n_wt, 256)), dim3(256), 0, st, gc->tperm.p, gc->mult.p, (int32_t)K,
                       gc->n_wt, tm.p);
    gc->tile_mult_h.assign((size_t)gc->n_wt, 0);
    MR_TRY(tm.download(ctx, gc->tile_mult_h.data(), (size_t)gc->n_wt));
    MR_TRY(gc->kind.alloc(ctx, (size_t)K));   // the class sizes, as the preference reads them
    MR_TRY_HIP(ctx, hipMemcpyAsync(gc->kind.p, gc->mult.p, (size_t)K * 8, hipMemcpyDeviceToDevice, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    MR_TRY(rank_kc(gc.get()));
    g->kc_kinds = K;
    g->kc = std::move(gc);
    return MR_OK;
}

extern "C" int mr_pagerank(mr_ctx* ctx, mr_graph* g, int anomaly, double d, double alpha, int iters,
                           int precision, uint32_t flags) {
    if (g) g->phi = 0.5;
    if (flags & MR_PR_KIND_COMPRESS) return kind_compressed_pagerank(ctx, g, anomaly, d, alpha, iters, precision, flags);
    return mr_pagerank_batch_impl(ctx, &g, &anomaly, 1, d, alpha, iters, precision, flags);
}

extern "C" int mr_pagerank_ex(mr_ctx* ctx, mr_graph* g, int anomaly, double d, double alpha, int iters, double phi,
                              int precision, uint32_t flags) {
    if (!g || !(phi > 0.0)) return mr_fail(ctx, MR_ERR_ARG, "mr_pagerank_ex: bad graph or phi");
    g->phi = phi;
    const int rc = (flags & MR_PR_KIND_COMPRESS) ? kind_compressed_pagerank(ctx, g, anomaly, d, alpha, iters, precision, flags)
                                                 : mr_pagerank_batch_impl(ctx, &g, &anomaly, 1, d, alpha, iters, precision, flags);
    g->phi = 0.5;
    return rc;
}

int mr_pagerank_async_commit(mr_ctx* ctx, PrAsync* a) {
    MR_TRY_HIP(ctx, hipMemcpyAsync(a->hflag, a->fl.p, (size_t)4 * a->ng * sizeof(int32_t), hipMemcpyDeviceToHost,
                                   ctx->stream));
    if (!a->ev) MR_TRY_HIP(ctx, hipEventCreateWithFlags(&a->ev, hipEventDisableTiming));
    MR_TRY_HIP(ctx, hipEventRecord(a->ev, ctx->stream));
    a->committed = true;
    return MR_OK;
}
int mr_pagerank_batch_async(mr_ctx* ctx, mr_graph* const* gs, const int* anomaly, int ng, double d, double alpha,
                            int iters, int precision, int32_t* hflag, PrAsync** out, bool defer) {
    std::unique_ptr<PrAsync> a(new PrAsync());
    a->hflag = hflag;
    a->defer = defer;
    bool collided = false;
    MR_TRY(pagerank_attempt(ctx, gs, anomaly, ng, d, alpha, iters, precision, 0, false, kind_seed(0), kind_hmask(0),
                            &collided, a.get()));
    *out = a.release();
    return MR_OK;
}
int mr_pagerank_async_finish(mr_ctx* ctx, PrAsync* a, bool* rerun) {
    *rerun = false;
    if (!a->committed) MR_TRY(mr_pagerank_async_commit(ctx, a));   // (a deferred batch nobody committed)
    MR_TRY_HIP(ctx, hipEventSynchronize(a->ev));
    for (int i = 0; i < a->ng; ++i) {
        const int32_t* w = a->hflag + 4 * i;
        if (w[0] & 1) {   // a kind-hash collision: the caller reruns
            *rerun = true;
            return MR_OK;
        }
        if (w[2] & 1) return mr_fail(ctx, MR_ERR_STATE, "trace kinds: a partition exceeded its table");
        if (a->anomaly[(size_t)i] && (w[1] & 1)) return mr_fail(ctx, MR_ERR_ZERODIV, "float division by zero");
    }
    return MR_OK;
}
void mr_pagerank_async_free(PrAsync* a) { delete a; }

extern "C" int mr_pagerank_batch(mr_ctx* ctx, mr_graph* const* graphs, const int* anomaly, int n_graphs, double d,
                                 double alpha, int iters, int precision, uint32_t flags) {
    return mr_pagerank_batch_impl(ctx, graphs, anomaly, n_graphs, d, alpha, iters, precision, flags);
}

// ------------------------------------------------------------------------------ sharded graphs
// the kind classes over the ranks through the peer regions: records partitioned by owner (one
// exchange round), merged by their owners, totals returned (a second round).  Each rank sends and
// receives ~ its own class count, instead of receiving every rank's list (the all-gather below).
static int shard_kinds_peer(mr_ctx* ctx, mr_graph* g, uint64_t cap, const DBuf<int32_t>& fl, const DBuf<int64_t>& pos,
                            int64_t Kl) {
    hipStream_t st = ctx->stream;
    const int32_t T = g->T;
    const int R = ctx->nranks, me = ctx->rank;
    DBuf<uint64_t> rec, send;
    DBuf<int64_t> spos;
    DBuf<unsigned long long> cnt;
    MR_TRY(rec.alloc(ctx, (size_t)3 * std::max<int64_t>(Kl, 1)));
    MR_TRY(send.alloc(ctx, (size_t)3 * std::max<int64_t>(Kl, 1)));
    MR_TRY(spos.alloc(ctx, (size_t)std::max<int64_t>(Kl, 1)));
    MR_TRY(cnt.zero(ctx, (size_t)R));
    hipLaunchKernelGGL(k_sh_kind_list, dim3(cdiv(cap, 256)), dim3(256), 0, st, g->ht_key.p, g->ht_cr.p, g->ht_chk.p,
                       (int64_t)cap, fl.p, pos.p, rec.p);
    if (Kl) hipLaunchKernelGGL(k_kx_count, dim3(cdiv(Kl, 256)), dim3(256), 0, st, rec.p, Kl, R, cnt.p);
    std::vector<int64_t> scnt((size_t)R), M((size_t)R * R);
    MR_TRY_HIP(ctx, hipMemcpyAsync(scnt.data(), cnt.p, sizeof(int64_t) * R, hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    std::vector<int64_t> soff((size_t)R + 1, 0);
    for (int o = 0; o < R; ++o) soff[(size_t)o + 1] = soff[(size_t)o] + scnt[(size_t)o];
    MR_TRY(cnt.upload(ctx, (const unsigned long long*)soff.data(), (size_t)R));   // cursors
    if (Kl) hipLaunchKernelGGL(k_kx_place, dim3(cdiv(Kl, 256)), dim3(256), 0, st, rec.p, Kl, R, cnt.p, send.p, spos.p);
    {   // every rank's counts per owner: M[s * R + o]
        DBuf<int64_t> mine, all;
        MR_TRY(mine.upload(ctx, scnt.data(), (size_t)R));
        MR_TRY(all.alloc(ctx, (size_t)R * R));
        MR_TRY(mr_coll_allgather(ctx, mine.p, all.p, R, MR_DT_I64));
        MR_TRY(all.download(ctx, M.data(), (size_t)R * R));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    }
    int64_t xa = 1, xb = 1;   // words: area A receives 3 per record owned, area B one total per record sent
    for (int o = 0; o < R; ++o) {
        int64_t in = 0, out = 0;
        for (int s = 0; s < R; ++s) {
            in += M[(size_t)s * R + o];
            out += M[(size_t)o * R + s];
        }
        xa = std::max(xa, 3 * in);
        xb = std::max(xb, out);
    }
    MR_TRY(mr_peer_xensure(ctx, xa, xb));
    // round 1: my records to their owners' areas A (after the records of lower ranks)
    for (int o = 0; o < R; ++o) {
        int64_t at = 0;
        for (int s = 0; s < me; ++s) at += M[(size_t)s * R + o];
        MR_TRY(mr_peer_put(ctx, (const unsigned long long*)send.p + 3 * soff[(size_t)o], 3 * scnt[(size_t)o], o, 0, 3 * at));
    }
    MR_TRY(mr_peer_round(ctx));
    // merge the records I own
    std::vector<int64_t> roff((size_t)R + 1, 0), dbase((size_t)R);
    for (int s = 0; s < R; ++s) {
        roff[(size_t)s + 1] = roff[(size_t)s] + M[(size_t)s * R + me];
        int64_t b = 0;   // where s keeps the totals of its records for me: its send offset of owner me
        for (int o = 0; o < me; ++o) b += M[(size_t)s * R + o];
        dbase[(size_t)s] = b;
    }
    const int64_t n = roff[(size_t)R];
    const uint64_t* in = (const uint64_t*)mr_peer_area(ctx, me, 0);
    uint64_t gcap = 1;
    while (gcap < 2 * (uint64_t)std::max<int64_t>(n, 1)) gcap <<= 1;
    DBuf<uint64_t> gk, gh;
    DBuf<unsigned long long> gc;
    DBuf<int64_t> droff, ddbase;
    MR_TRY(gk.zero(ctx, gcap));
    MR_TRY(gh.zero(ctx, gcap));
    MR_TRY(gc.zero(ctx, gcap));
    MR_TRY(droff.upload(ctx, roff.data(), roff.size()));
    MR_TRY(ddbase.upload(ctx, dbase.data(), dbase.size()));
    std::vector<unsigned long long*> areas((size_t)R);
    for (int s = 0; s < R; ++s) areas[(size_t)s] = mr_peer_area(ctx, s, 1);
    DBuf<unsigned long long*> dareas;
    MR_TRY(dareas.upload(ctx, areas.data(), areas.size()));
    if (n) {
        hipLaunchKernelGGL(k_sh_kind_merge, dim3(cdiv(n, 256)), dim3(256), 0, st, in, n, gk.p, gh.p, gc.p, gcap - 1,
                           g->flag.p);
        hipLaunchKernelGGL(k_sh_kind_check, dim3(cdiv(n, 256)), dim3(256), 0, st, in, n, gk.p, gh.p, gcap - 1, g->flag.p);
        // round 2: every record's total back to its sender's area B
        hipLaunchKernelGGL(k_kx_return, dim3(cdiv(n, 256)), dim3(256), 0, st, in, n, gk.p, gc.p, gcap - 1, droff.p,
                           ddbase.p, R, dareas.p);
    }
    MR_TRY(mr_peer_round(ctx));
    if (T)
        hipLaunchKernelGGL(k_kx_apply, dim3(cdiv(T, 256)), dim3(256), 0, st, g->ht_key.p, g->slot_of.p, fl.p, pos.p,
                           spos.p, (const unsigned long long*)mr_peer_area(ctx, me, 1), T, g->kind.p);
    MR_TRY_HIP(ctx, hipGetLastError());
    return mr_peer_check(ctx, "kind exchange");   // (syncs: the scratch leaves scope)
}

static int shard_kinds(mr_ctx* ctx, mr_graph* g, uint64_t cap) {
    hipStream_t st = ctx->stream;
    const int32_t T = g->T;
    DBuf<int32_t> fl;
    DBuf<int64_t> pos, tmp;
    MR_TRY(fl.alloc(ctx, cap));
    MR_TRY(pos.alloc(ctx, cap + 1));
    MR_TRY(tmp.alloc(ctx, scan_tmp_elems((int64_t)cap)));
    hipLaunchKernelGGL(k_sh_kind_flags, dim3(cdiv(cap, 256)), dim3(256), 0, st, g->ht_key.p, (int64_t)cap, fl.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, fl.p, pos.p, (int64_t)cap, tmp.p));
    DBuf<int64_t> kn;
    MR_TRY(kn.alloc(ctx, 1));
    MR_TRY_HIP(ctx, hipMemcpyAsync(kn.p, pos.p + cap, sizeof(int64_t), hipMemcpyDeviceToDevice, st));
    int64_t Kl = 0;
    MR_TRY(kn.download(ctx, &Kl, 1));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    if (mr_peer_ready(ctx)) {   // MR_ERR_STATE: the ranks could not map each other's regions (collective)
        const int rc = shard_kinds_peer(ctx, g, cap, fl, pos, Kl);
        if (rc != MR_ERR_STATE) return rc;
    }
    MR_TRY(mr_coll_allreduce(ctx, kn.p, 1, MR_DT_I64, 1));
    int64_t Kmax = 0;
    MR_TRY(kn.download(ctx, &Kmax, 1));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    const int R = ctx->nranks;
    DBuf<uint64_t> send, recv;
    MR_TRY(send.zero(ctx, (size_t)3 * std::max<int64_t>(Kmax, 1)));
    MR_TRY(recv.alloc(ctx, (size_t)3 * std::max<int64_t>(Kmax, 1) * R));
    hipLaunchKernelGGL(k_sh_kind_list, dim3(cdiv(cap, 256)), dim3(256), 0, st, g->ht_key.p, g->ht_cr.p, g->ht_chk.p,
                       (int64_t)cap, fl.p, pos.p, send.p);
    MR_TRY(mr_coll_allgather(ctx, send.p, recv.p, 3 * std::max<int64_t>(Kmax, 1), MR_DT_U64));
    const int64_t n = std::max<int64_t>(Kmax, 1) * R;
    uint64_t gcap = 1;
    while (gcap < 2 * (uint64_t)n) gcap <<= 1;
    DBuf<uint64_t> gk, gh;
    DBuf<unsigned long long> gc;
    MR_TRY(gk.zero(ctx, gcap));
    MR_TRY(gh.zero(ctx, gcap));
    MR_TRY(gc.zero(ctx, gcap));
    hipLaunchKernelGGL(k_sh_kind_merge, dim3(cdiv(n, 256)), dim3(256), 0, st, recv.p, n, gk.p, gh.p, gc.p, gcap - 1,
                       g->flag.p);
    hipLaunchKernelGGL(k_sh_kind_check, dim3(cdiv(n, 256)), dim3(256), 0, st, recv.p, n, gk.p, gh.p, gcap - 1, g->flag.p);
    if (T)
        hipLaunchKernelGGL(k_sh_kind_apply, dim3(cdiv(T, 256)), dim3(256), 0, st, g->ht_key.p, g->slot_of.p, T, gk.p,
                           gc.p, gcap - 1, g->kind.p);
    MR_TRY_HIP(ctx, hipGetLastError());
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // scratch leaves scope
    return MR_OK;
}

// once per graph: per-op sums, the union of the call edges, the number of traces
static int shard_exchange(mr_ctx* ctx, mr_graph* g) {
    hipStream_t st = ctx->stream;
    const int32_t N = g->N;
    MR_TRY(mr_coll_allreduce(ctx, g->len_o.p, N, MR_DT_I32, 0));
    MR_TRY(mr_coll_allreduce(ctx, g->nchild.p, N, MR_DT_I32, 0));
    MR_TRY(mr_coll_allreduce(ctx, g->cov.p, N, MR_DT_I32, 0));
    if (N) hipLaunchKernelGGL(k_op_consts, dim3(cdiv(N, 256)), dim3(256), 0, st, g->len_o.p, g->nchild.p, g->u_o.p, g->pw.p, N);
    DBuf<int64_t> sc;
    MR_TRY(sc.alloc(ctx, 2));
    int64_t h[2] = {(int64_t)g->T, g->E};
    MR_TRY(sc.upload(ctx, h, 2));
    MR_TRY(mr_coll_allreduce(ctx, sc.p, 1, MR_DT_I64, 0));       // traces over all ranks
    MR_TRY(mr_coll_allreduce(ctx, sc.p + 1, 1, MR_DT_I64, 1));   // largest local edge list
    MR_TRY(sc.download(ctx, h, 2));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    g->T_all = h[0];
    const int64_t Emax = std::max<int64_t>(h[1], 1);
    const int R = ctx->nranks;
    const int nb = std::max(1, bits_for((uint64_t)std::max(N - 1, 0)));
    const uint64_t pad = 1ull << (2 * nb);   // above every real key
    DBuf<uint64_t> send, recv;
    MR_TRY(send.alloc(ctx, (size_t)Emax));
    MR_TRY(recv.alloc(ctx, (size_t)Emax * R));
    if (N) hipLaunchKernelGGL(k_sh_edge_keys, dim3(cdiv(N, 256)), dim3(256), 0, st, g->ss_off.p, g->ss_par.p, N, nb, send.p);
    if (Emax > g->E) hipLaunchKernelGGL(k_sh_pad, dim3(cdiv(Emax - g->E, 256)), dim3(256), 0, st, send.p, g->E, Emax, pad);
    MR_TRY(mr_coll_allgather(ctx, send.p, recv.p, Emax, MR_DT_U64));
    const int64_t n = Emax * R;
    SortScratch ws;
    MR_TRY(mr_radix_sort(ctx, recv.p, nullptr, n, 2 * nb + 1, ws));
    DBuf<int32_t> head, ccount;
    DBuf<int64_t> pos, tmp;
    MR_TRY(head.alloc(ctx, n));
    MR_TRY(pos.alloc(ctx, n + 1));
    MR_TRY(tmp.alloc(ctx, std::max(scan_tmp_elems(n), scan_tmp_elems(std::max(N, 1)))));
    hipLaunchKernelGGL(k_sh_edge_heads, dim3(cdiv(n, 256)), dim3(256), 0, st, recv.p, n, pad, head.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, head.p, pos.p, n, tmp.p));
    int64_t E = 0;
    MR_TRY_HIP(ctx, hipMemcpyAsync(&E, pos.p + n, sizeof E, hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    MR_TRY(ccount.zero(ctx, N));
    g->ss_par.reset();
    MR_TRY(g->ss_par.alloc(ctx, (size_t)std::max<int64_t>(E, 1)));
    hipLaunchKernelGGL(k_sh_edge_out, dim3(cdiv(n, 256)), dim3(256), 0, st, recv.p, head.p, pos.p, n, nb, g->ss_par.p,
                       ccount.p);
    MR_TRY(mr_exclusive_scan_i32(ctx, ccount.p, g->ss_off.p, N, tmp.p));
    g->E = E;
    MR_TRY_HIP(ctx, hipGetLastError());
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    return MR_OK;
}

extern "C" int mr_pagerank_sharded(mr_ctx* ctx, mr_graph* g, int anomaly, double d, double alpha, int iters,
                                   int precision, uint32_t flags) {
    if (!ctx || !g || g->ctx != ctx) return mr_fail(ctx, MR_ERR_ARG, "mr_pagerank_sharded: bad handles");
    if (!mr_coll_ready(ctx) && ctx->nranks != 1) return mr_fail(ctx, MR_ERR_COMM, "no collective backend");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    if (!g->sharded_done) {   // the graph-level exchange happens once per graph
        if (mr_coll_ready(ctx) && ctx->nranks > 1) {
            // every rank must run the same iteration (the fused path's u64 limb all-reduce or the
            // tile path's fp64 op sums): the fused choice depends on this shard (e.g. a trace
            // without ops), so the ranks agree on it -- fused only if fused everywhere
            DBuf<int32_t> f;
            int32_t tile = g->fused ? 0 : 1;   // MAX over ranks: 1 if any rank takes the tile path
            MR_TRY(f.upload(ctx, &tile, 1));
            MR_TRY(mr_coll_allreduce(ctx, f.p, 1, MR_DT_I32, 1));
            MR_TRY(f.download(ctx, &tile, 1));
            MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
            if (g->fused && tile) {
                g->force_tile = true;
                MR_TRY(mr_graph_prepare(ctx, g));   // the P_sr tiles (before the per-op sums below)
            }
        }
        MR_TRY(shard_exchange(ctx, g));
        g->sharded_done = true;
    }
    // the per-iteration all-reduce buffer: the per-op sums, then one r' max slot per rank
    if (g->fused) MR_TRY(g->fx_limb.alloc(ctx, 2 * (size_t)g->N + (size_t)ctx->nranks));   // fixed-point limbs
    else MR_TRY(g->op_sum.alloc(ctx, (size_t)g->N + (size_t)ctx->nranks));                  // tile path: fp64 sums
    return mr_pagerank_batch_impl(ctx, &g, &anomaly, 1, d, alpha, iters, precision, flags, true);
}
