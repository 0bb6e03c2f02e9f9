// K2: personalised PageRank of pagerank.trace_pagerank (pagerank.py:15-130) on gfx950.
//
// Sparse, HBM-bound: no MFMA.  Each Jacobi iteration k -> k+1 (T8) is ONE launch with two
// block roles that both read only iteration-k state:
//   trace role  r'[t] = d * sum_{o in rs(t)} u_o * s_k[o] + fp32((1-d) v_t)      (pagerank.py:125)
//               q'[t] = w_t * r'[t]      (the P_sr-weighted value the op role sums next time)
//               s_k*u is staged in LDS; the block's contiguous id range is read coalesced into
//               LDS, then each thread sums its trace in node order.
//   op role     one wave per fixed 1024-entry segment of an op's trace list sums q'_k; the
//               LAST segment of an op to finish (agent-scope acq_rel counter) combines the
//               partials in segment order and adds the call-graph term:
//               s'[o] = d * (sum q'_k / M_r(k) + alpha * sum_{p in ss(o)} pw_p * s_k[p])  (:122-124)
// Maxima M_s, M_r (np.amax, :126-127) travel as bit patterns of non-negative doubles through
// atomicMax, which is exact and order-independent.  Normalisation of r is deferred:
// sum_t w_t (r'_t / M_r) is evaluated as (sum_t w_t r'_t) / M_r.  Every float reduction has a
// fixed order (no float atomics), so results are bitwise reproducible run to run.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "mr_internal.h"
#include "mr_prim.h"

namespace {

constexpr int SEG = 1024;           // op-list segment length (entries)
constexpr int TB = 256;             // trace-role block size (one trace per thread)
constexpr int LDS_NODES = 8192;     // su staged in LDS up to this many nodes (64 KiB)
constexpr int VCAP = 2048;          // trace-role ids staged per round in LDS (16 KiB of values)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void k_pr_reset(int32_t T, int64_t cap, int32_t N, float* pref, float* c_t, uint64_t* hk, uint32_t* hc,
                           int32_t* hr, uint32_t* op_cnt, int32_t* flag, double* scal) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < T) {
        pref[i] = 0.0f;
        c_t[i] = 0.0f;
    }
    if (i < cap) {
        hk[i] = 0ull;
        hc[i] = 0u;
        hr[i] = -1;
    }
    if (i < N) op_cnt[i] = 0u;
    if (i < 4) flag[i] = 0;
    if (i < 8) scal[i] = 0.0;
}

// ---------------------------------------------------------------- graph constants
__global__ void k_trace_consts(const int32_t* len_t, float* w_t, int32_t T) {
    int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < T) w_t[t] = len_t[t] > 0 ? (float)(1.0 / (double)len_t[t]) : 0.0f;   // fp64 1/n -> fp32
}

__global__ void k_op_consts(const int32_t* len_o, const int32_t* nchild, const int64_t* sr_off,
                            float* u_o, float* pw, int32_t* cov, int32_t* nseg_of, int32_t N) {
    int32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= N) return;
    u_o[o] = len_o[o] > 0 ? (float)(1.0 / (double)len_o[o]) : 0.0f;
    pw[o] = nchild[o] > 0 ? (float)(1.0 / (double)nchild[o]) : 0.0f;
    int64_t c = sr_off[o + 1] - sr_off[o];
    cov[o] = (int32_t)c;                                  // trace_num_list (pagerank.py:98-104)
    nseg_of[o] = c > 0 ? (int32_t)((c + SEG - 1) / SEG) : 1;   // >= 1: every op gets a finisher
}

__global__ void k_fill_segments(const int64_t* op_seg64, const int64_t* sr_off, int32_t* op_seg,
                                int32_t* seg_op, int64_t* seg_beg, int32_t N) {
    int32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o > N) return;
    op_seg[o] = (int32_t)op_seg64[o];
    if (o == N) return;
    int64_t s0 = op_seg64[o], s1 = op_seg64[o + 1];
    for (int64_t s = s0; s < s1; ++s) {
        seg_op[s] = o;
        seg_beg[s] = sr_off[o] + (s - s0) * SEG;
    }
}

// ---------------------------------------------------------------- kinds (pagerank.py:54-66)
// kind[t] = size of the class of traces with an equal P_sr column: key = (op set, fp32(1/len_t)).
// Open-addressing hash table of 64-bit keys; a second pass verifies every member against the
// slot's representative, so a hash collision is detected (flag) rather than miscounted.
constexpr int KB = 256, KLDS = 512;   // kinds: block size, LDS table slots

__device__ __forceinline__ uint64_t kind_hash(const int64_t* off, const int32_t* ops, const float* w_t,
                                              int32_t t, uint64_t seed) {
    int64_t e0 = off[t], e1 = off[t + 1];
    uint32_t wb = e1 > e0 ? __float_as_uint(w_t[t]) : 0u;
    uint64_t h = mix64(seed ^ (uint64_t)wb);
    for (int64_t e = e0; e < e1; ++e) h = mix64(h ^ (uint64_t)(uint32_t)ops[e]);
    return h ? h : 1;
}

// Two-level insertion: traces of a block are first counted in an LDS table (hot kinds -- the
// same few call paths in thousands of traces -- would otherwise serialise on one global
// counter), then each distinct key of the block does ONE global insert + add.
__global__ void __launch_bounds__(KB) k_kind_insert(const int64_t* off, const int32_t* ops, const float* w_t,
                                                    int32_t T, uint64_t* keys, uint32_t* cnt, int32_t* rep,
                                                    int32_t* slot_of, uint64_t mask, uint64_t seed) {
    __shared__ unsigned long long lkey[KLDS];
    __shared__ uint32_t lcnt[KLDS];
    __shared__ int32_t lrep[KLDS];
    __shared__ int32_t lglob[KLDS];
    for (int i = threadIdx.x; i < KLDS; i += KB) {
        lkey[i] = 0ull;
        lcnt[i] = 0u;
        lrep[i] = -1;
    }
    __syncthreads();
    const int32_t t = blockIdx.x * KB + threadIdx.x;
    int myslot = -1;
    if (t < T) {
        const uint64_t h = kind_hash(off, ops, w_t, t, seed);
        int s = (int)(h & (KLDS - 1));
        for (;;) {
            unsigned long long k = atomicCAS(&lkey[s], 0ull, (unsigned long long)h);
            if (k == 0ull || k == h) break;
            s = (s + 1) & (KLDS - 1);
        }
        atomicAdd(&lcnt[s], 1u);
        atomicCAS(&lrep[s], -1, t);
        myslot = s;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < KLDS; i += KB) {
        const uint64_t h = lkey[i];
        if (!h) continue;
        uint64_t slot = h & mask;
        for (;;) {
            uint64_t k = atomicCAS((unsigned long long*)&keys[slot], 0ull, (unsigned long long)h);
            if (k == 0 || k == h) break;
            slot = (slot + 1) & mask;
        }
        atomicAdd(&cnt[slot], lcnt[i]);
        atomicCAS(&rep[slot], -1, lrep[i]);
        lglob[i] = (int32_t)slot;
    }
    __syncthreads();
    if (t < T) slot_of[t] = lglob[myslot];
}

__global__ void k_kind_verify(const int64_t* off, const int32_t* ops, const float* w_t, int32_t T,
                              const uint32_t* cnt, const int32_t* rep, const int32_t* slot_of,
                              double* kind, int32_t* flag) {
    int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    int32_t s = slot_of[t];
    int32_t r = rep[s];
    kind[t] = (double)cnt[s];
    if (r == t) return;
    int64_t a0 = off[t], a1 = off[t + 1], b0 = off[r], b1 = off[r + 1];
    bool eq = (a1 - a0) == (b1 - b0);
    if (eq && a1 > a0) eq = __float_as_uint(w_t[t]) == __float_as_uint(w_t[r]);
    for (int64_t i = 0; eq && i < a1 - a0; ++i) eq = ops[a0 + i] == ops[b0 + i];
    if (!eq) atomicOr(flag, 1);
}

// ---------------------------------------------------------------- preference (pagerank.py:68-85)
// sums over pr_trace entries: [0] sum 1/k, [1] sum 1/len; block partials then one fixed-order pass
__global__ void k_pref_partial(const double* kind, const int32_t* pr_trace, const int32_t* pr_len,
                               const int32_t* len_t, int32_t n_pr, double* part, int32_t* flag) {
    __shared__ double red[TB / WAVE];
    double a = 0.0, b = 0.0;
    int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_pr) {
        int32_t t = pr_trace ? pr_trace[i] : i;
        int32_t ln = pr_len ? pr_len[i] : len_t[t];
        a = 1.0 / kind[t];
        if (ln == 0) atomicOr(flag, 2);   // 1.0/len(pr_trace[t]) -> ZeroDivisionError
        b = ln ? 1.0 / (double)ln : 0.0;
    }
    a = block_sum(a, red);
    b = block_sum(b, red);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = a;
        part[2 * blockIdx.x + 1] = b;
    }
}

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

__global__ void k_pref_apply(const double* kind, const int32_t* pr_trace, const int32_t* pr_len,
                             const int32_t* len_t, int32_t n_pr, const double* scal, int anomaly,
                             float cd, float* pref, float* c_t) {
    int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pr) return;
    int32_t t = pr_trace ? pr_trace[i] : i;
    int32_t ln = pr_len ? pr_len[i] : len_t[t];
    double k = kind[t];
    double v;
    if (!anomaly) {
        v = 1.0 / k / scal[2];                                               // :74
    } else {
        v = 1.0 / (k / scal[2] * 0.5 + 1.0 / (double)ln) / scal[3] * 0.5;   // :80-85
    }
    float vf = (float)v;
    pref[t] = vf;
    c_t[t] = cd * vf;   // (1.0 - d) * v: float32 array times a Python float stays float32 (T4)
}

// ---------------------------------------------------------------- iteration
// M_s / M_r per iteration live in MSH shards (an atomicMax per block or op on ONE word would
// serialise ~2k same-address atomics per iteration); readers reduce the shards.
constexpr int MSH = 64;
__device__ __forceinline__ double bits2d(unsigned long long b) { return __longlong_as_double((long long)b); }
__device__ __forceinline__ unsigned long long d2bits(double v) {
    return (unsigned long long)__double_as_longlong(v);
}

__global__ void k_iter_init(const float* w_t, const float* u_o, int32_t N, int32_t T, double* sp0, double* su0,
                            double* q64, float* q32, int fp32, unsigned long long* mslot) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const double v0 = 1.0 / (double)(N + T);                   // pagerank.py:118-119
    if (i < N) {
        sp0[i] = v0;
        su0[i] = (double)u_o[i] * v0;
    }
    if (i < T) {
        double q = (double)w_t[i] * v0;
        if (fp32) q32[i] = (float)q; else q64[i] = q;
    }
    // M_s(0) = M_r(0) = 1: s_0, r_0 are used as they are; slots 1, 2 start cleared
    if (i < 6 * MSH) mslot[i] = i < 2 * MSH ? d2bits(1.0) : 0ull;
}

// Per-graph view for the batched iteration: one launch per Jacobi iteration covers every graph
// of a batch (the two graphs of an RCA window, or many windows), each graph owning a contiguous
// range of blocks [blk0, blk0 + n_tb + n_ob).
struct GDev {
    const int64_t* rs_off;
    const int32_t* rs_ops;
    const float* c_t;
    const float* w_t;
    const float* u_o;
    const float* pw;
    const int64_t* sr_off;
    const int32_t* sr_trs;
    const int32_t* seg_op;
    const int64_t* seg_beg;
    const int32_t* op_seg;
    const int64_t* ss_off;
    const int32_t* ss_par;
    void* q[2];
    double* sub[2];
    double* spb[2];
    double* part;
    uint32_t* op_cnt;
    unsigned long long* mslot;
    int32_t T, N, nseg, n_tb, lds_su, blk0;
};

// One Jacobi iteration k -> k+1.  Maxima are exchanged as the bit patterns of non-negative
// doubles through atomicMax (exact and order-independent); slot k%3 holds (M_s(k), M_r(k)),
// slot (k+1)%3 collects iteration k+1, slot (k+2)%3 is cleared here for k+2.  s' is carried
// unnormalised together with su'[o] = u_o * s'[o]; the division by M_s(k) is applied to each
// finished sum instead of to every term.
template <class Q>
__global__ void __launch_bounds__(TB) k_iter(const GDev* __restrict__ gs, int32_t ng, double d, double alpha, int it) {
    extern __shared__ double lds[];
    __shared__ double red[TB / WAVE];
    __shared__ double msr[2];
    __shared__ int32_t sg;
    if (threadIdx.x == 0) {   // this block's graph: the last one whose blk0 <= blockIdx.x
        int32_t lo = 0, hi = ng - 1;
        while (lo < hi) {
            const int32_t mid = (lo + hi + 1) >> 1;
            if (gs[mid].blk0 <= (int32_t)blockIdx.x) lo = mid; else hi = mid - 1;
        }
        sg = lo;
    }
    __syncthreads();
    const GDev& G = gs[sg];
    const int32_t lb = (int32_t)blockIdx.x - G.blk0;
    const int cur = it & 1, nxt = cur ^ 1, k3 = it % 3;
    const uint32_t epoch = (uint32_t)it + 1u;
    const int32_t T = G.T, N = G.N;
    unsigned long long* mslot = G.mslot;
    // slot layout: [k%3][s|r][MSH]
    const unsigned long long* Mcur = mslot + (size_t)2 * MSH * k3;
    unsigned long long* Mnext = mslot + (size_t)2 * MSH * ((k3 + 1) % 3);
    if (lb == 0 && threadIdx.x < 2 * MSH) mslot[(size_t)2 * MSH * ((k3 + 2) % 3) + threadIdx.x] = 0ull;
    if (threadIdx.x < WAVE) {
        double ms = bits2d(Mcur[threadIdx.x]), mr = bits2d(Mcur[MSH + threadIdx.x]);
        ms = wave_max(ms);
        mr = wave_max(mr);
        if (threadIdx.x == 0) {
            msr[0] = ms;
            msr[1] = mr;
        }
    }
    __syncthreads();
    const double Ms = msr[0], Mr = msr[1];
    const int shard = blockIdx.x % MSH;
    if (lb < G.n_tb) {
        // ---- trace role: r'[t] = d * (sum_o u_o s'_k[o]) / M_s(k) + c_t  (pagerank.py:125)
        // The block's contiguous id range is read coalesced in rounds of VCAP ids (all loads in
        // flight before any gather), su' gathered from LDS into LDS, then each thread continues
        // its own trace's sum in node order.
        const int64_t* __restrict__ rs_off = G.rs_off;
        const int32_t* __restrict__ rs_ops = G.rs_ops;
        const double* su = G.sub[cur];
        if (G.lds_su) {
            for (int32_t o = threadIdx.x; o < N; o += TB) lds[o] = su[o];
            su = lds;
        }
        double* vals = lds + (G.lds_su ? N : 0);
        const int32_t t0 = lb * TB;
        const int32_t t1 = min(t0 + TB, T);
        const int64_t e0 = rs_off[t0], e1 = rs_off[t1];
        const int32_t t = t0 + threadIdx.x;
        const bool own = t < T;
        const int64_t a = own ? rs_off[t] : 0, b = own ? rs_off[t + 1] : 0;
        double acc = 0.0;
        for (int64_t lo = e0; lo < e1; lo += VCAP) {
            const int64_t hi = min(lo + (int64_t)VCAP, e1);
            __syncthreads();
            int32_t id[VCAP / TB];
#pragma unroll
            for (int j = 0; j < VCAP / TB; ++j) id[j] = rs_ops[min(lo + threadIdx.x + (int64_t)j * TB, hi - 1)];
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
        double rmax = -__builtin_huge_val();
        if (own) {
            const double rp = d * (acc / Ms) + (double)G.c_t[t];
            ((Q*)G.q[nxt])[t] = (Q)((double)G.w_t[t] * rp);
            rmax = rp;
        }
        rmax = block_max(rmax, red);
        if (threadIdx.x == 0) atomicMax(&Mnext[MSH + shard], d2bits(rmax));
        return;
    }
    // ---- op role: one wave per fixed segment of an op's trace list  (pagerank.py:122-124)
    const int32_t seg = (lb - G.n_tb) * (TB / WAVE) + (int32_t)(threadIdx.x / WAVE);
    if (seg >= G.nseg) return;
    const int lane = threadIdx.x & (WAVE - 1);
    const int32_t o = G.seg_op[seg];
    const int64_t b = G.seg_beg[seg];
    const int64_t end = min(b + (int64_t)SEG, G.sr_off[o + 1]);
    const Q* __restrict__ q_cur = (const Q*)G.q[cur];
    const int32_t* __restrict__ sr_trs = G.sr_trs;
    double acc = 0.0;
    if (end > b) {   // ids first, then every gather, then the sum in element order
        int32_t id[SEG / WAVE];
#pragma unroll
        for (int j = 0; j < SEG / WAVE; ++j) id[j] = sr_trs[min(b + lane + (int64_t)j * WAVE, end - 1)];
        double v[SEG / WAVE];
#pragma unroll
        for (int j = 0; j < SEG / WAVE; ++j) v[j] = (double)q_cur[id[j]];
#pragma unroll
        for (int j = 0; j < SEG / WAVE; ++j)
            if (b + lane + (int64_t)j * WAVE < end) acc += v[j];
    }
    acc = wave_sum(acc);
    const int32_t s0 = G.op_seg[o], s1 = G.op_seg[o + 1];
    uint32_t old = 0;
    if (lane == 0) {
        if (s1 - s0 > 1) {
            // hand-off without L2 write-back: write-through (sc1) payload, drain, relaxed counter
            __hip_atomic_store(&G.part[seg], acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            old = __hip_atomic_fetch_add(&G.op_cnt[o], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            old = epoch - 1u;   // single segment: this wave finishes the op
        }
    }
    old = __shfl(old, 0, WAVE);
    if (old != epoch * (uint32_t)(s1 - s0) - 1u) return;
    // last segment of op o to finish: combine the partials (sc1 loads) in a fixed order
    double sum = 0.0;
    if (s1 - s0 > 1) {
        for (int32_t s = s0 + lane; s < s1; s += WAVE)
            sum += __hip_atomic_load(&G.part[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        sum = wave_sum(sum);
    } else {
        sum = acc;
    }
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
void mr_prof_end(mr_ctx* ctx, double bytes);

int mr_graph_prepare(mr_ctx* ctx, mr_graph* g) {
    const int32_t N = g->N, T = g->T;
    MR_TRY(g->w_t.alloc(ctx, (size_t)T));
    MR_TRY(g->u_o.alloc(ctx, (size_t)N));
    MR_TRY(g->pw.alloc(ctx, (size_t)N));
    MR_TRY(g->cov.alloc(ctx, (size_t)N));
    DBuf<int32_t> nseg_of;
    DBuf<int64_t> op_seg64, tmp;
    MR_TRY(nseg_of.alloc(ctx, (size_t)N));
    MR_TRY(op_seg64.alloc(ctx, (size_t)N + 1));
    MR_TRY(tmp.alloc(ctx, (size_t)scan_tmp_elems(N)));
    if (T) hipLaunchKernelGGL(k_trace_consts, dim3(cdiv(T, 256)), dim3(256), 0, ctx->stream, g->len_t.p, g->w_t.p, T);
    if (N)
        hipLaunchKernelGGL(k_op_consts, dim3(cdiv(N, 256)), dim3(256), 0, ctx->stream, g->len_o.p, g->nchild.p,
                           g->sr_off.p, g->u_o.p, g->pw.p, g->cov.p, nseg_of.p, N);
    MR_TRY(mr_exclusive_scan_i32(ctx, nseg_of.p, op_seg64.p, N, tmp.p));
    int64_t nseg = 0;
    MR_TRY_HIP(ctx, hipMemcpyAsync(&nseg, op_seg64.p + N, sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    g->nseg = (int32_t)nseg;
    MR_TRY(g->op_seg.alloc(ctx, (size_t)N + 1));
    MR_TRY(g->seg_op.alloc(ctx, (size_t)nseg));
    MR_TRY(g->seg_beg.alloc(ctx, (size_t)nseg));
    hipLaunchKernelGGL(k_fill_segments, dim3(cdiv(N + 1, 256)), dim3(256), 0, ctx->stream, op_seg64.p, g->sr_off.p,
                       g->op_seg.p, g->seg_op.p, g->seg_beg.p, N);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;   // scratch returns to the stream-ordered pool: no sync needed
}

// kinds, preference vector and iteration state of one graph (everything before the iterations)
static int pagerank_setup(mr_ctx* ctx, mr_graph* g, int anomaly, double d, bool fp32, uint32_t flags) {
    hipStream_t st = ctx->stream;
    const int32_t N = g->N, T = g->T;
    uint64_t cap = 1;
    while (cap < 2ull * (uint64_t)T) cap <<= 1;
    const int32_t n_pr = g->n_pr;
    const int nbp = cdiv(n_pr > 0 ? n_pr : 1, TB);
    MR_TRY(g->kind.alloc(ctx, (size_t)T));
    MR_TRY(g->pref.alloc(ctx, (size_t)T));
    MR_TRY(g->c_t.alloc(ctx, (size_t)T));
    MR_TRY(g->flag.alloc(ctx, 4));
    MR_TRY(g->scal.alloc(ctx, 8));
    MR_TRY(g->ppart.alloc(ctx, 2 * (size_t)nbp));
    MR_TRY(g->ht_key.alloc(ctx, cap));
    MR_TRY(g->ht_cnt.alloc(ctx, cap));
    MR_TRY(g->ht_rep.alloc(ctx, cap));
    MR_TRY(g->slot_of.alloc(ctx, (size_t)T));
    MR_TRY(g->op_cnt.alloc(ctx, (size_t)N));
    MR_TRY(g->mslot.alloc(ctx, 6 * MSH));
    MR_TRY(g->sn.alloc(ctx, (size_t)N));
    MR_TRY(g->spb[0].alloc(ctx, (size_t)N));
    MR_TRY(g->spb[1].alloc(ctx, (size_t)N));
    MR_TRY(g->sub[0].alloc(ctx, (size_t)N));
    MR_TRY(g->sub[1].alloc(ctx, (size_t)N));
    MR_TRY(g->weight.alloc(ctx, (size_t)N));
    MR_TRY(g->part.alloc(ctx, (size_t)g->nseg));
    for (int i = 0; i < 2; ++i) {
        if (fp32) MR_TRY(g->q32[i].alloc(ctx, (size_t)T));
        else MR_TRY(g->q64[i].alloc(ctx, (size_t)T));
    }
    // one launch clears every per-call word (instead of a memset per buffer)
    hipLaunchKernelGGL(k_pr_reset, dim3(cdiv(std::max<int64_t>({(int64_t)T, (int64_t)cap, (int64_t)N, 16}), 256)),
                       dim3(256), 0, st, T, (int64_t)cap, N, g->pref.p, g->c_t.p, g->ht_key.p, g->ht_cnt.p, g->ht_rep.p,
                       g->op_cnt.p, g->flag.p, g->scal.p);
    MR_DEBUG_CHECK(ctx, "k_pr_reset");
    // ---- kinds
    const int64_t* koff = g->rs_is_sr ? g->rs_off.p : g->srt_off.p;
    const int32_t* kops = g->rs_is_sr ? g->rs_ops.p : g->srt_ops.p;
    hipLaunchKernelGGL(k_kind_insert, dim3(cdiv(T, KB)), dim3(KB), 0, st, koff, kops, g->w_t.p, T, g->ht_key.p,
                       g->ht_cnt.p, g->ht_rep.p, g->slot_of.p, (uint64_t)(cap - 1), 0x5eed5eedull);
    MR_DEBUG_CHECK(ctx, "k_kind_insert");
    hipLaunchKernelGGL(k_kind_verify, dim3(cdiv(T, 256)), dim3(256), 0, st, koff, kops, g->w_t.p, T, g->ht_cnt.p,
                       g->ht_rep.p, g->slot_of.p, g->kind.p, g->flag.p);
    MR_DEBUG_CHECK(ctx, "k_kind_verify");
    // ---- preference
    const int32_t* prt = g->pr_identity ? nullptr : g->pr_trace.p;
    const int32_t* prl = g->pr_identity ? nullptr : g->pr_len.p;
    if (n_pr > 0)
        hipLaunchKernelGGL(k_pref_partial, dim3(nbp), dim3(TB), 0, st, g->kind.p, prt, prl, g->len_t.p, n_pr,
                           g->ppart.p, g->flag.p);
    if (flags & MR_PR_EXACT_SUMS)
        hipLaunchKernelGGL(k_pref_total_exact, dim3(1), dim3(64), 0, st, g->kind.p, prt, prl, g->len_t.p, n_pr,
                           g->scal.p);
    else
        hipLaunchKernelGGL(k_pref_total, dim3(1), dim3(1024), 0, st, g->ppart.p, nbp, g->scal.p);
    MR_DEBUG_CHECK(ctx, "k_pref");
    const float cd = (float)(1.0 - d);
    if (n_pr > 0)
        hipLaunchKernelGGL(k_pref_apply, dim3(nbp), dim3(TB), 0, st, g->kind.p, prt, prl, g->len_t.p, n_pr,
                           g->scal.p, anomaly, cd, g->pref.p, g->c_t.p);
    MR_DEBUG_CHECK(ctx, "k_pref_apply");
    hipLaunchKernelGGL(k_iter_init, dim3(cdiv(std::max<int64_t>({N, T, 6 * MSH}), 256)), dim3(256), 0, st, g->w_t.p,
                       g->u_o.p, N, T, g->spb[0].p, g->sub[0].p, g->q64[0].p, g->q32[0].p, (int)fp32, g->mslot.p);
    MR_DEBUG_CHECK(ctx, "k_iter_init");
    return MR_OK;
}

// algorithmic bytes of one iteration of one graph: op ids once, offsets, the
// r/v/len_t streams, call edges and three N-vectors; o = 4-byte offsets below 2^31 nonzeros
static double iter_bytes(const mr_graph* g, bool fp32) {
    const double w = fp32 ? 4.0 : 8.0, o = g->nnz_sr < (1ll << 31) ? 4.0 : 8.0;
    return 4.0 * (double)g->nnz_sr + o * ((double)g->T + 1) + 4.0 * w * (double)g->T + (8.0 + w) * (double)g->E +
           3.0 * w * (double)g->N;
}

int mr_pagerank_batch_impl(mr_ctx* ctx, mr_graph* const* gs, const int* anomaly, int ng, double d, double alpha,
                           int iters, int precision, uint32_t flags) {
    if (!ctx || ng <= 0 || !gs || !anomaly) return mr_fail(ctx, MR_ERR_ARG, "mr_pagerank: bad arguments");
    if (iters < 0) return mr_fail(ctx, MR_ERR_ARG, "iters < 0");
    for (int i = 0; i < ng; ++i) {
        if (!gs[i] || gs[i]->ctx != ctx) return mr_fail(ctx, MR_ERR_STATE, "mr_pagerank: bad handles");
        if (gs[i]->N == 0 || gs[i]->T == 0)   // np.amax of an empty vector (pagerank.py:126-127)
            return mr_fail(ctx, MR_ERR_VALUE, "zero-size array to reduction operation maximum which has no identity");
    }
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const bool fp32 = precision == MR_FP32;
    for (int i = 0; i < ng; ++i) MR_TRY(pagerank_setup(ctx, gs[i], anomaly[i], d, fp32, flags));
    // ---- batched power iteration: one launch per iteration for every graph
    int mask = 3;
    if (const char* rm = getenv("MR_ROLE_MASK")) mask = atoi(rm);   // profiling knob: 1 trace / 2 op role
    std::vector<GDev> hv((size_t)ng);
    int32_t blocks = 0;
    size_t lds = VCAP * sizeof(double);
    double bytes = 0.0;
    for (int i = 0; i < ng; ++i) {
        mr_graph* g = gs[i];
        GDev& v = hv[(size_t)i];
        v.rs_off = g->rs_off.p;
        v.rs_ops = g->rs_ops.p;
        v.c_t = g->c_t.p;
        v.w_t = g->w_t.p;
        v.u_o = g->u_o.p;
        v.pw = g->pw.p;
        v.sr_off = g->sr_off.p;
        v.sr_trs = g->sr_trs.p;
        v.seg_op = g->seg_op.p;
        v.seg_beg = g->seg_beg.p;
        v.op_seg = g->op_seg.p;
        v.ss_off = g->ss_off.p;
        v.ss_par = g->ss_par.p;
        for (int j = 0; j < 2; ++j) {
            v.q[j] = fp32 ? (void*)g->q32[j].p : (void*)g->q64[j].p;
            v.sub[j] = g->sub[j].p;
            v.spb[j] = g->spb[j].p;
        }
        v.part = g->part.p;
        v.op_cnt = g->op_cnt.p;
        v.mslot = g->mslot.p;
        v.T = g->T;
        v.N = g->N;
        v.nseg = (mask & 2) ? g->nseg : 0;
        v.n_tb = (mask & 1) ? cdiv(g->T, TB) : 0;
        v.lds_su = g->N <= LDS_NODES;
        v.blk0 = blocks;
        blocks += v.n_tb + cdiv(v.nseg, TB / WAVE);
        if (v.lds_su) lds = std::max(lds, ((size_t)g->N + VCAP) * sizeof(double));
        bytes += iter_bytes(g, fp32);
    }
    DBuf<GDev> dv;
    MR_TRY(dv.upload(ctx, hv.data(), hv.size()));
    for (int it = 0; it < iters && blocks > 0; ++it) {
        mr_prof_begin(ctx);
        if (fp32) hipLaunchKernelGGL(k_iter<float>, dim3(blocks), dim3(TB), lds, st, dv.p, ng, d, alpha, it);
        else hipLaunchKernelGGL(k_iter<double>, dim3(blocks), dim3(TB), lds, st, dv.p, ng, d, alpha, it);
        MR_DEBUG_CHECK(ctx, "k_iter");
        mr_prof_end(ctx, bytes);
    }
    for (int i = 0; i < ng; ++i) {
        mr_graph* g = gs[i];
        hipLaunchKernelGGL(k_weights, dim3(1), dim3(1024), 0, st, g->spb[iters & 1].p, g->mslot.p, iters % 3, g->N,
                           (int)((flags & MR_PR_EXACT_SUMS) != 0), g->sn.p, g->weight.p, g->scal.p);
        MR_DEBUG_CHECK(ctx, "k_weights");
    }
    MR_TRY_HIP(ctx, hipGetLastError());
    // the only host round trip of the call: error words raised by the kernels
    std::vector<int32_t> hflag((size_t)4 * ng, 0);
    for (int i = 0; i < ng; ++i)
        MR_TRY_HIP(ctx, hipMemcpyAsync(&hflag[(size_t)4 * i], gs[i]->flag.p, 4 * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    for (int i = 0; i < ng; ++i) {
        if (hflag[(size_t)4 * i] & 1) return mr_fail(ctx, MR_ERR_STATE, "trace-kind hash collision (retry with another seed)");
        if (anomaly[i] && (hflag[(size_t)4 * i] & 2)) return mr_fail(ctx, MR_ERR_ZERODIV, "float division by zero");
    }
    return MR_OK;
}

extern "C" int mr_pagerank(mr_ctx* ctx, mr_graph* g, int anomaly, double d, double alpha, int iters,
                           int precision, uint32_t flags) {
    return mr_pagerank_batch_impl(ctx, &g, &anomaly, 1, d, alpha, iters, precision, flags);
}

extern "C" int mr_pagerank_batch(mr_ctx* ctx, mr_graph* const* graphs, const int* anomaly, int n_graphs, double d,
                                 double alpha, int iters, int precision, uint32_t flags) {
    return mr_pagerank_batch_impl(ctx, graphs, anomaly, n_graphs, d, alpha, iters, precision, flags);
}
