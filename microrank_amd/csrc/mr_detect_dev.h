// The window detector's per-block body (anormaly_detector.system_anomaly_detect on whole traces),
// shared by k_ix_detect (mr_span_index.hip) and the fused detector + selection scan of a window's
// two graph builds (k_ix_detect_scan2, mr_graph_build.hip).
//
// A trace is in the window iff its trace-level [start, end] lies in [t0, t1] (T15); expect = sum
// over the trace's service-ops in name order of count * (mean + 3 std) (sequential, no FMA: T14);
// abnormal iff max duration / 1000 > expect; traces with max <= 0 are dropped
// (preprocess_data.py:117).
#pragma once
#include "mr_internal.h"

constexpr int DB = 256, DCAP = 16;   // detector: traces per block, staged entries per thread
constexpr int CSH = 64;              // counter shards
static_assert(CSH == MR_DETECT_SHARDS, "detector counter shards");

struct DetIn {
    const int32_t* tlen;
    const long long *tts, *tte, *tmaxd;
    const int64_t* sv_off;
    const int32_t *sv_op, *sv_cnt;
    const double* a3;
    const uint8_t* a3v;
    int64_t t0, t1;
    uint8_t* state;                 // out: 0 out / 1 normal / 2 abnormal, every trace
    unsigned long long* counts;     // out: 3 * CSH counter shards (abnormal, normal, in-window rows)
};

// Block of DB threads, trace blk * DB + threadIdx.x per thread: its state (also returned) and the
// block's counts.  `term` is the caller's LDS of DB * DCAP doubles.  blk: the block's index among
// the window's (blockIdx.x, or its offset in a launch over several windows)
__device__ __forceinline__ int detect_block(int32_t NT, const DetIn& d, double* term, int32_t blk = -1) {
    if (blk < 0) blk = (int32_t)blockIdx.x;
    const int32_t tb = blk * DB, te_ = min(tb + DB, NT);
    const int32_t t = tb + threadIdx.x;
    // the thread's trace, loaded before the block's entries so both latencies overlap
    bool in = false;
    int64_t rows = 0, a = 0, b = 0;
    long long mx = 0;
    if (t < NT) {
        const int32_t len = d.tlen[t];
        const long long ts = d.tts[t], te = d.tte[t];
        mx = d.tmaxd[t];
        a = d.sv_off[t];
        b = d.sv_off[t + 1];
        in = len > 0 && ts >= d.t0 && te <= d.t1;
        rows = in ? len : 0;
    }
    const bool need = in && mx > 0;   // grouped[grouped['duration'] > 0] (preprocess_data.py:117)
    // the block's (count * (mean + 3 std)) terms, entry-parallel in stages of DB * DCAP entries
    // (one product per entry as the reference rounds it; ops without an SLO contribute +0.0, an
    // exact no-op on the sum); after each stage every thread adds the staged terms of its trace
    // in name order (T14: a trace's entries are contiguous, the stages ascend -- the sequential
    // sum of anormaly_detector.py:64-65).  C3 windows carry ~5k entries per block: two stages.
    const int64_t r0 = d.sv_off[tb], r1 = d.sv_off[te_];
    double expect = 0.0;
    for (int64_t c0 = r0; c0 < r1; c0 += (int64_t)DB * DCAP) {   // (block-uniform bounds)
        const int64_t c1 = min(c0 + (int64_t)DB * DCAP, r1);
        int32_t op[DCAP], cn[DCAP];   // all loads of a thread in flight together
#pragma unroll
        for (int j = 0; j < DCAP; ++j) {
            const int64_t r = min(c0 + threadIdx.x + (int64_t)j * DB, c1 - 1);
            op[j] = d.sv_op[r];
            cn[j] = d.sv_cnt[r];
        }
        double av[DCAP];
        uint8_t vv[DCAP];
#pragma unroll
        for (int j = 0; j < DCAP; ++j) {
            av[j] = d.a3[op[j]];
            vv[j] = d.a3v[op[j]];
        }
#pragma unroll
        for (int j = 0; j < DCAP; ++j) {
            const int64_t r = c0 + threadIdx.x + (int64_t)j * DB;
            if (r < c1) term[r - c0] = vv[j] ? (double)cn[j] * av[j] : 0.0;
        }
        __syncthreads();
        if (need)
            for (int64_t r = max(a, c0), re = min(b, c1); r < re; ++r) expect += term[r - c0];
        __syncthreads();
    }
    int st = 0;
    if (t < NT) {
        if (need) st = (double)mx / 1000.0 > expect ? 2 : 1;   // :58, :69
        d.state[t] = (uint8_t)st;
    }
    // counts: per wave, per block, then one add per block into one of CSH shards (~200k traces
    // on three same-address counters had cost ~0.1 ms of serialised atomics)
    __shared__ unsigned long long bc[3][DB / 64];
    const uint64_t ab = __ballot(st == 2), nr = __ballot(st == 1);
    int64_t rw = rows;
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) rw += __shfl_xor(rw, m, 64);
    const int w = threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0) {
        bc[0][w] = (unsigned long long)__popcll(ab);
        bc[1][w] = (unsigned long long)__popcll(nr);
        bc[2][w] = (unsigned long long)rw;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        unsigned long long v = 0;
        for (int k = 0; k < DB / 64; ++k) v += bc[threadIdx.x][k];
        if (v) atomicAdd(&d.counts[(size_t)(blk % CSH) * 3 + threadIdx.x], v);
    }
    return st;
}

inline DetIn mr_detect_in(const mr_spans* s, int64_t t0, int64_t t1, const double* a3, const uint8_t* a3v,
                          uint8_t* state, unsigned long long* counts) {
    return DetIn{s->tlen.p, s->tts.p, s->tte.p, s->tmaxd.p, s->sv_off.p, s->sv_op.p, s->sv_cnt.p, a3, a3v, t0, t1,
                 state, counts};
}
