// Device primitives shared by the kernels: wave/block reductions (fixed order, so results
// are bitwise reproducible run to run) and a multi-block exclusive scan.
#pragma once
#include "mr_internal.h"

// NaN-propagating max (np.amax semantics: any NaN makes the max NaN).
__device__ __forceinline__ double nmax(double a, double b) {
    if (a != a) return a;
    if (b != b) return b;
    return a > b ? a : b;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, WAVE);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = nmax(v, __shfl_xor(v, m, WAVE));
    return v;
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, WAVE);
    return v;
}

// Block-wide reductions; every thread gets the result.  `red` must hold blockDim/64 doubles.
__device__ __forceinline__ double block_sum(double v, double* red) {
    const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE, nw = blockDim.x / WAVE;
    v = wave_sum(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    double t = 0.0;
    for (int i = 0; i < nw; ++i) t += red[i];   // fixed order
    return t;
}
__device__ __forceinline__ double block_max(double v, double* red) {
    const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE, nw = blockDim.x / WAVE;
    v = wave_max(v);
    __syncthreads();
    if (lane == 0) red[w] = v;
    __syncthreads();
    double t = -__builtin_huge_val();
    for (int i = 0; i < nw; ++i) t = nmax(t, red[i]);
    return t;
}

// Exclusive scan of int64 counts: out[i] = sum(in[0..i)), out[n] = total (out has n+1 slots).
// in == out is allowed.  Uses `tmp` device scratch of at least scan_tmp_elems(n) int64.
int64_t scan_tmp_elems(int64_t n);
// Decoupled look-back chains (single-pass scans, mr_prim.hip): status words
// [epoch:20 | flag:2 | value:42] -- flag 1 = the tile's own sum, 2 = its inclusive prefix.
// mr_dl_status hands out >= `words` per-context words with a fresh epoch (no clearing launch).
constexpr int DL_EB = 20, DL_VB = 42;
constexpr unsigned long long DL_VMASK = (1ull << DL_VB) - 1ull;
int mr_dl_status(mr_ctx* ctx, int64_t words, unsigned long long** st, uint64_t* epoch);
__device__ __forceinline__ unsigned long long dl_word(uint64_t epoch, unsigned flag, int64_t v) {
    return (epoch << (DL_VB + 2)) | ((unsigned long long)flag << DL_VB) | ((unsigned long long)v & DL_VMASK);
}
// Tile `tile` publishes its sum, walks back over the tiles before it (lower block indices: already
// dispatched) and publishes its inclusive prefix.  ONE whole wave calls it (every lane, uniformly):
// lane l polls tile (hi - l), so a poll covers 64 predecessors -- a one-thread walk pays one
// cross-XCD round trip per predecessor that has only its own sum up (~1 us each: 100 tiles had
// cost ~30 us), this one pays one per 64.  Lanes [0, L] count, L the nearest tile with its
// inclusive prefix (flag 2), and only they must have published.  Relaxed agent-scope atomics: the
// word carries its value, nothing else is published.  Returns the exclusive prefix to every lane.
__device__ __forceinline__ int64_t dl_lookback_wave(unsigned long long* st, int64_t tile, int64_t agg, uint64_t epoch) {
    const int lane = threadIdx.x & (WAVE - 1);
    if (tile == 0) {
        if (lane == 0) __hip_atomic_store(&st[0], dl_word(epoch, 2, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (lane == 0) __hip_atomic_store(&st[tile], dl_word(epoch, 1, agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int64_t excl = 0;
    for (int64_t hi = tile - 1;;) {
        const int64_t j = hi - lane;
        const unsigned long long w = j >= 0 ? __hip_atomic_load(&st[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                            : dl_word(epoch, 2, 0);
        const unsigned flag = (unsigned)(w >> DL_VB) & 3u;
        const bool ok = (w >> (DL_VB + 2)) == epoch && flag != 0;
        const unsigned long long inc = __ballot(ok && flag == 2), bad = __ballot(!ok);
        const int L = inc ? __builtin_ctzll(inc) : WAVE;
        const unsigned long long need = L == WAVE ? ~0ull : (2ull << L) - 1ull;
        if (bad & need) {   // a tile this poll needs has not published this call's value yet
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        int64_t v = lane <= L ? (int64_t)(w & DL_VMASK) : 0;
#pragma unroll
        for (int m = WAVE / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, WAVE);
        excl += v;
        if (inc) break;
        hi -= WAVE;
    }
    if (lane == 0)
        __hip_atomic_store(&st[tile], dl_word(epoch, 2, excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}
// LIMIT: the default single-pass path carries tile prefixes in the status words' 42-bit value
// field, so the total must stay below 2^42 (4.4e12); every caller scans counts of rows, pairs,
// traces or tiles (C5's 2e9 spans: < 2^31).  MR_SCAN_3PASS selects the 3-pass path (full int64).
int mr_exclusive_scan(mr_ctx* ctx, const int64_t* in, int64_t* out, int64_t n, int64_t* tmp);
// int32 counts -> int64 offsets
int mr_exclusive_scan_i32(mr_ctx* ctx, const int32_t* in, int64_t* out, int64_t n, int64_t* tmp);
