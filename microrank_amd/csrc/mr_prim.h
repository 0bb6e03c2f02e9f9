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
int mr_exclusive_scan(mr_ctx* ctx, const int64_t* in, int64_t* out, int64_t n, int64_t* tmp);
// int32 counts -> int64 offsets
int mr_exclusive_scan_i32(mr_ctx* ctx, const int32_t* in, int64_t* out, int64_t n, int64_t* tmp);
