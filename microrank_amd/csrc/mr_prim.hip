// Multi-block exclusive scan (reduce -> scan block sums -> scan tiles), 2048 elements per tile.
#include "mr_prim.h"

namespace {
constexpr int SCAN_T = 256, SCAN_I = 8, SCAN_TILE = SCAN_T * SCAN_I;

template <class In>
__global__ void __launch_bounds__(SCAN_T) k_scan_reduce(const In* in, int64_t n, int64_t* bsum) {
    __shared__ int64_t red[SCAN_T / WAVE];
    int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    int64_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_I; ++i) {
        int64_t j = base + (int64_t)i * SCAN_T + threadIdx.x;
        if (j < n) s += (int64_t)in[j];
    }
    s = wave_sum_i64(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x / WAVE] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t t = 0;
        for (int w = 0; w < SCAN_T / WAVE; ++w) t += red[w];
        bsum[blockIdx.x] = t;
    }
}

// single block: exclusive scan of nb block sums in place, total -> *total
__global__ void __launch_bounds__(1024) k_scan_blocks(int64_t* bsum, int64_t nb, int64_t* total) {
    __shared__ int64_t part[1024];
    const int tid = threadIdx.x;
    int64_t per = (nb + 1023) / 1024;
    int64_t b0 = tid * per, b1 = b0 + per < nb ? b0 + per : nb;
    int64_t s = 0;
    for (int64_t i = b0; i < b1; ++i) s += bsum[i];
    part[tid] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        int64_t v = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int64_t run = tid ? part[tid - 1] : 0;
    for (int64_t i = b0; i < b1; ++i) {
        int64_t v = bsum[i];
        bsum[i] = run;
        run += v;
    }
    if (tid == 1023) *total = part[1023];
}

template <class In>
__global__ void __launch_bounds__(SCAN_T) k_scan_tiles(const In* in, int64_t* out, int64_t n,
                                                       const int64_t* bsum) {
    __shared__ int64_t tsum[SCAN_T];
    int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
    int64_t v[SCAN_I];
    int64_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_I; ++i) {
        int64_t j = base + i;
        v[i] = j < n ? (int64_t)in[j] : 0;
        s += v[i];
    }
    tsum[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < SCAN_T; off <<= 1) {
        int64_t a = threadIdx.x >= off ? tsum[threadIdx.x - off] : 0;
        __syncthreads();
        tsum[threadIdx.x] += a;
        __syncthreads();
    }
    int64_t run = bsum[blockIdx.x] + (threadIdx.x ? tsum[threadIdx.x - 1] : 0);
#pragma unroll
    for (int i = 0; i < SCAN_I; ++i) {
        int64_t j = base + i;
        if (j < n) out[j] = run;
        run += v[i];
    }
}

template <class In>
int scan_impl(mr_ctx* ctx, const In* in, int64_t* out, int64_t n, int64_t* tmp) {
    int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (nb == 0) {
        MR_TRY_HIP(ctx, hipMemsetAsync(out, 0, sizeof(int64_t), ctx->stream));
        return MR_OK;
    }
    hipLaunchKernelGGL(k_scan_reduce<In>, dim3((unsigned)nb), dim3(SCAN_T), 0, ctx->stream, in, n, tmp);
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, ctx->stream, tmp, nb, out + n);
    hipLaunchKernelGGL(k_scan_tiles<In>, dim3((unsigned)nb), dim3(SCAN_T), 0, ctx->stream, in, out, n, tmp);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}
}  // namespace

int64_t scan_tmp_elems(int64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

int mr_exclusive_scan(mr_ctx* ctx, const int64_t* in, int64_t* out, int64_t n, int64_t* tmp) {
    return scan_impl<int64_t>(ctx, in, out, n, tmp);
}
int mr_exclusive_scan_i32(mr_ctx* ctx, const int32_t* in, int64_t* out, int64_t n, int64_t* tmp) {
    return scan_impl<int32_t>(ctx, in, out, n, tmp);
}
