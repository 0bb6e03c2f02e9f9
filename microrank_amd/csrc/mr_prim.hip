// Exclusive scan: one block for small n, else one decoupled look-back launch of 2048-element tiles.
#include "mr_prim.h"

namespace {
constexpr int SCAN_T = 256, SCAN_I = 8, SCAN_TILE = SCAN_T * SCAN_I;

// small n: one launch, one 1024-thread block walking tiles of 8192 with a running carry
constexpr int SS_T = 1024, SS_I = 8;
constexpr int64_t SCAN_SINGLE_MAX = 2 * SS_T * SS_I;
template <class In>
__global__ void __launch_bounds__(SS_T) k_scan_single(const In* in, int64_t* out, int64_t n) {
    __shared__ int64_t wsum[SS_T / WAVE];
    const int tid = threadIdx.x, lane = tid & (WAVE - 1), w = tid / WAVE;
    int64_t carry = 0;
    for (int64_t base = 0; base < n; base += (int64_t)SS_T * SS_I) {
        int64_t v[SS_I], s = 0;
#pragma unroll
        for (int j = 0; j < SS_I; ++j) {
            const int64_t idx = base + (int64_t)tid * SS_I + j;
            v[j] = idx < n ? (int64_t)in[idx] : 0;
            s += v[j];
        }
        int64_t inc = s;   // inclusive scan over the wave
#pragma unroll
        for (int off = 1; off < WAVE; off <<= 1) {
            const int64_t o = __shfl_up(inc, off, WAVE);
            if (lane >= off) inc += o;
        }
        if (lane == WAVE - 1) wsum[w] = inc;
        __syncthreads();
        int64_t wpre = 0, tot = 0;
        for (int k = 0; k < SS_T / WAVE; ++k) {
            if (k < w) wpre += wsum[k];
            tot += wsum[k];
        }
        int64_t run = carry + wpre + inc - s;
#pragma unroll
        for (int j = 0; j < SS_I; ++j) {
            const int64_t idx = base + (int64_t)tid * SS_I + j;
            if (idx < n) out[idx] = run;
            run += v[j];
        }
        carry += tot;
        __syncthreads();   // wsum reused by the next tile
    }
    if (tid == 0) out[n] = carry;
}

// larger n: ONE launch, a tile of SCAN_TILE per block, tiles chained by decoupled look-back.  A
// tile publishes its sum (flag 1), then -- once its exclusive prefix is known from the tiles
// before it -- its inclusive prefix (flag 2); a block waits only on lower block indices, which
// the dispatcher has already placed.  Status words [epoch:20 | flag:2 | value:42] live in a
// per-context buffer; the epoch changes every call, so no clearing launch is needed (the buffer
// is cleared once per 2^20 calls, when the epoch wraps).  Relaxed agent-scope atomics (sc1):
// the word carries its value, no other data is published through it.
template <class In>
__global__ void __launch_bounds__(SCAN_T) k_scan_dl(const In* in, int64_t* out, int64_t n, unsigned long long* st,
                                                    uint64_t epoch) {
    __shared__ int64_t tsum[SCAN_T];
    __shared__ int64_t s_excl;
    const int64_t tile = blockIdx.x;
    const int64_t base = tile * SCAN_TILE + (int64_t)threadIdx.x * SCAN_I;
    int64_t v[SCAN_I];
    int64_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_I; ++i) {
        const int64_t j = base + i;
        v[i] = j < n ? (int64_t)in[j] : 0;
        s += v[i];
    }
    tsum[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < SCAN_T; off <<= 1) {
        const int64_t a = threadIdx.x >= off ? tsum[threadIdx.x - off] : 0;
        __syncthreads();
        tsum[threadIdx.x] += a;
        __syncthreads();
    }
    const int64_t agg = tsum[SCAN_T - 1];
    if (threadIdx.x < WAVE) {
        const int64_t excl = dl_lookback_wave(st, tile, agg, epoch);
        if (threadIdx.x == 0) {
            s_excl = excl;
            if (tile == (int64_t)gridDim.x - 1) out[n] = excl + agg;
        }
    }
    __syncthreads();
    int64_t run = s_excl + (threadIdx.x ? tsum[threadIdx.x - 1] : 0);
#pragma unroll
    for (int i = 0; i < SCAN_I; ++i) {
        const int64_t j = base + i;
        if (j < n) out[j] = run;
        run += v[i];
    }
}

template <class In>
int scan_impl(mr_ctx* ctx, const In* in, int64_t* out, int64_t n, int64_t* tmp) {
    if (n > 0 && n <= SCAN_SINGLE_MAX) {
        hipLaunchKernelGGL(k_scan_single<In>, dim3(1), dim3(SS_T), 0, ctx->stream, in, out, n);
        MR_TRY_HIP(ctx, hipGetLastError());
        return MR_OK;
    }
    int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (nb == 0) {
        MR_TRY_HIP(ctx, hipMemsetAsync(out, 0, sizeof(int64_t), ctx->stream));
        return MR_OK;
    }
    unsigned long long* st = nullptr;
    uint64_t epoch = 0;
    MR_TRY(mr_dl_status(ctx, nb, &st, &epoch));
    hipLaunchKernelGGL(k_scan_dl<In>, dim3((unsigned)nb), dim3(SCAN_T), 0, ctx->stream, in, out, n, st, epoch);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}
}  // namespace

int64_t scan_tmp_elems(int64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

int mr_dl_status(mr_ctx* ctx, int64_t words, unsigned long long** st, uint64_t* epoch) {
    if ((size_t)words > ctx->scan_cap) {   // grow the status words (stream-ordered: sync first)
        MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
        if (ctx->scan_st) MR_TRY_HIP(ctx, hipFree(ctx->scan_st));
        ctx->scan_st = nullptr;
        const size_t cap = std::max<size_t>((size_t)words, 8192);
        MR_TRY_HIP(ctx, hipMalloc((void**)&ctx->scan_st, cap * sizeof(unsigned long long)));
        MR_TRY_HIP(ctx, hipMemsetAsync(ctx->scan_st, 0, cap * sizeof(unsigned long long), ctx->stream));
        ctx->scan_cap = cap;
        ctx->scan_epoch = 0;
    }
    ctx->scan_epoch = (ctx->scan_epoch + 1) & ((1u << DL_EB) - 1u);
    if (ctx->scan_epoch == 0) {   // wrapped: clear every word (epoch 0 marks a cleared word)
        MR_TRY_HIP(ctx, hipMemsetAsync(ctx->scan_st, 0, ctx->scan_cap * sizeof(unsigned long long), ctx->stream));
        ctx->scan_epoch = 1;
    }
    *st = ctx->scan_st;
    *epoch = ctx->scan_epoch;
    return MR_OK;
}

int mr_exclusive_scan(mr_ctx* ctx, const int64_t* in, int64_t* out, int64_t n, int64_t* tmp) {
    return scan_impl<int64_t>(ctx, in, out, n, tmp);
}
int mr_exclusive_scan_i32(mr_ctx* ctx, const int32_t* in, int64_t* out, int64_t n, int64_t* tmp) {
    return scan_impl<int32_t>(ctx, in, out, n, tmp);
}
