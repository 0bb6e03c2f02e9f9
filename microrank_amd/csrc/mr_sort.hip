// Stable LSD radix sort of 64-bit keys (optionally carrying 32-bit values), 8-bit digits.
// Per pass: block histograms (digit-major) -> exclusive scan -> stable scatter.  Stability
// inside a block comes from ranking keys in position order: chunk by chunk, wave by wave,
// and within a wave by lane (peer masks from 8 ballots, one per digit bit).
#include "mr_prim.h"
#include "mr_sort.h"

namespace {
constexpr int RT = 256;               // threads per block
constexpr int RC = 8;                 // chunks of RT keys per block (tile = 2048 keys)
constexpr int RTILE = RT * RC;
constexpr int NW = RT / WAVE;

__global__ void __launch_bounds__(RT) k_radix_hist(const uint64_t* keys, int64_t n, int shift, int64_t nb,
                                                   int64_t* hist) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const int64_t base = (int64_t)blockIdx.x * RTILE;
#pragma unroll
    for (int c = 0; c < RC; ++c) {
        int64_t i = base + (int64_t)c * RT + threadIdx.x;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    hist[(int64_t)threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];   // digit-major
}

__device__ __forceinline__ uint64_t peers_of(uint32_t digit) {
    uint64_t m = ~0ull;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        uint64_t bal = __ballot((digit >> b) & 1u);
        m &= ((digit >> b) & 1u) ? bal : ~bal;
    }
    return m;
}

template <bool HASV>
__global__ void __launch_bounds__(RT) k_radix_scatter(const uint64_t* keys, const uint32_t* vals, uint64_t* okeys,
                                                      uint32_t* ovals, int64_t n, int shift, int64_t nb,
                                                      const int64_t* offs) {
    __shared__ int64_t run[256];
    __shared__ uint32_t wcnt[NW][256];
    const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    run[threadIdx.x] = offs[(int64_t)threadIdx.x * nb + blockIdx.x];
    const int64_t base = (int64_t)blockIdx.x * RTILE;
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int c = 0; c < RC; ++c) {
        for (int i = threadIdx.x; i < NW * 256; i += RT) (&wcnt[0][0])[i] = 0;
        __syncthreads();
        const int64_t i = base + (int64_t)c * RT + threadIdx.x;
        const bool valid = i < n;
        uint64_t k = valid ? keys[i] : 0ull;
        uint32_t dg = valid ? (uint32_t)((k >> shift) & 255u) : 256u;   // 256: sentinel, never written
        uint64_t act = __ballot(valid);
        uint64_t pm = peers_of(dg & 255u) & act;
        if (!valid) pm = 0;
        const uint32_t rank = (uint32_t)__popcll(pm & lt);
        if (valid && rank == 0) wcnt[w][dg] = (uint32_t)__popcll(pm);
        __syncthreads();
        if (valid) {
            int64_t pos = run[dg] + rank;
            for (int ww = 0; ww < w; ++ww) pos += wcnt[ww][dg];
            okeys[pos] = k;
            if (HASV) ovals[pos] = vals[i];
        }
        __syncthreads();
        uint32_t tot = 0;
        for (int ww = 0; ww < NW; ++ww) tot += wcnt[ww][threadIdx.x];
        run[threadIdx.x] += tot;
        __syncthreads();
    }
}

__global__ void k_copy_u64(const uint64_t* a, uint64_t* b, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}
__global__ void k_copy_u32(const uint32_t* a, uint32_t* b, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}
// small n: one launch, one block; bitonic sort in LDS of (masked key, position) pairs, so equal
// keys keep their input order (stable, like the radix path)
constexpr int SL_MAX = 4096, SL_T = 1024;
__global__ void __launch_bounds__(SL_T) k_sort_lds(uint64_t* keys, uint32_t* vals, int32_t n, uint64_t mask) {
    __shared__ uint64_t sk[SL_MAX];
    __shared__ uint32_t sp[SL_MAX];
    int32_t m = 1;
    while (m < n) m <<= 1;
    for (int32_t i = threadIdx.x; i < m; i += SL_T) {
        sk[i] = i < n ? (keys[i] & mask) : ~0ull;
        sp[i] = (uint32_t)i;
    }
    __syncthreads();
    for (int32_t k = 2; k <= m; k <<= 1) {
        for (int32_t j = k >> 1; j > 0; j >>= 1) {
            for (int32_t i = threadIdx.x; i < m; i += SL_T) {
                const int32_t l = i ^ j;
                if (l > i) {
                    const uint64_t a = sk[i], b = sk[l];
                    const uint32_t pa = sp[i], pb = sp[l];
                    const bool gt = a > b || (a == b && pa > pb);
                    if (((i & k) == 0) == gt) {   // ascending in the lower half of each k-run
                        sk[i] = b;
                        sk[l] = a;
                        sp[i] = pb;
                        sp[l] = pa;
                    }
                }
            }
            __syncthreads();
        }
    }
    // gather the originals in sorted order (keys keep their unmasked bits)
    uint64_t ok[SL_MAX / SL_T];
    uint32_t ov[SL_MAX / SL_T];
#pragma unroll
    for (int r = 0; r < SL_MAX / SL_T; ++r) {
        const int32_t i = threadIdx.x + r * SL_T;
        if (i < n) {
            ok[r] = keys[sp[i]];
            if (vals) ov[r] = vals[sp[i]];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < SL_MAX / SL_T; ++r) {
        const int32_t i = threadIdx.x + r * SL_T;
        if (i < n) {
            keys[i] = ok[r];
            if (vals) vals[i] = ov[r];
        }
    }
}
}  // namespace

int mr_radix_sort(mr_ctx* ctx, uint64_t* keys, uint32_t* vals, int64_t n, int bits, SortScratch& ws) {
    if (n <= 1 || bits <= 0) return MR_OK;
    if (n <= SL_MAX) {
        const uint64_t mask = bits >= 64 ? ~0ull : ((1ull << bits) - 1ull);
        hipLaunchKernelGGL(k_sort_lds, dim3(1), dim3(SL_T), 0, ctx->stream, keys, vals, (int32_t)n, mask);
        MR_TRY_HIP(ctx, hipGetLastError());
        return MR_OK;
    }
    const int64_t nb = (n + RTILE - 1) / RTILE;
    MR_TRY(ws.k2.alloc(ctx, (size_t)n));
    if (vals) MR_TRY(ws.v2.alloc(ctx, (size_t)n));
    MR_TRY(ws.hist.alloc(ctx, (size_t)(256 * nb + 1)));
    MR_TRY(ws.tmp.alloc(ctx, (size_t)scan_tmp_elems(256 * nb)));
    uint64_t *ka = keys, *kb = ws.k2.p;
    uint32_t *va = vals, *vb = vals ? ws.v2.p : nullptr;
    const int passes = (bits + 7) / 8;
    for (int p = 0; p < passes; ++p) {
        const int shift = 8 * p;
        hipLaunchKernelGGL(k_radix_hist, dim3((unsigned)nb), dim3(RT), 0, ctx->stream, ka, n, shift, nb, ws.hist.p);
        MR_TRY(mr_exclusive_scan(ctx, ws.hist.p, ws.hist.p, 256 * nb, ws.tmp.p));
        if (vals)
            hipLaunchKernelGGL(k_radix_scatter<true>, dim3((unsigned)nb), dim3(RT), 0, ctx->stream, ka, va, kb, vb, n,
                               shift, nb, ws.hist.p);
        else
            hipLaunchKernelGGL(k_radix_scatter<false>, dim3((unsigned)nb), dim3(RT), 0, ctx->stream, ka, va, kb, vb, n,
                               shift, nb, ws.hist.p);
        std::swap(ka, kb);
        std::swap(va, vb);
    }
    if (ka != keys) {
        hipLaunchKernelGGL(k_copy_u64, dim3(cdiv(n, 256)), dim3(256), 0, ctx->stream, ka, keys, n);
        if (vals) hipLaunchKernelGGL(k_copy_u32, dim3(cdiv(n, 256)), dim3(256), 0, ctx->stream, va, vals, n);
    }
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}

int bits_for(uint64_t maxval) {
    int b = 0;
    while (b < 64 && (maxval >> b)) ++b;
    return b;
}
