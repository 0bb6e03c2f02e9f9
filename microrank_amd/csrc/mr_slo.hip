// K4: preprocess_data.get_operation_slo (preprocess_data.py:262-290) on gfx950.
//
// Per service-op over all spans: mean = (exact int64 sum) / n -- numpy's float64 sum of
// integer durations is exact below 2^53, so this is bit-identical to np.mean -- and the
// population std with numpy's pairwise summation of (x - mean)^2 in row order (numpy
// loops_utils pairwise_sum: 8 accumulators over blocks of <= 128, halving split rounded to a
// multiple of 8), then round(x/1000, 4) = rint(x/1000 * 1e4) / 1e4 (T13).  The result is
// therefore bit-exact to the reference, not just within a tolerance.
//
// Rows are grouped by a stable radix sort on the op code (row order kept inside an op, as
// pandas' groupby(...).apply(list) does).  One block per op: thread 0 enumerates the leaves
// of the pairwise tree, the block sums the leaves in parallel, thread 0 folds the leaf sums
// back in tree order.
#include <algorithm>

#include "mr_prim.h"
#include "mr_sort.h"

namespace {
constexpr int SLO_LEAVES = 4096;   // leaves per LDS pass (an op of up to ~400k spans per pass)

__global__ void k_slo_keys(const int32_t* svcop, int64_t S, uint64_t* key, uint32_t* row) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < S) {
        key[i] = (uint64_t)(uint32_t)svcop[i];
        row[i] = (uint32_t)i;
    }
}
// leaf = [lo, lo+n) with n <= 128: numpy's inner block
__device__ double pw_leaf(const double* x, int64_t n) {
    if (n < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < n; ++i) r += x[i];
        return r;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = x[j];
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += x[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += x[i];
    return res;
}

__global__ void __launch_bounds__(256) k_slo_op(const int64_t* off, const int64_t* cnt, const uint32_t* row,
                                                const int64_t* dur, int32_t n_ops, double* dev, double* mean_out,
                                                double* std_out, int64_t* count_out) {
    __shared__ int64_t leaf_lo[SLO_LEAVES];
    __shared__ int32_t leaf_n[SLO_LEAVES];
    __shared__ double leaf_v[SLO_LEAVES];
    __shared__ double s_mean;
    const int32_t o = blockIdx.x;
    if (o >= n_ops) return;
    const int64_t n = cnt[o];
    if (threadIdx.x == 0) count_out[o] = n;
    if (n == 0) {
        if (threadIdx.x == 0) mean_out[o] = std_out[o] = 0.0;
        return;
    }
    const int64_t a = off[o];
    // exact integer sum
    int64_t si = 0;
    for (int64_t i = threadIdx.x; i < n; i += 256) si += dur[row[a + i]];
    si = wave_sum_i64(si);
    __shared__ int64_t isum[256 / WAVE];
    if ((threadIdx.x & 63) == 0) isum[threadIdx.x / WAVE] = si;
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t t = 0;
        for (int w = 0; w < 256 / WAVE; ++w) t += isum[w];
        s_mean = (double)t / (double)n;
    }
    __syncthreads();
    const double mean = s_mean;
    double* x = dev + a;   // (x - mean)^2 in row order, scratch laid out like the sorted rows
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        const double d = (double)dur[row[a + i]] - mean;
        x[i] = d * d;
    }
    __syncthreads();
    // pairwise tree: explicit-stack traversal; leaves processed in LDS-sized passes
    // (thread 0 walks the tree; a pass collects up to SLO_LEAVES leaves, sums them in parallel,
    // and folds them into the running stack of partial sums)
    __shared__ int nleaves;
    __shared__ int done;
    // pass p sums leaves [p*SLO_LEAVES, (p+1)*SLO_LEAVES) (left-to-right order) in parallel and
    // parks each leaf sum at the leaf's first slot of x; the fold below walks the tree again
    int pass = 0;
    for (;;) {
        if (threadIdx.x == 0) {
            // enumerate leaves left to right, keep those of this pass
            int64_t slo[64], sn[64];
            int top = 0;
            slo[0] = 0;
            sn[0] = n;
            int64_t leaf_id = 0;
            int cnt_l = 0;
            const int64_t first = (int64_t)pass * SLO_LEAVES, last = first + SLO_LEAVES;
            while (top >= 0) {
                const int64_t lo = slo[top], m = sn[top];
                --top;
                if (m <= 128) {
                    if (leaf_id >= first && leaf_id < last) {
                        leaf_lo[cnt_l] = lo;
                        leaf_n[cnt_l] = (int32_t)m;
                        ++cnt_l;
                    }
                    ++leaf_id;
                    if (leaf_id >= last) break;
                } else {
                    int64_t n2 = m / 2;
                    n2 -= n2 % 8;
                    // push right then left (left processed first)
                    ++top;
                    slo[top] = lo + n2;
                    sn[top] = m - n2;
                    ++top;
                    slo[top] = lo;
                    sn[top] = n2;
                }
            }
            nleaves = cnt_l;
            done = (leaf_id < last) ? 1 : 0;
        }
        __syncthreads();
        const int nl = nleaves;
        for (int i = threadIdx.x; i < nl; i += 256) leaf_v[i] = pw_leaf(x + leaf_lo[i], leaf_n[i]);
        __syncthreads();
        if (threadIdx.x == 0) {
            // store leaf sums of this pass into global scratch positions (one per leaf, at its lo)
            for (int i = 0; i < nl; ++i) x[leaf_lo[i]] = leaf_v[i];
        }
        __syncthreads();
        const int d_ = done;
        __syncthreads();
        if (d_) break;
        ++pass;
    }
    // fold: the tree again, leaves read back from x[lo]
    if (threadIdx.x == 0) {
        // recursive evaluation with an explicit stack of (lo, n, state, left value)
        int64_t slo[64], sn[64];
        int ss[64];
        double sv[64];
        int top = 0;
        slo[0] = 0;
        sn[0] = n;
        ss[0] = 0;
        double ret = 0.0;
        while (top >= 0) {
            const int64_t lo = slo[top], m = sn[top];
            if (m <= 128) {
                ret = x[lo];
                --top;
            } else if (ss[top] == 0) {
                int64_t n2 = m / 2;
                n2 -= n2 % 8;
                ss[top] = 1;
                ++top;
                slo[top] = lo;
                sn[top] = n2;
                ss[top] = 0;
                continue;
            } else if (ss[top] == 1) {
                sv[top] = ret;   // left sum
                int64_t n2 = m / 2;
                n2 -= n2 % 8;
                ss[top] = 2;
                ++top;
                slo[top] = lo + n2;
                sn[top] = m - n2;
                ss[top] = 0;
                continue;
            } else {
                ret = sv[top] + ret;   // left + right
                --top;
            }
            // after a leaf or a finished node, control returns to the parent (loop continues)
        }
        const double var = ret / (double)n;
        const double sd = sqrt(var);
        // round(v, 4) == rint(v * 1e4) / 1e4 (numpy around), applied to mean/1000 and std/1000
        mean_out[o] = rint(mean / 1000.0 * 10000.0) / 10000.0;
        std_out[o] = rint(sd / 1000.0 * 10000.0) / 10000.0;
    }
}

// ops are contiguous after the stable sort: record each op's [start, end)
__global__ void k_slo_count(const uint64_t* key, int64_t S, int64_t* off, int64_t* endp) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S) return;
    const uint64_t k = key[i];
    if (i == 0 || key[i - 1] != k) off[k] = i;
    if (i == S - 1 || key[i + 1] != k) endp[k] = i + 1;
}
__global__ void k_slo_fix(const int64_t* off, const int64_t* endp, int64_t* cnt, int32_t n) {
    int32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o < n) cnt[o] = endp[o] - off[o];
}
}  // namespace

extern "C" int mr_slo(mr_ctx* ctx, const mr_spans* s, double* mean, double* std_, int64_t* count) {
    if (!ctx || !s || s->ctx != ctx || !mean || !std_ || !count) return mr_fail(ctx, MR_ERR_ARG, "mr_slo: bad arguments");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int64_t S = s->S;
    const int32_t NO = s->n_svcops;
    DBuf<uint64_t> key;
    DBuf<uint32_t> row;
    DBuf<int64_t> off, endp, cnt;
    DBuf<double> dev, dm, dsd;
    DBuf<int64_t> dc;
    MR_TRY(key.alloc(ctx, S));
    MR_TRY(row.alloc(ctx, S));
    MR_TRY(off.zero(ctx, NO + 1));
    MR_TRY(endp.zero(ctx, NO));
    MR_TRY(cnt.zero(ctx, NO));
    MR_TRY(dev.alloc(ctx, S));
    MR_TRY(dm.alloc(ctx, NO));
    MR_TRY(dsd.alloc(ctx, NO));
    MR_TRY(dc.alloc(ctx, NO));
    if (S) {
        hipLaunchKernelGGL(k_slo_keys, dim3(cdiv(S, 256)), dim3(256), 0, st, s->svcop.p, S, key.p, row.p);
        SortScratch ws;
        MR_TRY(mr_radix_sort(ctx, key.p, row.p, S, std::max(1, bits_for((uint64_t)std::max(NO - 1, 0))), ws));
        hipLaunchKernelGGL(k_slo_count, dim3(cdiv(S, 256)), dim3(256), 0, st, key.p, S, off.p, endp.p);
        hipLaunchKernelGGL(k_slo_fix, dim3(cdiv(NO, 256)), dim3(256), 0, st, off.p, endp.p, cnt.p, NO);
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // sort scratch dies here
    }
    if (NO)
        hipLaunchKernelGGL(k_slo_op, dim3(NO), dim3(256), 0, st, off.p, cnt.p, row.p, s->duration.p, NO, dev.p, dm.p,
                           dsd.p, dc.p);
    MR_TRY_HIP(ctx, hipGetLastError());
    MR_TRY(dm.download(ctx, mean, NO));
    MR_TRY(dsd.download(ctx, std_, NO));
    MR_TRY(dc.download(ctx, count, NO));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    return MR_OK;
}
