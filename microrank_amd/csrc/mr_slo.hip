// K4: preprocess_data.get_operation_slo (preprocess_data.py:50-78) on gfx950.
//
// Per service-op over all spans (row order kept inside an op, as pandas'
// groupby(...).apply(list) does): mean = (exact int64 sum) / n -- numpy's float64 sum of integer
// durations is exact below 2^53, so this is bit-identical to np.mean -- and the population std
// as np.std computes it: the squared deviations are reduced by np.add.reduce, which numpy runs
// over 8192-element buffers (NPY_BUFSIZE) accumulated sequentially, each buffer summed pairwise
// (loops_utils pairwise_sum: 8 accumulators over blocks of <= 128, halving split rounded down to
// a multiple of 8).  Then round(x/1000, 4) = rint(x/1000 * 1e4) / 1e4 (T13).  Bit-exact, pinned
// by tests/golden/slo_large.json (ops of 1..131075 spans).
//
// Work decomposition: rows are grouped by a stable radix sort on the op code; every op is cut
// into numpy's 8192-element chunks and the chunks of all ops form one flat grid:
//   k_slo_isum   one wave per chunk: exact int64 partial sums        (coalesced)
//   k_slo_mean   one thread per op: mean = sum / n
//   k_slo_pw     one 128-thread block per chunk: the pairwise tree of a chunk has depth <= 7
//                below the chunk root (a right child is at most half + 8), so thread h owns the
//                subtree at heap position h of depth 7; threads whose path reaches a leaf
//                (<= 128 elements) early stand for that leaf if they are its leftmost
//                descendant.  Leaf sums are then folded level by level in LDS: a node adds its
//                children iff it is internal, so the fold reproduces numpy's tree exactly.
//   k_slo_final  one thread per op: chunk sums added in chunk order, sqrt, rounding.
#include <algorithm>
#include <vector>

#include "mr_prim.h"
#include "mr_sort.h"

namespace {
constexpr int64_t NPY_BUF = 8192;   // numpy's default ufunc buffer size
constexpr int PW_BLOCK = 128;       // numpy's PW_BLOCKSIZE
constexpr int PW_DEPTH = 7;         // 8192 -> 128 worst-case levels, see above
constexpr int PW_SLOTS = 1 << PW_DEPTH;

__global__ void k_slo_keys(const int32_t* svcop, int64_t S, uint64_t* key, uint32_t* row) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < S) {
        key[i] = (uint64_t)(uint32_t)svcop[i];
        row[i] = (uint32_t)i;
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

struct Chunk {
    int64_t beg;   // first sorted-row position
    int32_t n;     // <= NPY_BUF
    int32_t op;
};

// exact integer partial sum of one chunk (a wave per chunk, 4 chunks per block)
__global__ void __launch_bounds__(256) k_slo_isum(const Chunk* ch, int64_t K, const uint32_t* row, const int64_t* dur,
                                                  int64_t* isum) {
    const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= K) return;
    const Chunk c = ch[k];
    int64_t s = 0;
    for (int i = threadIdx.x & 63; i < c.n; i += 64) s += dur[row[c.beg + i]];
    s = wave_sum_i64(s);
    if ((threadIdx.x & 63) == 0) isum[k] = s;
}
__global__ void k_slo_mean(const int64_t* cnt, const int64_t* ch0, const int64_t* isum, int32_t n_ops, double* mean) {
    const int32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_ops) return;
    const int64_t n = cnt[o];
    int64_t t = 0;
    for (int64_t k = ch0[o]; k < ch0[o + 1]; ++k) t += isum[k];
    mean[o] = n ? (double)t / (double)n : 0.0;
}

// numpy's inner block for m <= 128 elements, squared deviations computed on the fly
__device__ __forceinline__ double sq(const uint32_t* row, const int64_t* dur, int64_t i, double mean) {
    const double d = (double)dur[row[i]] - mean;
    return d * d;
}
__device__ double pw_leaf(const uint32_t* row, const int64_t* dur, int64_t lo, int m, double mean) {
    if (m < 8) {
        double r = 0.0;
        for (int i = 0; i < m; ++i) r += sq(row, dur, lo + i, mean);
        return r;
    }
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = sq(row, dur, lo + j, mean);
    int i = 8;
    for (; i < m - (m % 8); i += 8)
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += sq(row, dur, lo + i + j, mean);
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < m; ++i) res += sq(row, dur, lo + i, mean);
    return res;
}

__global__ void __launch_bounds__(PW_SLOTS) k_slo_pw(const Chunk* ch, const uint32_t* row, const int64_t* dur,
                                                     const double* mean, double* csum) {
    __shared__ double val[PW_SLOTS];
    __shared__ uint8_t leafd[PW_SLOTS];   // depth at which this slot's path reached a leaf
    const Chunk c = ch[blockIdx.x];
    const int h = threadIdx.x;
    int64_t lo = 0;
    int m = c.n;
    int depth = 0;
    bool rep = true;
    for (; depth < PW_DEPTH; ++depth) {
        if (m <= PW_BLOCK) {
            rep = (h & ((1 << (PW_DEPTH - depth)) - 1)) == 0;   // leftmost descendant stands for the leaf
            break;
        }
        int n2 = m / 2;
        n2 -= n2 % 8;
        if ((h >> (PW_DEPTH - 1 - depth)) & 1) {
            lo += n2;
            m -= n2;
        } else {
            m = n2;
        }
    }
    leafd[h] = (uint8_t)depth;
    // depth == PW_DEPTH implies m <= 128: a child has at most ceil(m/2) + 7 elements, and
    // 8192 -> 4103 -> 2059 -> 1037 -> 526 -> 270 -> 142 -> 78 bounds the deepest path
    val[h] = rep ? pw_leaf(row, dur, c.beg + lo, m, mean[c.op]) : 0.0;
    __syncthreads();
    // fold: a node at depth L (leftmost slot s) is internal iff its leftmost path went deeper
    for (int L = PW_DEPTH - 1; L >= 0; --L) {
        const int span = 1 << (PW_DEPTH - L);
        if ((h & (span - 1)) == 0 && leafd[h] > L) val[h] = val[h] + val[h + span / 2];
        __syncthreads();
    }
    if (h == 0) csum[blockIdx.x] = val[0];
}

__global__ void k_slo_final(const int64_t* cnt, const int64_t* ch0, const double* csum, const double* mean, int32_t n_ops,
                            double* mean_out, double* std_out, int64_t* count_out) {
    const int32_t o = blockIdx.x * blockDim.x + threadIdx.x;
    if (o >= n_ops) return;
    const int64_t n = cnt[o];
    count_out[o] = n;
    if (n == 0) {
        mean_out[o] = std_out[o] = 0.0;
        return;
    }
    double acc = 0.0;   // DOUBLE_add reduce: io1 += pairwise_sum(buffer), buffers in order
    for (int64_t k = ch0[o]; k < ch0[o + 1]; ++k) acc += csum[k];
    const double sd = sqrt(acc / (double)n);
    mean_out[o] = rint(mean[o] / 1000.0 * 10000.0) / 10000.0;
    std_out[o] = rint(sd / 1000.0 * 10000.0) / 10000.0;
}
}  // namespace

extern "C" int mr_slo(mr_ctx* ctx, const mr_spans* s, double* mean, double* std_, int64_t* count) {
    if (!ctx || !s || s->ctx != ctx || !mean || !std_ || !count) return mr_fail(ctx, MR_ERR_ARG, "mr_slo: bad arguments");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    const int64_t S = s->S;
    const int32_t NO = s->n_svcops;
    if (NO == 0) return MR_OK;
    std::vector<int64_t> h_off(NO, 0), h_end(NO, 0);
    DBuf<uint64_t> key;
    DBuf<uint32_t> row;
    DBuf<int64_t> off, endp;
    MR_TRY(key.alloc(ctx, S));
    MR_TRY(row.alloc(ctx, S));
    MR_TRY(off.zero(ctx, NO));
    MR_TRY(endp.zero(ctx, NO));
    if (S) {
        hipLaunchKernelGGL(k_slo_keys, dim3(cdiv(S, 256)), dim3(256), 0, st, s->svcop.p, S, key.p, row.p);
        SortScratch ws;
        MR_TRY(mr_radix_sort(ctx, key.p, row.p, S, std::max(1, bits_for((uint64_t)std::max(NO - 1, 0))), ws));
        hipLaunchKernelGGL(k_slo_count, dim3(cdiv(S, 256)), dim3(256), 0, st, key.p, S, off.p, endp.p);
        MR_TRY(off.download(ctx, h_off.data(), NO));
        MR_TRY(endp.download(ctx, h_end.data(), NO));
        MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    }
    // chunk table: numpy's 8192-element buffers of every op, ops in code order
    std::vector<Chunk> hch;
    std::vector<int64_t> hch0(NO + 1), hcnt(NO);
    for (int32_t o = 0; o < NO; ++o) {
        hch0[o] = (int64_t)hch.size();
        hcnt[o] = h_end[o] - h_off[o];
        for (int64_t b = 0; b < hcnt[o]; b += NPY_BUF)
            hch.push_back(Chunk{h_off[o] + b, (int32_t)std::min<int64_t>(NPY_BUF, hcnt[o] - b), o});
    }
    hch0[NO] = (int64_t)hch.size();
    const int64_t K = (int64_t)hch.size();
    DBuf<Chunk> dch;
    DBuf<int64_t> dch0, dcnt, isum, dc;
    DBuf<double> dmean, csum, dm, dsd;
    MR_TRY(dch0.upload(ctx, hch0.data(), NO + 1));
    MR_TRY(dcnt.upload(ctx, hcnt.data(), NO));
    MR_TRY(dmean.alloc(ctx, NO));
    MR_TRY(dm.alloc(ctx, NO));
    MR_TRY(dsd.alloc(ctx, NO));
    MR_TRY(dc.alloc(ctx, NO));
    if (K) {
        MR_TRY(dch.upload(ctx, hch.data(), K));
        MR_TRY(isum.alloc(ctx, K));
        MR_TRY(csum.alloc(ctx, K));
        hipLaunchKernelGGL(k_slo_isum, dim3(cdiv(K, 4)), dim3(256), 0, st, dch.p, K, row.p, s->duration.p, isum.p);
    }
    hipLaunchKernelGGL(k_slo_mean, dim3(cdiv(NO, 256)), dim3(256), 0, st, dcnt.p, dch0.p, isum.p, NO, dmean.p);
    if (K) hipLaunchKernelGGL(k_slo_pw, dim3(K), dim3(PW_SLOTS), 0, st, dch.p, row.p, s->duration.p, dmean.p, csum.p);
    hipLaunchKernelGGL(k_slo_final, dim3(cdiv(NO, 256)), dim3(256), 0, st, dcnt.p, dch0.p, csum.p, dmean.p, NO, dm.p,
                       dsd.p, dc.p);
    MR_TRY_HIP(ctx, hipGetLastError());
    MR_TRY(dm.download(ctx, mean, NO));
    MR_TRY(dsd.download(ctx, std_, NO));
    MR_TRY(dc.download(ctx, count, NO));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));
    return MR_OK;
}
