// SURVEY §8(f) f2 -- span ingest on the device: the OTel span export (collect_data.py:35-46,
// renamed at online_rca.py:221-244) as Arrow-style string columns -> the int-coded span table
// (mr_spans) with the dictionaries the reference's string operations imply:
//   * traceID codes = rank in sorted (code-point) order: the groupby/sort order of
//     preprocess_data.py:165 and anormaly_detector.py:56 (T10);
//   * podop = podName + '_' + op, svcop = serviceName + '_' + op, op = operationName or, for
//     service ts-ui-dashboard, operationName.rsplit('/', 1)[0] (preprocess_data.py:26-33, 53-57,
//     100-104, 151-155), each coded by rank in sorted order -- the names themselves are compared,
//     so two (pod, op) pairs that concatenate to one name share a code, as in pandas;
//   * spanID codes by equality only; ParentSpanId -> the code of the equal spanID, or -1 (null,
//     or no such span: the merge at :157-158 finds nothing).
// UTF-8 byte order equals code-point order, so sorting bytes sorts like Python str.
//
// Per dictionary: a 64-bit hash of every row's name, a radix sort of (hash, row) -> runs of
// equal hashes -> every row compared byte for byte with its run's first row (a collision retries
// with another seed, never a wrong code) -> the distinct names sorted
// by LSD passes over big-endian 8-byte chunks (a length pass first: a prefix sorts first) ->
// codes.  All passes are streaming integer work: HBM-bound, no MFMA.
#include <algorithm>
#include <climits>
#include <cstring>
#include <vector>

#include "mr_prim.h"
#include "mr_sort.h"

int mr_spans_finish(mr_ctx* ctx, mr_spans* s);   // mr_graph_build.hip: spanID multimap + index

namespace {
constexpr int IB = 256;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// A row's name: segment A, then (join) '_' + segment B.  Bytes come from 8-aligned word loads
// (the byte buffers carry 16 zero bytes of tail padding).
struct VStr {
    const uint8_t* a;
    int64_t la;
    const uint8_t* b;
    int64_t lb;
    bool join;
    __device__ int64_t len() const { return join ? la + 1 + lb : la; }
};
__device__ __forceinline__ uint64_t load8(const uint8_t* p) {   // 8 bytes from any address, little-endian
    const uintptr_t u = (uintptr_t)p;
    const uint64_t* w = (const uint64_t*)(u & ~(uintptr_t)7);
    const int sh = (int)(u & 7) * 8;
    const uint64_t w0 = w[0];
    return sh ? (w0 >> sh) | (w[1] << (64 - sh)) : w0;
}
// 8 bytes of a segment starting at byte `off` (zero beyond its end)
__device__ __forceinline__ uint64_t seg8(const uint8_t* p, int64_t len, int64_t off) {
    if (off >= len) return 0;
    const uint64_t v = load8(p + off);
    const int64_t n = len - off;
    return n >= 8 ? v : v & ((1ull << (8 * n)) - 1ull);
}
// bytes [8k, 8k+8) of the name, little-endian, zero padded
__device__ uint64_t vchunk(const VStr& s, int64_t k) {
    const int64_t o = 8 * k;
    if (!s.join) return seg8(s.a, s.la, o);
    uint64_t v = 0;
    if (o < s.la) v = seg8(s.a, s.la, o);
    const int64_t us = s.la - o;   // position of '_' inside this chunk
    if (us >= 0 && us < 8) v |= (uint64_t)'_' << (8 * us);
    // segment B starts at la + 1
    const int64_t bo = o - (s.la + 1);
    if (bo >= 0) {
        v |= seg8(s.b, s.lb, bo);
    } else if (bo > -8) {   // B starts inside this chunk at byte -bo
        v |= seg8(s.b, s.lb, 0) << (8 * (-bo));
    }
    return v;
}
// hash of the byte sequence over its 8-byte chunks (the same chunks the sort and the comparison
// read, so a name hashes alike however it is split into segments); seeded per attempt
__device__ uint64_t vhash(const VStr& s, uint64_t seed) {
    const int64_t n = s.len();
    uint64_t h = mix64(seed ^ (uint64_t)n);
    for (int64_t k = 0; 8 * k < n; ++k) h = mix64(h ^ (vchunk(s, k) * 0x9e3779b97f4a7c15ull + (uint64_t)k));
    return h;
}
__device__ bool veq(const VStr& s, const VStr& t) {
    const int64_t n = s.len();
    if (n != t.len()) return false;
    for (int64_t k = 0; 8 * k < n; ++k)
        if (vchunk(s, k) != vchunk(t, k)) return false;
    return true;
}
__device__ __forceinline__ uint64_t bswap64(uint64_t v) { return __builtin_bswap64(v); }

// column c of the ingest: raw (trace / span / parent) or joined (podop / svcop)
struct Cols {
    const int64_t* off[6];    // traceID, spanID, ParentSpanId, serviceName, operationName, podName
    const uint8_t* bytes[6];
    const uint8_t* valid2;    // ParentSpanId validity (Arrow bitmap, LSB first) or null
    const int32_t* op_len;    // operationName length after the ts-ui-dashboard rule
};
enum { C_TRACE = 0, C_SPAN = 1, C_PARENT = 2, C_SVC = 3, C_OP = 4, C_POD = 5 };
// dictionary d: 0 trace, 1 podop, 2 svcop, 3 span, 4 parent (looked up in span's)
__device__ __forceinline__ VStr row_str(const Cols& c, int d, int64_t i) {
    VStr s;
    if (d == 1 || d == 2) {
        const int ca = d == 1 ? C_POD : C_SVC;
        s.a = c.bytes[ca] + c.off[ca][i];
        s.la = c.off[ca][i + 1] - c.off[ca][i];
        s.b = c.bytes[C_OP] + c.off[C_OP][i];
        s.lb = c.op_len[i];
        s.join = true;
    } else {
        const int cc = d == 0 ? C_TRACE : d == 3 ? C_SPAN : C_PARENT;
        s.a = c.bytes[cc] + c.off[cc][i];
        s.la = c.off[cc][i + 1] - c.off[cc][i];
        s.b = nullptr;
        s.lb = 0;
        s.join = false;
    }
    return s;
}

// operationName with the ts-ui-dashboard rule: rsplit('/', 1)[0] (the part before the last '/';
// '/' is one byte that never occurs inside a UTF-8 multibyte sequence)
__global__ void k_op_len(Cols c, int64_t S, int32_t* op_len) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S) return;
    const int64_t o0 = c.off[C_OP][i], o1 = c.off[C_OP][i + 1];
    int64_t n = o1 - o0;
    const int64_t s0 = c.off[C_SVC][i], s1 = c.off[C_SVC][i + 1];
    const char ui[] = "ts-ui-dashboard";
    bool is_ui = s1 - s0 == 15;
    for (int j = 0; is_ui && j < 15; ++j) is_ui = c.bytes[C_SVC][s0 + j] == (uint8_t)ui[j];
    if (is_ui) {
        const uint8_t* p = c.bytes[C_OP] + o0;
        for (int64_t j = n - 1; j >= 0; --j)
            if (p[j] == '/') {
                n = j;
                break;
            }
    }
    op_len[i] = (int32_t)n;
}
__global__ void k_row_hash(Cols c, int d, int64_t S, uint64_t x, uint64_t* key, uint32_t* val) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S) return;
    key[i] = vhash(row_str(c, d, i), x);
    val[i] = (uint32_t)i;
}
__global__ void k_heads64(const uint64_t* key, int64_t n, int32_t* head) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) head[i] = (i == 0 || key[i] != key[i - 1]) ? 1 : 0;
}
// run of sorted position i: cls[row] = run, rep[run] = first row (the smallest: stable sort over
// row order), rkey[run] = hash
__global__ void k_runs(const uint64_t* key, const uint32_t* val, const int32_t* head, const int64_t* hpos, int64_t n,
                       int32_t* cls, int32_t* rep, uint64_t* rkey) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t r = hpos[i + 1] - 1;   // inclusive: the run this position belongs to
    cls[val[i]] = (int32_t)r;
    if (head[i]) {
        rep[r] = (int32_t)val[i];
        if (rkey) rkey[r] = key[i];
    }
}
// every row equal to its run's first row, byte for byte (else: a hash collision)
__global__ void k_verify(Cols c, int d, int64_t S, const int32_t* cls, const int32_t* rep, int32_t* bad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S) return;
    const int32_t r = rep[cls[i]];
    if (r != (int32_t)i && !veq(row_str(c, d, i), row_str(c, d, r))) atomicOr(bad, 1);
}
// sort passes over the distinct names (perm: current order of runs)
__global__ void k_len_key(Cols c, int d, const int32_t* rep, int64_t U, uint64_t* key, uint32_t* perm) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= U) return;
    key[u] = (uint64_t)row_str(c, d, rep[u]).len();
    perm[u] = (uint32_t)u;
}
__global__ void k_chunk_key(Cols c, int d, const int32_t* rep, const uint32_t* perm, int64_t U, int64_t k,
                            uint64_t* key) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= U) return;
    key[i] = bswap64(vchunk(row_str(c, d, rep[perm[i]]), k));   // big-endian: numeric = byte order
}
// code of run perm[i] = i; the representative row of each code (for the host's name lists)
__global__ void k_rank(const uint32_t* perm, int64_t U, const int32_t* rep, int32_t* code_of_run, int32_t* rep_sorted) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= U) return;
    code_of_run[perm[i]] = (int32_t)i;
    rep_sorted[i] = rep[perm[i]];
}
template <class T>
__global__ void k_codes(const int32_t* cls, const int32_t* code_of_run, int64_t S, T* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < S) out[i] = (T)(code_of_run ? code_of_run[cls[i]] : cls[i]);
}
// ParentSpanId -> span code: binary search of its hash among the spanID runs (sorted by hash,
// distinct after verification), then an exact comparison with that run's first row
__global__ void k_parent(Cols c, int64_t S, uint64_t x, const uint64_t* rkey, const int32_t* rep, int64_t U,
                         int64_t* parent) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= S) return;
    int64_t out = -1;
    const bool ok = !c.valid2 || ((c.valid2[i >> 3] >> (i & 7)) & 1u);
    if (ok) {
        const VStr p = row_str(c, 4, i);
        const uint64_t h = vhash(p, x);
        int64_t lo = 0, hi = U;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (rkey[mid] < h) lo = mid + 1;
            else hi = mid;
        }
        if (lo < U && rkey[lo] == h && veq(p, row_str(c, 3, rep[lo]))) out = lo;
    }
    parent[i] = out;
}
}  // namespace

struct IngestDict {
    int64_t U = 0;
    DBuf<int32_t> cls, rep, code_of_run, rep_sorted;
    DBuf<uint64_t> rkey;
};

// one dictionary: runs of equal names (verified) and, when `sorted`, codes in name order
static int build_dict(mr_ctx* ctx, const Cols& c, int d, int64_t S, bool sorted, IngestDict& D, uint64_t* x_used) {
    hipStream_t st = ctx->stream;
    DBuf<uint64_t> key;
    DBuf<uint32_t> val;
    DBuf<int32_t> head, bad;
    DBuf<int64_t> hpos, tmp;
    MR_TRY(key.alloc(ctx, (size_t)S));
    MR_TRY(val.alloc(ctx, (size_t)S));
    MR_TRY(head.alloc(ctx, (size_t)S));
    MR_TRY(hpos.alloc(ctx, (size_t)S + 1));
    MR_TRY(tmp.alloc(ctx, (size_t)std::max<int64_t>(scan_tmp_elems(S), 1)));
    MR_TRY(D.cls.alloc(ctx, (size_t)S));
    MR_TRY(bad.alloc(ctx, 2));   // (read back as one 8-byte word)
    static const uint64_t seeds[4] = {0x1b873593c2b2ae35ull, 0x0f3a8c5e27d4b961ull, 0x152e4d7a9b3c6f11ull,
                                      0x0a4c1e9d3f7b2d85ull};
    for (int attempt = 0;; ++attempt) {
        if (attempt == 4) return mr_fail(ctx, MR_ERR_VALUE, "mr_spans_ingest: name hash collisions under every seed");
        const uint64_t x = seeds[attempt];
        MR_TRY_HIP(ctx, hipMemsetAsync(bad.p, 0, 2 * sizeof(int32_t), st));
        hipLaunchKernelGGL(k_row_hash, dim3(cdiv(S, IB)), dim3(IB), 0, st, c, d, S, x, key.p, val.p);
        SortScratch ws;
        MR_TRY(mr_radix_sort(ctx, key.p, val.p, S, 64, ws));
        hipLaunchKernelGGL(k_heads64, dim3(cdiv(S, IB)), dim3(IB), 0, st, key.p, S, head.p);
        MR_TRY(mr_exclusive_scan_i32(ctx, head.p, hpos.p, S, tmp.p));
        // hpos[i + 1] - 1 needs the inclusive form: hpos has n + 1 slots, hpos[n] = runs
        int64_t h[1];
        MR_TRY(mr_read_words(ctx, hpos.p + S, 1, h));
        D.U = h[0];
        MR_TRY(D.rep.alloc(ctx, (size_t)std::max<int64_t>(D.U, 1)));
        if (d == 3) MR_TRY(D.rkey.alloc(ctx, (size_t)std::max<int64_t>(D.U, 1)));
        hipLaunchKernelGGL(k_runs, dim3(cdiv(S, IB)), dim3(IB), 0, st, key.p, val.p, head.p, hpos.p, S, D.cls.p, D.rep.p,
                           d == 3 ? D.rkey.p : nullptr);
        hipLaunchKernelGGL(k_verify, dim3(cdiv(S, IB)), dim3(IB), 0, st, c, d, S, D.cls.p, D.rep.p, bad.p);
        int64_t hb[1];
        MR_TRY(mr_read_words(ctx, (const int64_t*)bad.p, 1, hb));
        if ((int32_t)hb[0] == 0) {
            *x_used = x;
            break;
        }
    }
    if (!sorted) return MR_OK;
    const int64_t U = D.U;
    // longest name among the distinct ones (chunk passes)
    DBuf<uint64_t> k2;
    DBuf<uint32_t> perm;
    MR_TRY(k2.alloc(ctx, (size_t)std::max<int64_t>(U, 1)));
    MR_TRY(perm.alloc(ctx, (size_t)std::max<int64_t>(U, 1)));
    hipLaunchKernelGGL(k_len_key, dim3(cdiv(std::max<int64_t>(U, 1), IB)), dim3(IB), 0, st, c, d, D.rep.p, U, k2.p, perm.p);
    SortScratch ws;
    MR_TRY(mr_radix_sort(ctx, k2.p, perm.p, U, 32, ws));   // by length: the least significant key
    int64_t maxlen = 0;
    if (U) MR_TRY(mr_read_words(ctx, (const int64_t*)(k2.p + U - 1), 1, &maxlen));
    for (int64_t k = (maxlen + 7) / 8 - 1; k >= 0; --k) {   // then chunks, last to first (LSD)
        hipLaunchKernelGGL(k_chunk_key, dim3(cdiv(U, IB)), dim3(IB), 0, st, c, d, D.rep.p, perm.p, U, k, k2.p);
        MR_TRY(mr_radix_sort(ctx, k2.p, perm.p, U, 64, ws));
    }
    MR_TRY(D.code_of_run.alloc(ctx, (size_t)std::max<int64_t>(U, 1)));
    MR_TRY(D.rep_sorted.alloc(ctx, (size_t)std::max<int64_t>(U, 1)));
    if (U)
        hipLaunchKernelGGL(k_rank, dim3(cdiv(U, IB)), dim3(IB), 0, st, perm.p, U, D.rep.p, D.code_of_run.p,
                           D.rep_sorted.p);
    MR_TRY_HIP(ctx, hipGetLastError());
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // scratch is released on return
    return MR_OK;
}

static const char* const COL_NAME[6] = {"traceID", "spanID", "ParentSpanId", "serviceName", "operationName", "podName"};

static int upload_str(mr_ctx* ctx, const mr_str_col& col, int64_t S, const char* name, DBuf<int64_t>& off,
                      DBuf<uint8_t>& bytes) {
    if (!col.offsets) return mr_fail(ctx, MR_ERR_ARG, "mr_spans_ingest: column %s missing", name);
    const int64_t base = col.offsets[0], nb = col.offsets[S] - base;
    if (base < 0 || nb < 0) return mr_fail(ctx, MR_ERR_ARG, "mr_spans_ingest: column %s: bad offsets", name);
    if (nb && !col.bytes) return mr_fail(ctx, MR_ERR_ARG, "mr_spans_ingest: column %s: no bytes", name);
    MR_TRY(bytes.alloc(ctx, (size_t)nb + 16));
    MR_TRY_HIP(ctx, hipMemsetAsync(bytes.p + nb, 0, 16, ctx->stream));
    if (nb) MR_TRY_HIP(ctx, hipMemcpyAsync(bytes.p, col.bytes + base, (size_t)nb, hipMemcpyHostToDevice, ctx->stream));
    if (base == 0) {
        MR_TRY(off.upload(ctx, col.offsets, (size_t)S + 1));
    } else {
        std::vector<int64_t> o((size_t)S + 1);
        for (int64_t i = 0; i <= S; ++i) o[(size_t)i] = col.offsets[i] - base;
        MR_TRY(off.upload(ctx, o.data(), (size_t)S + 1));
        MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));   // o is released on return
    }
    return MR_OK;
}

static int check_strings(mr_ctx* ctx, const mr_span_strings* in, const char* fn) {
    const int64_t S = in->n_spans;
    if (S <= 0 || S >= (1ll << 31)) return mr_fail(ctx, MR_ERR_ARG, "%s: n_spans out of range (1 .. 2^31-1)", fn);
    if (!in->duration) return mr_fail(ctx, MR_ERR_ARG, "%s: duration missing", fn);
    const mr_str_col* sc[6] = {&in->trace_id, &in->span_id, &in->parent_id, &in->service, &in->operation, &in->pod};
    for (int k = 0; k < 6; ++k)
        if (k != C_PARENT && sc[k]->valid)
            return mr_fail(ctx, MR_ERR_ARG, "%s: column %s must have no nulls", fn, COL_NAME[k]);
    for (int k = 0; k < 6; ++k)
        for (int64_t i = 0; i < S; ++i)
            if (sc[k]->offsets && sc[k]->offsets[i + 1] < sc[k]->offsets[i])
                return mr_fail(ctx, MR_ERR_ARG, "%s: column %s: offsets not ascending", fn, COL_NAME[k]);
    return MR_OK;
}

// The dictionaries, code columns and index of a table whose string columns are on the device
// (c: offsets / bytes / validity; op_len is filled here).  s->S, the value columns and the
// times flag are set by the caller.
static int ingest_core(mr_ctx* ctx, Cols c, mr_spans* s) {
    hipStream_t st = ctx->stream;
    const int64_t S = s->S;
    DBuf<int32_t> op_len;
    MR_TRY(op_len.alloc(ctx, (size_t)S));
    c.op_len = op_len.p;
    hipLaunchKernelGGL(k_op_len, dim3(cdiv(S, IB)), dim3(IB), 0, st, c, S, op_len.p);
    s->row_bits = bits_for((uint64_t)std::max<int64_t>(S, 1));
    IngestDict dt, dp, dv, ds;
    uint64_t x = 0, xs = 0;
    MR_TRY(build_dict(ctx, c, 0, S, true, dt, &x));
    MR_TRY(build_dict(ctx, c, 1, S, true, dp, &x));
    MR_TRY(build_dict(ctx, c, 2, S, true, dv, &x));
    MR_TRY(build_dict(ctx, c, 3, S, false, ds, &xs));
    s->n_traces = (int32_t)dt.U;
    s->n_podops = (int32_t)dp.U;
    s->n_svcops = (int32_t)dv.U;
    s->n_span_codes = ds.U;
    MR_TRY(s->trace.alloc(ctx, (size_t)S));
    MR_TRY(s->podop.alloc(ctx, (size_t)S));
    MR_TRY(s->svcop.alloc(ctx, (size_t)S));
    MR_TRY(s->span.alloc(ctx, (size_t)S));
    MR_TRY(s->parent.alloc(ctx, (size_t)S));
    hipLaunchKernelGGL(k_codes<int32_t>, dim3(cdiv(S, IB)), dim3(IB), 0, st, dt.cls.p, dt.code_of_run.p, S, s->trace.p);
    hipLaunchKernelGGL(k_codes<int32_t>, dim3(cdiv(S, IB)), dim3(IB), 0, st, dp.cls.p, dp.code_of_run.p, S, s->podop.p);
    hipLaunchKernelGGL(k_codes<int32_t>, dim3(cdiv(S, IB)), dim3(IB), 0, st, dv.cls.p, dv.code_of_run.p, S, s->svcop.p);
    hipLaunchKernelGGL(k_codes<int64_t>, dim3(cdiv(S, IB)), dim3(IB), 0, st, ds.cls.p, (const int32_t*)nullptr, S,
                       s->span.p);
    hipLaunchKernelGGL(k_parent, dim3(cdiv(S, IB)), dim3(IB), 0, st, c, S, xs, ds.rkey.p, ds.rep.p, ds.U, s->parent.p);
    if (hipGetLastError() != hipSuccess) return mr_fail(ctx, MR_ERR_HIP, "mr_spans_ingest: kernel launch failed");
    // the representative row of every code, for the host's name lists (mr_spans_dict_rows)
    MR_TRY(s->dict_rows[0].alloc(ctx, (size_t)std::max(s->n_traces, 1)));
    MR_TRY(s->dict_rows[1].alloc(ctx, (size_t)std::max(s->n_podops, 1)));
    MR_TRY(s->dict_rows[2].alloc(ctx, (size_t)std::max(s->n_svcops, 1)));
    MR_TRY_HIP(ctx, hipMemcpyAsync(s->dict_rows[0].p, dt.rep_sorted.p, dt.U * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    MR_TRY_HIP(ctx, hipMemcpyAsync(s->dict_rows[1].p, dp.rep_sorted.p, dp.U * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    MR_TRY_HIP(ctx, hipMemcpyAsync(s->dict_rows[2].p, dv.rep_sorted.p, dv.U * sizeof(int32_t), hipMemcpyDeviceToDevice, st));
    return mr_spans_finish(ctx, s);
}

extern "C" int mr_spans_ingest(mr_ctx* ctx, const mr_span_strings* in, mr_spans** out) {
    if (!ctx || !in || !out) return mr_fail(ctx, MR_ERR_ARG, "mr_spans_ingest: null argument");
    *out = nullptr;
    MR_TRY(check_strings(ctx, in, "mr_spans_ingest"));
    const int64_t S = in->n_spans;
    const mr_str_col* sc[6] = {&in->trace_id, &in->span_id, &in->parent_id, &in->service, &in->operation, &in->pod};
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    DBuf<int64_t> off[6];
    DBuf<uint8_t> bytes[6], valid2;
    for (int k = 0; k < 6; ++k) MR_TRY(upload_str(ctx, *sc[k], S, COL_NAME[k], off[k], bytes[k]));
    if (in->parent_id.valid) MR_TRY(valid2.upload(ctx, in->parent_id.valid, (size_t)(S + 7) / 8));
    Cols c;
    for (int k = 0; k < 6; ++k) {
        c.off[k] = off[k].p;
        c.bytes[k] = bytes[k].p;
    }
    c.valid2 = in->parent_id.valid ? valid2.p : nullptr;
    std::unique_ptr<mr_spans> s(new mr_spans());
    s->ctx = ctx;
    s->S = S;
    s->has_times = in->tstart && in->tend;
    MR_TRY(s->duration.upload(ctx, in->duration, (size_t)S));
    if (s->has_times) {
        MR_TRY(s->tstart.upload(ctx, in->tstart, (size_t)S));
        MR_TRY(s->tend.upload(ctx, in->tend, (size_t)S));
    }
    MR_TRY(ingest_core(ctx, c, s.get()));
    mr_handle_add(ctx, s.get(), [](void* h) { delete (mr_spans*)h; });
    *out = s.release();
    return MR_OK;
}

// ---------------------------------------------------------------------------------- streaming
// mr_spans_append: the previous table's rows whose trace-level start is >= keep_from, then the
// chunk's rows, as one new table -- the same table mr_spans_ingest builds from those rows' strings
// in that order.  The kept rows are gathered device to device; only the chunk crosses PCIe.
namespace {
__global__ void k_keep_flag(const int64_t* tstart, int64_t n, int64_t keep_from, int32_t* flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = tstart[i] >= keep_from ? 1 : 0;
}
// from[j] = the source of output row j: a kept row i of the previous table (< Sp) or Sp + b for
// chunk row b
__global__ void k_keep_from(const int32_t* flag, const int64_t* pos, int64_t Sp, int64_t K, int64_t Sc, int64_t* from) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < Sp && flag[i]) from[pos[i]] = i;
    if (i < Sc) from[K + i] = Sp + i;
}
struct StrSrc {
    const int64_t* off[2];    // previous table / chunk
    const uint8_t* bytes[2];
};
__global__ void k_str_len(const int64_t* from, int64_t S, int64_t Sp, StrSrc src, int64_t* len) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= S) return;
    const int64_t f = from[j];
    const int w = f >= Sp;
    const int64_t r = w ? f - Sp : f;
    len[j] = src.off[w][r + 1] - src.off[w][r];
}
// one wave per row, a byte per lane: rows are tens of bytes, so the copy stays coalesced
__global__ void k_str_copy(const int64_t* from, int64_t S, int64_t Sp, StrSrc src, const int64_t* off, uint8_t* out) {
    const int64_t j = (int64_t)blockIdx.x * (blockDim.x / WAVE) + threadIdx.x / WAVE;
    const int lane = threadIdx.x & (WAVE - 1);
    if (j >= S) return;
    const int64_t f = from[j];
    const int w = f >= Sp;
    const int64_t r = w ? f - Sp : f;
    const int64_t b0 = src.off[w][r], n = src.off[w][r + 1] - b0, o = off[j];
    for (int64_t k = lane; k < n; k += WAVE) out[o + k] = src.bytes[w][b0 + k];
}
// ParentSpanId validity, 8 rows per output byte (a source without a bitmap: all valid)
__global__ void k_valid_pack(const int64_t* from, int64_t S, int64_t Sp, const uint8_t* vp, const uint8_t* vc,
                             uint8_t* out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q * 8 >= S) return;
    unsigned v = 0;
    for (int b = 0; b < 8 && q * 8 + b < S; ++b) {
        const int64_t f = from[q * 8 + b];
        const uint8_t* m = f >= Sp ? vc : vp;
        const int64_t r = f >= Sp ? f - Sp : f;
        if (!m || ((m[r >> 3] >> (r & 7)) & 1u)) v |= 1u << b;
    }
    out[q] = (uint8_t)v;
}
// value columns: previous table's value, or the chunk's (chunk == null: src_base + chunk row)
__global__ void k_gather_i64(const int64_t* from, int64_t S, int64_t Sp, const int64_t* prev, const int64_t* chunk,
                             int64_t src_base, int64_t* out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= S) return;
    const int64_t f = from[j];
    out[j] = f < Sp ? prev[f] : chunk ? chunk[f - Sp] : src_base + (f - Sp);
}
__global__ void k_dict_src(const int32_t* rows, int64_t n, const int64_t* src, int64_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = src[rows[i]];
}
}  // namespace

extern "C" int mr_spans_append(mr_ctx* ctx, const mr_spans* prev, int64_t keep_from, const mr_span_strings* in,
                               mr_spans** out) {
    if (!ctx || !in || !out) return mr_fail(ctx, MR_ERR_ARG, "mr_spans_append: null argument");
    *out = nullptr;
    if (prev && (prev->ctx != ctx || !prev->raw))
        return mr_fail(ctx, MR_ERR_STATE, "mr_spans_append: the previous table was not built by mr_spans_append on this context");
    MR_TRY(check_strings(ctx, in, "mr_spans_append"));
    if (!in->tstart || !in->tend) return mr_fail(ctx, MR_ERR_ARG, "mr_spans_append: trace start / end times missing");
    const int64_t Sc = in->n_spans, Sp = prev ? prev->S : 0;
    const mr_str_col* sc[6] = {&in->trace_id, &in->span_id, &in->parent_id, &in->service, &in->operation, &in->pod};
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    // the chunk: one upload
    DBuf<int64_t> off[6], cdur, cts, cte;
    DBuf<uint8_t> bytes[6], cvalid;
    for (int k = 0; k < 6; ++k) MR_TRY(upload_str(ctx, *sc[k], Sc, COL_NAME[k], off[k], bytes[k]));
    if (in->parent_id.valid) MR_TRY(cvalid.upload(ctx, in->parent_id.valid, (size_t)(Sc + 7) / 8));
    MR_TRY(cdur.upload(ctx, in->duration, (size_t)Sc));
    MR_TRY(cts.upload(ctx, in->tstart, (size_t)Sc));
    MR_TRY(cte.upload(ctx, in->tend, (size_t)Sc));
    // the kept rows of the previous table
    int64_t K = 0;
    DBuf<int32_t> flag;
    DBuf<int64_t> pos, tmp;
    MR_TRY(tmp.alloc(ctx, (size_t)std::max<int64_t>(scan_tmp_elems(Sp + Sc), 1)));   // covers both scans
    if (Sp) {
        MR_TRY(flag.alloc(ctx, (size_t)Sp));
        MR_TRY(pos.alloc(ctx, (size_t)Sp + 1));
        hipLaunchKernelGGL(k_keep_flag, dim3(cdiv(Sp, IB)), dim3(IB), 0, st, prev->tstart.p, Sp, keep_from, flag.p);
        MR_TRY(mr_exclusive_scan_i32(ctx, flag.p, pos.p, Sp, tmp.p));
        MR_TRY(mr_read_words(ctx, pos.p + Sp, 1, &K));
    }
    const int64_t S = K + Sc;
    if (S >= (1ll << 31)) return mr_fail(ctx, MR_ERR_ARG, "mr_spans_append: table would exceed 2^31-1 spans");
    DBuf<int64_t> from;
    MR_TRY(from.alloc(ctx, (size_t)S));
    hipLaunchKernelGGL(k_keep_from, dim3(cdiv(std::max(Sp, Sc), IB)), dim3(IB), 0, st, flag.p, pos.p, Sp, K, Sc, from.p);
    std::unique_ptr<mr_spans> s(new mr_spans());
    s->ctx = ctx;
    s->S = S;
    s->has_times = true;
    s->raw = true;
    // string columns: lengths -> offsets -> bytes
    DBuf<int64_t> len;
    MR_TRY(len.alloc(ctx, (size_t)S));
    Cols c;
    for (int k = 0; k < 6; ++k) {
        StrSrc src;
        src.off[0] = prev ? prev->raw_off[k].p : nullptr;
        src.bytes[0] = prev ? prev->raw_bytes[k].p : nullptr;
        src.off[1] = off[k].p;
        src.bytes[1] = bytes[k].p;
        MR_TRY(s->raw_off[k].alloc(ctx, (size_t)S + 1));
        hipLaunchKernelGGL(k_str_len, dim3(cdiv(S, IB)), dim3(IB), 0, st, from.p, S, Sp, src, len.p);
        MR_TRY(mr_exclusive_scan(ctx, len.p, s->raw_off[k].p, S, tmp.p));
        int64_t nb = 0;
        MR_TRY(mr_read_words(ctx, s->raw_off[k].p + S, 1, &nb));
        MR_TRY(s->raw_bytes[k].alloc(ctx, (size_t)nb + 16));
        MR_TRY_HIP(ctx, hipMemsetAsync(s->raw_bytes[k].p + nb, 0, 16, st));
        hipLaunchKernelGGL(k_str_copy, dim3(cdiv(S, IB / WAVE)), dim3(IB), 0, st, from.p, S, Sp, src,
                           s->raw_off[k].p, s->raw_bytes[k].p);
        c.off[k] = s->raw_off[k].p;
        c.bytes[k] = s->raw_bytes[k].p;
    }
    const uint8_t* pv = prev && prev->raw_valid.p ? prev->raw_valid.p : nullptr;
    c.valid2 = nullptr;
    if (pv || cvalid.p) {
        MR_TRY(s->raw_valid.alloc(ctx, (size_t)(S + 7) / 8));
        hipLaunchKernelGGL(k_valid_pack, dim3(cdiv((S + 7) / 8, IB)), dim3(IB), 0, st, from.p, S, Sp, pv, cvalid.p,
                           s->raw_valid.p);
        c.valid2 = s->raw_valid.p;
    }
    // value columns and the stream row numbers
    const int64_t src_base = prev ? prev->src_next : 0;
    MR_TRY(s->duration.alloc(ctx, (size_t)S));
    MR_TRY(s->tstart.alloc(ctx, (size_t)S));
    MR_TRY(s->tend.alloc(ctx, (size_t)S));
    MR_TRY(s->src.alloc(ctx, (size_t)S));
    hipLaunchKernelGGL(k_gather_i64, dim3(cdiv(S, IB)), dim3(IB), 0, st, from.p, S, Sp, prev ? prev->duration.p : nullptr,
                       cdur.p, 0, s->duration.p);
    hipLaunchKernelGGL(k_gather_i64, dim3(cdiv(S, IB)), dim3(IB), 0, st, from.p, S, Sp, prev ? prev->tstart.p : nullptr,
                       cts.p, 0, s->tstart.p);
    hipLaunchKernelGGL(k_gather_i64, dim3(cdiv(S, IB)), dim3(IB), 0, st, from.p, S, Sp, prev ? prev->tend.p : nullptr,
                       cte.p, 0, s->tend.p);
    hipLaunchKernelGGL(k_gather_i64, dim3(cdiv(S, IB)), dim3(IB), 0, st, from.p, S, Sp, prev ? prev->src.p : nullptr,
                       (const int64_t*)nullptr, src_base, s->src.p);
    MR_TRY_HIP(ctx, hipGetLastError());
    s->src_next = src_base + Sc;
    MR_TRY(ingest_core(ctx, c, s.get()));
    MR_TRY_HIP(ctx, hipStreamSynchronize(st));   // the chunk's staging buffers are released on return
    mr_handle_add(ctx, s.get(), [](void* h) { delete (mr_spans*)h; });
    *out = s.release();
    return MR_OK;
}

extern "C" int mr_spans_dict_sources(const mr_spans* s, int which, int64_t* src) {
    if (!s || which < 0 || which > 2 || !src) return MR_ERR_ARG;
    mr_ctx* ctx = s->ctx;
    if (!s->raw) return mr_fail(ctx, MR_ERR_STATE, "mr_spans_dict_sources: table was not built by mr_spans_append");
    const int64_t n = which == 0 ? s->n_traces : which == 1 ? s->n_podops : s->n_svcops;
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    DBuf<int64_t> out;
    MR_TRY(out.alloc(ctx, (size_t)std::max<int64_t>(n, 1)));
    if (n) hipLaunchKernelGGL(k_dict_src, dim3(cdiv(n, IB)), dim3(IB), 0, ctx->stream, s->dict_rows[which].p, n, s->src.p, out.p);
    MR_TRY_HIP(ctx, hipGetLastError());
    MR_TRY(out.download(ctx, src, (size_t)n));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return MR_OK;
}

extern "C" int mr_spans_info(const mr_spans* s, int64_t* n_spans, int32_t* n_traces, int32_t* n_podops,
                             int32_t* n_svcops) {
    if (!s) return MR_ERR_ARG;
    if (n_spans) *n_spans = s->S;
    if (n_traces) *n_traces = s->n_traces;
    if (n_podops) *n_podops = s->n_podops;
    if (n_svcops) *n_svcops = s->n_svcops;
    return MR_OK;
}

extern "C" int mr_spans_dict_rows(const mr_spans* s, int which, int32_t* rows) {
    if (!s || which < 0 || which > 2 || !rows) return MR_ERR_ARG;
    mr_ctx* ctx = s->ctx;
    const int64_t n = which == 0 ? s->n_traces : which == 1 ? s->n_podops : s->n_svcops;
    if (!s->dict_rows[which].p) return mr_fail(ctx, MR_ERR_STATE, "mr_spans_dict_rows: table was not ingested from strings");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    MR_TRY(s->dict_rows[which].download(ctx, rows, (size_t)n));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return MR_OK;
}

extern "C" int mr_spans_codes(const mr_spans* s, int32_t* trace, int32_t* podop, int32_t* svcop, int64_t* span,
                              int64_t* parent) {
    if (!s) return MR_ERR_ARG;
    mr_ctx* ctx = s->ctx;
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    const size_t S = (size_t)s->S;
    if (trace) MR_TRY(s->trace.download(ctx, trace, S));
    if (podop) MR_TRY(s->podop.download(ctx, podop, S));
    if (svcop) MR_TRY(s->svcop.download(ctx, svcop, S));
    if (span) MR_TRY(s->span.download(ctx, span, S));
    if (parent) MR_TRY(s->parent.download(ctx, parent, S));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return MR_OK;
}
