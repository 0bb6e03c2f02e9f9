// Context, error reporting, graph upload from host index arrays, result fetch.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

#include "mr_internal.h"
#include "mr_prim.h"

int mr_fail(mr_ctx* ctx, int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (ctx) ctx->err = buf;
    return code;
}

PhaseTimer::PhaseTimer(hipStream_t s, const char* t) : st(s), tag(t), on(getenv("MR_WIN_TIMING") != nullptr) {
    mark("start");
}
void PhaseTimer::mark(const char* name) {
    if (!on) return;
    (void)hipStreamSynchronize(st);
    marks.emplace_back(name, std::chrono::duration<double, std::micro>(
                                 std::chrono::steady_clock::now().time_since_epoch()).count());
}
PhaseTimer::~PhaseTimer() {
    if (!on || marks.size() < 2) return;
    fprintf(stderr, "[%s]", tag);
    for (size_t i = 1; i < marks.size(); ++i) fprintf(stderr, " %s %.1f", marks[i].first, marks[i].second - marks[i - 1].second);
    fprintf(stderr, " us\n");
}

extern "C" int mr_version(void) { return 100; }

extern "C" int mr_device_count(int* n) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    if (n) *n = c;
    return MR_OK;
}

extern "C" int mr_ctx_create(int device, uint32_t flags, mr_ctx** out) {
    if (!out) return MR_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MR_ERR_HIP;
    if (device < 0 || device >= n) return MR_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return MR_ERR_HIP;
    auto* c = new mr_ctx();
    c->device = device;
    c->flags = flags;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return MR_ERR_HIP;
    }
    *out = c;
    return MR_OK;
}

void mr_comm_destroy(mr_ctx* ctx);  // mr_comm.hip

void mr_graph_delete(mr_graph* g) { delete g; }

// ------------------------------------------------------------------------------ pool
static size_t pool_round(size_t b) {
    if (b <= 4096) return (b + 255) & ~(size_t)255;
    if (b <= (1u << 20)) return (b + 4095) & ~(size_t)4095;
    return (b + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
}

// Give cached device memory back to the driver after an allocation failed: this context's free
// blocks, the window graphs it holds for release by its next mr_windows_batch call, and its
// auxiliary contexts' free blocks (each stream synchronised first: a free block may still be read
// by work queued before it was freed).  Called without the context's pool lock held.
static void pool_trim(mr_ctx* ctx) {
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->side) (void)hipStreamSynchronize(ctx->side);
    for (mr_ctx* a : ctx->aux) (void)hipStreamSynchronize(a->stream);
    std::vector<struct mr_graph*> dead;
    dead.swap(ctx->graveyard);
    for (struct mr_graph* g : dead) mr_graph_delete(g);   // (their blocks return to the aux pools)
    auto drain = [](mr_ctx* c) {
        std::lock_guard<std::mutex> lk(c->pool_mu);
        for (auto& kv : c->pool_free)
            for (void* q : kv.second) {
                (void)hipFree(q);
                c->pool_all.erase(q);
                c->pool_bytes -= kv.first;
            }
        c->pool_free.clear();
    };
    for (mr_ctx* a : ctx->aux) drain(a);
    drain(ctx);
}

void* mr_pool_alloc(mr_ctx* ctx, size_t bytes, size_t* cls) {
    const size_t want = pool_round(bytes);
    std::unique_lock<std::mutex> lk(ctx->pool_mu);
    auto it = ctx->pool_free.lower_bound(want);
    if (it != ctx->pool_free.end() && it->first <= 2 * want) {   // reuse a block at most 2x too big
        void* p = it->second.back();   // (a class is erased when it empties: never empty here)
        *cls = it->first;
        it->second.pop_back();
        if (it->second.empty()) ctx->pool_free.erase(it);
        return p;
    }
    void* p = nullptr;
    if (hipMalloc(&p, want) != hipSuccess) {
        (void)hipGetLastError();
        lk.unlock();   // give the cached blocks back and retry once
        pool_trim(ctx);
        lk.lock();
        if (hipMalloc(&p, want) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
    }
    ctx->pool_bytes += want;
    ctx->pool_all[p] = want;
    *cls = want;
    return p;
}

void mr_pool_free(mr_ctx* ctx, void* p, size_t cls) {
    if (!ctx || !p) return;
    std::lock_guard<std::mutex> lk(ctx->pool_mu);
    ctx->pool_free[cls].push_back(p);   // stream-ordered reuse: no sync needed
}

int mr_read_bytes(mr_ctx* ctx, const void* dev, size_t bytes, unsigned char** host) {
    if (bytes > MR_PIN_BYTES) return mr_fail(ctx, MR_ERR_ARG, "mr_read_bytes: %zu bytes", bytes);
    if (!ctx->pin) MR_TRY_HIP(ctx, hipHostMalloc((void**)&ctx->pin, MR_PIN_BYTES, hipHostMallocDefault));
    if (bytes) MR_TRY_HIP(ctx, hipMemcpyAsync(ctx->pin, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *host = (unsigned char*)ctx->pin;
    return MR_OK;
}
int mr_read_words(mr_ctx* ctx, const int64_t* dev, int n, int64_t* out) {
    if (n <= 0) return MR_OK;
    if (n > 64) return mr_fail(ctx, MR_ERR_ARG, "mr_read_words: %d words", n);
    unsigned char* h = nullptr;
    MR_TRY(mr_read_bytes(ctx, dev, (size_t)n * sizeof(int64_t), &h));
    memcpy(out, h, (size_t)n * sizeof(int64_t));
    return MR_OK;
}

void mr_pool_release(mr_ctx* ctx) {
    (void)hipStreamSynchronize(ctx->stream);
    std::lock_guard<std::mutex> lk(ctx->pool_mu);
    for (auto& kv : ctx->pool_free)
        for (void* q : kv.second) {
            (void)hipFree(q);
            ctx->pool_all.erase(q);
            ctx->pool_bytes -= kv.first;
        }
    ctx->pool_free.clear();
}

static void prof_clear(mr_ctx* ctx) {
    for (hipEvent_t e : ctx->prof_ev) (void)hipEventDestroy(e);
    ctx->prof_ev.clear();
    ctx->prof_bytes.clear();
    ctx->prof_iters.clear();
}

extern "C" int mr_ctx_profile(mr_ctx* ctx, int enable) {
    if (!ctx) return MR_ERR_ARG;
    (void)hipStreamSynchronize(ctx->stream);
    prof_clear(ctx);
    ctx->prof = enable != 0;
    return MR_OK;
}

extern "C" int mr_ctx_prof_read(mr_ctx* ctx, int64_t* launches, double* total_ms, double* total_bytes) {
    if (!ctx) return MR_ERR_ARG;
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    double ms = 0.0, by = 0.0;
    for (size_t i = 0; i + 1 < ctx->prof_ev.size(); i += 2) {
        float t = 0.0f;
        MR_TRY_HIP(ctx, hipEventElapsedTime(&t, ctx->prof_ev[i], ctx->prof_ev[i + 1]));
        ms += t;
        by += ctx->prof_bytes[i / 2];
    }
    int64_t its = 0;   // iterations covered
    for (size_t i = 0; i < ctx->prof_bytes.size(); ++i) its += i < ctx->prof_iters.size() ? ctx->prof_iters[i] : 1;
    if (launches) *launches = its;
    if (total_ms) *total_ms = ms;
    if (total_bytes) *total_bytes = by;
    prof_clear(ctx);
    return MR_OK;
}

// bracket a launch with events when profiling (called by the power iteration)
void mr_prof_begin(mr_ctx* ctx) {
    if (!ctx->prof) return;
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return;
    (void)hipEventRecord(e, ctx->stream);
    ctx->prof_ev.push_back(e);
}
void mr_prof_end(mr_ctx* ctx, double bytes, int64_t iters) {
    if (!ctx->prof) return;
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return;
    (void)hipEventRecord(e, ctx->stream);
    ctx->prof_ev.push_back(e);
    ctx->prof_bytes.push_back(bytes);
    ctx->prof_iters.push_back(iters);
}

static std::mutex g_handles_mu;
static std::map<void*, std::pair<mr_ctx*, void (*)(void*)>> g_handles;
void mr_handle_add(mr_ctx* ctx, void* h, void (*del)(void*)) {
    std::lock_guard<std::mutex> lk(g_handles_mu);
    g_handles[h] = {ctx, del};
}
bool mr_handle_take(void* h) {
    std::lock_guard<std::mutex> lk(g_handles_mu);
    return g_handles.erase(h) > 0;
}

extern "C" void mr_ctx_destroy(mr_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    if (ctx->side) (void)hipStreamSynchronize(ctx->side);
    for (mr_graph* g : ctx->graveyard) mr_graph_delete(g);   // (their blocks belong to the auxiliary contexts too)
    ctx->graveyard.clear();
    for (mr_ctx* a : ctx->aux) mr_ctx_destroy(a);
    ctx->aux.clear();
    {   // the context's live handles go first (their buffers return to its pool)
        std::vector<std::pair<void*, void (*)(void*)>> mine;
        {
            std::lock_guard<std::mutex> lk(g_handles_mu);
            for (auto it = g_handles.begin(); it != g_handles.end();) {
                if (it->second.first == ctx) {
                    mine.emplace_back(it->first, it->second.second);
                    it = g_handles.erase(it);
                } else {
                    ++it;
                }
            }
        }
        for (auto& m : mine) m.second(m.first);
    }
    mr_comm_peer_destroy(ctx);
    mr_comm_destroy(ctx);
    prof_clear(ctx);
    mr_pool_release(ctx);
    for (auto& kv : ctx->pool_all) (void)hipFree(kv.first);   // blocks of handles the caller leaked
    ctx->pool_all.clear();
    for (hipEvent_t& e : ctx->side_ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->side) (void)hipStreamDestroy(ctx->side);
    if (ctx->pin) (void)hipHostFree(ctx->pin);
    if (ctx->pin_flags) (void)hipHostFree(ctx->pin_flags);
    if (ctx->scan_st) (void)hipFree(ctx->scan_st);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

extern "C" const char* mr_last_error(const mr_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

// ---------------------------------------------------------------- measured copy peak
// STREAM copy, 16 B per lane per access, in two shapes: grid-stride (every lane moves 4 x 16 B
// per round, all loads in flight before the stores) and block tiles (a block copies U x 4 KB of
// consecutive lines once, every load in flight before the stores: the float4-copy shape of
// MI355X_MICROARCH.md's 6.29 TB/s row).  NT: non-temporal loads and stores (no L2 allocation).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ u32x4 cp_ld(const u32x4* p) { return NT ? __builtin_nontemporal_load(p) : *p; }
template <bool NT>
__device__ __forceinline__ void cp_st(u32x4* p, u32x4 v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}
template <bool NT>
__global__ void __launch_bounds__(256) k_copy16(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        const u32x4 a = cp_ld<NT>(src + i), b = cp_ld<NT>(src + i + stride), c = cp_ld<NT>(src + i + 2 * stride),
                    d = cp_ld<NT>(src + i + 3 * stride);
        cp_st<NT>(dst + i, a);
        cp_st<NT>(dst + i + stride, b);
        cp_st<NT>(dst + i + 2 * stride, c);
        cp_st<NT>(dst + i + 3 * stride, d);
    }
    for (; i < n; i += stride) cp_st<NT>(dst + i, cp_ld<NT>(src + i));
}
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_copy_tile(const u32x4* __restrict__ src, u32x4* __restrict__ dst, int64_t n) {
    const int64_t base = (int64_t)blockIdx.x * (256 * U) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t k = base + (int64_t)u * 256;
        v[u] = cp_ld<NT>(src + (k < n ? k : n - 1));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int64_t k = base + (int64_t)u * 256;
        if (k < n) cp_st<NT>(dst + k, v[u]);
    }
}
// The best rate of `reps` timed launches of each shape (after one untimed warm-up launch of each):
// bytes read + written / launch time.
extern "C" int mr_copy_peak(mr_ctx* ctx, int64_t bytes, int reps, double* gbs) {
    if (!ctx || bytes < 16 || reps < 1 || !gbs) return mr_fail(ctx, MR_ERR_ARG, "mr_copy_peak: bad arguments");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    const int64_t n = bytes / 16;
    DBuf<u32x4> a, b;
    MR_TRY(a.alloc(ctx, (size_t)n));
    MR_TRY(b.alloc(ctx, (size_t)n));
    MR_TRY_HIP(ctx, hipMemsetAsync(a.p, 1, (size_t)n * 16, ctx->stream));
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const unsigned gs_blocks = (unsigned)std::min<int64_t>((int64_t)cus * 16, (n + 255) / 256);
    auto launch = [&](int shape) {
        hipStream_t st = ctx->stream;
        switch (shape) {
            case 0: hipLaunchKernelGGL(k_copy16<false>, dim3(gs_blocks), dim3(256), 0, st, a.p, b.p, n); break;
            case 1: hipLaunchKernelGGL(k_copy16<true>, dim3(gs_blocks), dim3(256), 0, st, a.p, b.p, n); break;
            case 2: hipLaunchKernelGGL((k_copy_tile<4, false>), dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, st, a.p, b.p, n); break;
            case 3: hipLaunchKernelGGL((k_copy_tile<4, true>), dim3((unsigned)((n + 1023) / 1024)), dim3(256), 0, st, a.p, b.p, n); break;
            case 4: hipLaunchKernelGGL((k_copy_tile<8, false>), dim3((unsigned)((n + 2047) / 2048)), dim3(256), 0, st, a.p, b.p, n); break;
            default: hipLaunchKernelGGL((k_copy_tile<1, false>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a.p, b.p, n); break;
        }
    };
    hipEvent_t e0 = nullptr, e1 = nullptr;
    MR_TRY_HIP(ctx, hipEventCreate(&e0));
    if (hipEventCreate(&e1) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipEventDestroy(e0);
        return mr_fail(ctx, MR_ERR_HIP, "mr_copy_peak: hipEventCreate failed");
    }
    double best = 0.0;
    int rc = MR_OK;
    for (int shape = 0; shape < 6 && rc == MR_OK; ++shape)
        for (int r = -1; r < reps && rc == MR_OK; ++r) {   // r = -1: the shape's warm-up launch
            (void)hipEventRecord(e0, ctx->stream);
            launch(shape);
            (void)hipEventRecord(e1, ctx->stream);
            if (hipEventSynchronize(e1) != hipSuccess || hipGetLastError() != hipSuccess)
                rc = mr_fail(ctx, MR_ERR_HIP, "mr_copy_peak: launch failed");
            float ms = 0.0f;
            if (rc == MR_OK && r >= 0 && hipEventElapsedTime(&ms, e0, e1) == hipSuccess && ms > 0.0f)
                best = std::max(best, 2.0 * (double)n * 16.0 / (ms * 1e-3) / 1e9);
        }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    MR_TRY(rc);
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    *gbs = best;
    return MR_OK;
}

extern "C" int mr_ctx_sync(mr_ctx* ctx) {
    if (!ctx) return MR_ERR_ARG;
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return MR_OK;
}

extern "C" void* mr_ctx_stream(mr_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

// ------------------------------------------------------------------------------ upload
extern "C" int mr_graph_upload(mr_ctx* ctx, const mr_graph_desc* d, mr_graph** out) {
    if (!ctx || !d || !out) return mr_fail(ctx, MR_ERR_ARG, "mr_graph_upload: null argument");
    *out = nullptr;
    const int32_t N = d->n_nodes, T = d->n_traces;
    if (N < 0 || T < 0) return mr_fail(ctx, MR_ERR_ARG, "negative sizes");
    if (!d->sr_off || (d->nnz_sr && !d->sr_ops) || !d->len_t || !d->len_o || !d->ss_off || !d->nchild)
        return mr_fail(ctx, MR_ERR_ARG, "mr_graph_upload: missing array");
    if (d->sr_off[0] != 0 || d->sr_off[T] != d->nnz_sr)
        return mr_fail(ctx, MR_ERR_ARG, "sr_off inconsistent with nnz_sr");
    for (int64_t e = 0; e < d->nnz_sr; ++e)
        if (d->sr_ops[e] < 0 || d->sr_ops[e] >= N) return mr_fail(ctx, MR_ERR_ARG, "sr_ops out of range");
    if (d->ss_off[0] != 0 || d->ss_off[N] != d->n_edges)
        return mr_fail(ctx, MR_ERR_ARG, "ss_off inconsistent with n_edges");
    for (int64_t e = 0; e < d->n_edges; ++e)
        if (d->ss_par[e] < 0 || d->ss_par[e] >= N) return mr_fail(ctx, MR_ERR_ARG, "ss_par out of range");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    auto* g = new mr_graph();
    g->ctx = ctx;
    g->N = N;
    g->T = T;
    g->nnz_sr = d->nnz_sr;
    g->E = d->n_edges;
    g->rs_is_sr = d->rs_off == nullptr;
    g->nnz_rs = g->rs_is_sr ? d->nnz_sr : d->nnz_rs;
    for (int32_t t = 0; t < T && g->traces_nonempty; ++t) g->traces_nonempty = d->sr_off[t + 1] > d->sr_off[t];
    int rc = MR_OK;
    auto fail = [&](int code) {
        delete g;
        return code;
    };
    // the op-major side (tiles of P_sr) is derived on the device by mr_graph_prepare
    if ((rc = g->len_t.upload(ctx, d->len_t, (size_t)T)) || (rc = g->len_o.upload(ctx, d->len_o, (size_t)N)) ||
        (rc = g->ss_off.upload(ctx, d->ss_off, (size_t)N + 1)) ||
        (rc = g->ss_par.upload(ctx, d->ss_par, (size_t)d->n_edges)) ||
        (rc = g->nchild.upload(ctx, d->nchild, (size_t)N)))
        return fail(rc);
    if (g->rs_is_sr) {
        if ((rc = g->rs_off.upload(ctx, d->sr_off, (size_t)T + 1)) ||
            (rc = g->rs_ops.upload(ctx, d->sr_ops, (size_t)d->nnz_sr)))
            return fail(rc);
    } else {
        if (!d->rs_ops || d->rs_off[0] != 0 || d->rs_off[T] != d->nnz_rs) return fail(mr_fail(ctx, MR_ERR_ARG, "rs arrays"));
        for (int64_t e = 0; e < d->nnz_rs; ++e)
            if (d->rs_ops[e] < 0 || d->rs_ops[e] >= N) return fail(mr_fail(ctx, MR_ERR_ARG, "rs_ops out of range"));
        if ((rc = g->rs_off.upload(ctx, d->rs_off, (size_t)T + 1)) ||
            (rc = g->rs_ops.upload(ctx, d->rs_ops, (size_t)d->nnz_rs)) ||
            (rc = g->srt_off.upload(ctx, d->sr_off, (size_t)T + 1)) ||
            (rc = g->srt_ops.upload(ctx, d->sr_ops, (size_t)d->nnz_sr)))
            return fail(rc);
    }
    // pr_trace: identity when it is operation_trace itself (graph-builder output)
    g->n_pr = d->n_pr;
    bool ident = d->pr_trace == nullptr;
    if (!ident && d->n_pr == T) {
        ident = true;
        for (int32_t i = 0; i < T && ident; ++i) ident = d->pr_trace[i] == i && d->pr_len[i] == d->len_t[i];
    }
    g->pr_identity = ident;
    if (!ident) {
        for (int32_t i = 0; i < d->n_pr; ++i)
            if (d->pr_trace[i] < 0 || d->pr_trace[i] >= T) return fail(mr_fail(ctx, MR_ERR_ARG, "pr_trace out of range"));
        if ((rc = g->pr_trace.upload(ctx, d->pr_trace, (size_t)d->n_pr)) ||
            (rc = g->pr_len.upload(ctx, d->pr_len, (size_t)d->n_pr)))
            return fail(rc);
    } else {
        g->n_pr = T;
    }
    if ((rc = mr_graph_prepare(ctx, g))) return fail(rc);
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));  // host vectors go out of scope
    mr_handle_add(ctx, g, [](void* h) { delete (mr_graph*)h; });
    *out = g;
    return MR_OK;
}

extern "C" int mr_graph_free(mr_graph* g) {
    if (!g || !mr_handle_take(g)) return MR_OK;   // (freed with its context)
    (void)hipSetDevice(g->ctx->device);
    (void)hipStreamSynchronize(g->ctx->stream);
    delete g;
    return MR_OK;
}

extern "C" int mr_graph_info(const mr_graph* g, int32_t* n, int32_t* t, int64_t* nnz, int64_t* e) {
    if (!g) return MR_ERR_ARG;
    if (n) *n = g->N;
    if (t) *t = g->T;
    if (nnz) *nnz = g->nnz_sr;
    if (e) *e = g->E;
    return MR_OK;
}

extern "C" int mr_graph_fetch(mr_graph* g, double* weight, int32_t* cov, double* kind, float* pref) {
    if (!g) return MR_ERR_ARG;
    mr_ctx* ctx = g->ctx;
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    if (weight) {
        if (!g->weight.p) return mr_fail(ctx, MR_ERR_STATE, "mr_graph_fetch: mr_pagerank has not run");
        MR_TRY(g->weight.download(ctx, weight, (size_t)g->N));
    }
    if (cov) MR_TRY(g->cov.download(ctx, cov, (size_t)g->N));
    if (kind && g->kind.p) MR_TRY(g->kind.download(ctx, kind, (size_t)g->T));
    if (pref && g->pref.p) MR_TRY(g->pref.download(ctx, pref, (size_t)g->T));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return MR_OK;
}
