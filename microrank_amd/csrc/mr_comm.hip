// Collectives of the trace-sharded PageRank (mr_shard.hip): RCCL over xGMI, one process per GPU
// (librccl is dlopen'ed on first use so the library loads on machines without it), or a
// host-staged callback (ranks that share a GPU, CPU transports such as gloo in the tests).
#include <dlfcn.h>
#include <cstring>
#include <vector>
#include <rccl/rccl.h>

#include "mr_internal.h"

namespace {
struct RcclApi {
    void* h = nullptr;
    ncclResult_t (*getUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*commInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*allReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*allGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
    const char* (*getErrorString)(ncclResult_t) = nullptr;
    bool ok = false;
};

RcclApi& api() {
    static RcclApi a;
    static bool tried = false;
    if (tried) return a;
    tried = true;
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names) {
        a.h = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
        if (a.h) break;
    }
    if (!a.h) return a;
    a.getUniqueId = (decltype(a.getUniqueId))dlsym(a.h, "ncclGetUniqueId");
    a.commInitRank = (decltype(a.commInitRank))dlsym(a.h, "ncclCommInitRank");
    a.allReduce = (decltype(a.allReduce))dlsym(a.h, "ncclAllReduce");
    a.allGather = (decltype(a.allGather))dlsym(a.h, "ncclAllGather");
    a.commDestroy = (decltype(a.commDestroy))dlsym(a.h, "ncclCommDestroy");
    a.getErrorString = (decltype(a.getErrorString))dlsym(a.h, "ncclGetErrorString");
    a.ok = a.getUniqueId && a.commInitRank && a.allReduce && a.allGather && a.commDestroy;
    return a;
}
}  // namespace

void mr_comm_destroy(mr_ctx* ctx) {
    if (ctx && ctx->comm && api().ok) api().commDestroy((ncclComm_t)ctx->comm);
    if (ctx) ctx->comm = nullptr;
}

extern "C" int mr_comm_unique_id(uint8_t id[128]) {
    RcclApi& a = api();
    if (!a.ok) return MR_ERR_COMM;
    ncclUniqueId u;
    if (a.getUniqueId(&u) != ncclSuccess) return MR_ERR_COMM;
    static_assert(sizeof(u) == 128, "ncclUniqueId size");
    memcpy(id, &u, 128);
    return MR_OK;
}

extern "C" int mr_comm_init(mr_ctx* ctx, int nranks, int rank, const uint8_t id[128]) {
    if (!ctx) return MR_ERR_ARG;
    RcclApi& a = api();
    if (!a.ok) return mr_fail(ctx, MR_ERR_COMM, "librccl not loadable");
    MR_TRY_HIP(ctx, hipSetDevice(ctx->device));
    ncclUniqueId u;
    memcpy(&u, id, 128);
    ncclComm_t c = nullptr;
    ncclResult_t r = a.commInitRank(&c, nranks, u, rank);
    if (r != ncclSuccess) return mr_fail(ctx, MR_ERR_COMM, "ncclCommInitRank: %s", a.getErrorString ? a.getErrorString(r) : "?");
    mr_comm_destroy(ctx);
    ctx->comm = c;
    ctx->rank = rank;
    ctx->nranks = nranks;
    return MR_OK;
}

int mr_comm_allreduce(mr_ctx* ctx, const void* send, void* recv, size_t n, ncclDataType_t ty, ncclRedOp_t op) {
    RcclApi& a = api();
    if (!ctx->comm || !a.ok) return mr_fail(ctx, MR_ERR_COMM, "communicator not initialised");
    ncclResult_t r = a.allReduce(send, recv, n, ty, op, (ncclComm_t)ctx->comm, ctx->stream);
    if (r != ncclSuccess) return mr_fail(ctx, MR_ERR_COMM, "ncclAllReduce: %s", a.getErrorString ? a.getErrorString(r) : "?");
    return MR_OK;
}

int mr_comm_allgather(mr_ctx* ctx, const void* send, void* recv, size_t n, ncclDataType_t ty) {
    RcclApi& a = api();
    if (!ctx->comm || !a.ok) return mr_fail(ctx, MR_ERR_COMM, "communicator not initialised");
    ncclResult_t r = a.allGather(send, recv, n, ty, (ncclComm_t)ctx->comm, ctx->stream);
    if (r != ncclSuccess) return mr_fail(ctx, MR_ERR_COMM, "ncclAllGather: %s", a.getErrorString ? a.getErrorString(r) : "?");
    return MR_OK;
}

extern "C" int mr_comm_allreduce_f64(mr_ctx* ctx, double* buf, int64_t n, int op) {
    if (!ctx || !buf || n < 0) return MR_ERR_ARG;
    return mr_comm_allreduce(ctx, buf, buf, (size_t)n, ncclFloat64, op ? ncclMax : ncclSum);
}

extern "C" int mr_comm_set_host(mr_ctx* ctx, mr_host_coll_fn fn, void* user, int nranks, int rank) {
    if (!ctx || nranks < 1 || rank < 0 || rank >= nranks) return MR_ERR_ARG;
    ctx->host_coll = fn;
    ctx->host_user = user;
    ctx->nranks = fn ? nranks : 1;
    ctx->rank = fn ? rank : 0;
    return MR_OK;
}

static size_t dt_size(int dt) { return dt == MR_DT_I32 ? 4 : 8; }
static ncclDataType_t dt_nccl(int dt) {
    return dt == MR_DT_F64 ? ncclFloat64 : dt == MR_DT_I32 ? ncclInt32 : dt == MR_DT_U64 ? ncclUint64 : ncclInt64;
}

int mr_coll_allreduce(mr_ctx* ctx, void* dbuf, int64_t n, int dtype, int op) {
    if (n <= 0 || (ctx->nranks == 1 && !ctx->comm && !ctx->host_coll)) return MR_OK;
    if (ctx->comm) return mr_comm_allreduce(ctx, dbuf, dbuf, (size_t)n, dt_nccl(dtype), op ? ncclMax : ncclSum);
    if (!ctx->host_coll) return mr_fail(ctx, MR_ERR_COMM, "no collective backend (mr_comm_init / mr_comm_set_host)");
    std::vector<unsigned char> h((size_t)n * dt_size(dtype));
    MR_TRY_HIP(ctx, hipMemcpyAsync(h.data(), dbuf, h.size(), hipMemcpyDeviceToHost, ctx->stream));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->host_coll(ctx->host_user, 0, h.data(), n, dtype, op))
        return mr_fail(ctx, MR_ERR_COMM, "host allreduce callback failed");
    MR_TRY_HIP(ctx, hipMemcpyAsync(dbuf, h.data(), h.size(), hipMemcpyHostToDevice, ctx->stream));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return MR_OK;
}

int mr_coll_allgather(mr_ctx* ctx, const void* dsend, void* drecv, int64_t n, int dtype) {
    const size_t bytes = (size_t)n * dt_size(dtype);
    if (ctx->comm) return n > 0 ? mr_comm_allgather(ctx, dsend, drecv, (size_t)n, dt_nccl(dtype)) : MR_OK;
    if (!ctx->host_coll) {   // a single rank: the gather is the send buffer
        if (bytes) MR_TRY_HIP(ctx, hipMemcpyAsync(drecv, dsend, bytes, hipMemcpyDeviceToDevice, ctx->stream));
        return MR_OK;
    }
    if (n <= 0) return MR_OK;
    std::vector<unsigned char> h(bytes * (size_t)ctx->nranks);
    MR_TRY_HIP(ctx, hipMemcpyAsync(h.data() + bytes * (size_t)ctx->rank, dsend, bytes, hipMemcpyDeviceToHost, ctx->stream));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (ctx->host_coll(ctx->host_user, 1, h.data(), n, dtype, 0)) return mr_fail(ctx, MR_ERR_COMM, "host allgather callback failed");
    MR_TRY_HIP(ctx, hipMemcpyAsync(drecv, h.data(), h.size(), hipMemcpyHostToDevice, ctx->stream));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    return MR_OK;
}

// ------------------------------------------------------------------------------ one-shot peer all-reduce
// The per-iteration all-reduce of the trace-sharded PageRank (2N limb words + the r' maxima,
// 160 KB at C4) is latency-bound: RCCL's ring takes 2 (R - 1) dependent steps.  Here every rank
// writes its words straight into every rank's receive region (peer memory mapped by IPC: xGMI
// stores on a node, the same HBM for ranks sharing one GPU), then signals with one system-scope
// atomic add per block on each destination's flag word for it, and each rank sums the R slots of
// its own region in rank order once all R flags have counted this round's blocks: one hop, exact
// (integer sums), identical on every rank.  Regions are uncached device memory (no stale L2 lines
// across devices); slots alternate by round parity, so a rank one round ahead never overwrites a
// slot still being summed (its next push of that parity needs every rank's flag of the round
// between).  Every spin is bounded (PEER_TIMEOUT): a missing peer becomes an error, not a hang.
// region: [flag words][all-reduce slots: 2 parities x R x W][exchange area A][exchange area B]
//         [block flags: R x nbf] (the k_fx_b-fused exchange, mr_peer_fx_prepare)
// flag words: [0, 64) all-reduce arrivals by source rank, [64, 127) exchange arrivals by source,
// 127 the error word
constexpr int PEER_FLAGS = 128, PEER_XF = 64, PEER_ERR = 127, PEER_MAXR = 63;
constexpr int PEER_T = 256;
constexpr unsigned long long PEER_TIMEOUT = 200000000ull;   // 2 s of the 100 MHz s_memrealtime clock
#define GLBP __attribute__((address_space(1)))

__global__ void __launch_bounds__(PEER_T) k_peer_push(const unsigned long long* __restrict__ src, int64_t n,
                                                      unsigned long long* const* __restrict__ peers, int nranks, int rank,
                                                      int64_t W, uint64_t seq) {
    const int64_t j = (int64_t)blockIdx.x * PEER_T + threadIdx.x;
    const unsigned long long v = j < n ? src[j] : 0ull;
    const size_t slot = (size_t)PEER_FLAGS + ((size_t)(seq & 1) * nranks + rank) * (size_t)W;
    for (int r = 0; r < nranks; ++r)
        if (j < n)
            __hip_atomic_store((GLBP unsigned long long*)peers[r] + slot + j, v, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x < nranks) {   // this block's words are out: count it in every destination's flag
        __atomic_thread_fence(__ATOMIC_RELEASE);
        __hip_atomic_fetch_add((GLBP unsigned long long*)peers[threadIdx.x] + rank, 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <class T>
__global__ void __launch_bounds__(PEER_T) k_peer_reduce(T* __restrict__ dst, int64_t n,
                                                        unsigned long long* __restrict__ region, int nranks, int64_t W,
                                                        uint64_t seq, unsigned long long need,
                                                        unsigned long long timeout) {
    __shared__ int s_ok;
    GLBP unsigned long long* reg = (GLBP unsigned long long*)region;
    if (threadIdx.x == 0) {
        s_ok = 1;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (int r = 0; r < nranks && s_ok; ++r)
            while (__hip_atomic_load(reg + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < need) {
                __builtin_amdgcn_s_sleep(2);
                if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
                    s_ok = 0;
                    __hip_atomic_store(reg + PEER_ERR, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
            }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
    }
    __syncthreads();
    if (!s_ok) return;
    const int64_t j = (int64_t)blockIdx.x * PEER_T + threadIdx.x;
    if (j >= n) return;
    const size_t base = (size_t)PEER_FLAGS + (size_t)(seq & 1) * nranks * (size_t)W + (size_t)j;
    T s = (T)0;
    for (int r = 0; r < nranks; ++r) {   // rank order: the same sum, bit for bit, on every rank
        const unsigned long long w = __hip_atomic_load(reg + base + (size_t)r * W, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_SYSTEM);
        if constexpr (sizeof(T) == 8 && (T)0.5 != (T)0) s += __longlong_as_double((long long)w);
        else s += (T)w;
    }
    dst[j] = s;
}

// A replaced region is RETIRED, not freed: its memory and this process's mappings of the other
// ranks' old regions stay until the context goes.  Freeing it would let the next allocation reuse
// its address, and a peer re-opening the new handle could be handed its cached mapping of the old
// one -- its pushes and signals would land in freed memory (seen: a kind exchange after two region
// replacements timed out on every rank).  Regions are a few MB; a context replaces one a handful
// of times (sizes only grow) plus once per peer timeout (mr_peer_check): a context that keeps timing
// out keeps its regions until mr_comm_peer_destroy, which is collective like mr_comm_peer_enable(0)
// (every rank frees its retired regions there; re-enabling maps fresh regions on every rank).
// MR_PEER_RETIRE_MAX (default 64) bounds the list: past it the peer path turns off (the RCCL / host
// collective carries on) instead of growing.
static void peer_retire(mr_ctx* ctx) {
    if (ctx->peer_region || ctx->peer_dev || !ctx->peer_map.empty()) {
        if (ctx->peer_region) (void)hipStreamSynchronize(ctx->stream);
        ctx->peer_old.push_back(mr_ctx::PeerOld{ctx->peer_region, ctx->peer_dev, ctx->peer_map, ctx->rank});
        static const size_t cap = [] {
            const char* e = getenv("MR_PEER_RETIRE_MAX");
            return (size_t)(e && atoi(e) > 0 ? atoi(e) : 64);
        }();
        if (ctx->peer_old.size() >= cap) ctx->peer_on = false;   // (the same count on every rank)
    }
    ctx->peer_map.clear();
    ctx->peer_region = nullptr;
    ctx->peer_dev = nullptr;
    ctx->peer_words = ctx->peer_xa = ctx->peer_xb = ctx->peer_nbf = 0;
    ctx->peer_seq = ctx->peer_xseq = ctx->peer_arrived = 0;
}

void mr_comm_peer_destroy(mr_ctx* ctx) {
    if (!ctx) return;
    peer_retire(ctx);
    for (const mr_ctx::PeerOld& o : ctx->peer_old) {
        for (size_t r = 0; r < o.map.size(); ++r)
            if (o.map[r] && (int)r != o.rank) (void)hipIpcCloseMemHandle(o.map[r]);
        if (o.region) (void)hipFree(o.region);
        if (o.dev) (void)hipFree(o.dev);
    }
    ctx->peer_old.clear();
}

// (collective) a receive region of at least `words` words per slot on every rank, mapped everywhere
// (collective: every rank asks for the same sizes) words per all-reduce slot, words of exchange
// areas A and B; a region too small is replaced (and re-exported) on every rank
static int peer_ensure(mr_ctx* ctx, int64_t words, int64_t xa = 0, int64_t xb = 0, int64_t nbf = 0) {
    if (ctx->peer_region && ctx->peer_words >= words && ctx->peer_xa >= xa && ctx->peer_xb >= xb && ctx->peer_nbf >= nbf)
        return MR_OK;
    const int R = ctx->nranks;
    if (R > PEER_MAXR) return mr_fail(ctx, MR_ERR_ARG, "peer collectives: at most %d ranks", PEER_MAXR);
    words = std::max(words, ctx->peer_words);
    xa = std::max(xa, ctx->peer_xa);
    xb = std::max(xb, ctx->peer_xb);
    nbf = std::max(nbf, ctx->peer_nbf);
    // (a first region already holds any fused graph's all-reduce: 2 x 16384 limbs + the r' slots)
    words = std::max<int64_t>(words, 2 * 16384 + PEER_MAXR + 1);
    peer_retire(ctx);
    // the retired-region cap reached (peer_retire turned the path off, the same count on every
    // rank): no fresh region -- the callers fall back to RCCL / the host collective on this code
    if (!ctx->peer_on) return mr_fail(ctx, MR_ERR_STATE, "peer collectives: retired-region cap reached");
    const size_t bytes = ((size_t)PEER_FLAGS + 2 * (size_t)R * (size_t)words + (size_t)xa + (size_t)xb +
                          (size_t)R * (size_t)nbf) * sizeof(unsigned long long);
    // (the region allocation and the mappings fail locally without returning alone: they are agreed
    // over the ranks below, every rank reaching the same collectives.  The staging buffers and the
    // handle gather are not: a rank failing THERE returns alone and its peers wait in the gather
    // until the fallback collective's own timeout -- a device out of memory for a few hundred bytes)
    int32_t bad = 0;
    char why[160] = "";
    hipIpcMemHandle_t mine;
    memset(&mine, 0, sizeof mine);
    if (hipExtMallocWithFlags(&ctx->peer_region, bytes, hipDeviceMallocUncached) != hipSuccess ||
        hipMemsetAsync(ctx->peer_region, 0, bytes, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess || hipIpcGetMemHandle(&mine, ctx->peer_region) != hipSuccess) {
        (void)hipGetLastError();
        snprintf(why, sizeof why, "receive region of %zu bytes (uncached, IPC-exported)", bytes);
        bad = 1;
    }
    ctx->peer_words = words;
    ctx->peer_xa = xa;
    ctx->peer_xb = xb;
    ctx->peer_nbf = nbf;
    ctx->peer_seq = ctx->peer_xseq = ctx->peer_arrived = 0;
    static_assert(sizeof(hipIpcMemHandle_t) % 8 == 0, "IPC handle size");
    const int64_t hw = (int64_t)(sizeof(hipIpcMemHandle_t) / 8);
    // the handle and this rank's device (PCI domain / bus / device) in one gather: ranks that share
    // a device must not spin inside large launches (mr_peer_fx_prepare)
    std::vector<uint64_t> mine_w((size_t)hw + 1);
    memcpy(mine_w.data(), &mine, sizeof mine);
    {
        hipDeviceProp_t pr;
        mine_w[(size_t)hw] = hipGetDeviceProperties(&pr, ctx->device) == hipSuccess
                                 ? ((uint64_t)(uint32_t)pr.pciDomainID << 32 | (uint64_t)pr.pciBusID << 8 | (uint64_t)pr.pciDeviceID)
                                 : (uint64_t)ctx->rank + 1;   // (unknown: assume distinct)
    }
    DBuf<uint64_t> hs, all;
    MR_TRY(hs.upload(ctx, mine_w.data(), (size_t)hw + 1));
    MR_TRY(all.alloc(ctx, (size_t)(hw + 1) * R));
    MR_TRY(mr_coll_allgather(ctx, hs.p, all.p, hw + 1, MR_DT_U64));
    std::vector<uint64_t> allw((size_t)(hw + 1) * R);
    MR_TRY_HIP(ctx, hipMemcpyAsync(allw.data(), all.p, allw.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, ctx->stream));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    std::vector<hipIpcMemHandle_t> hh((size_t)R);
    ctx->peer_same_dev = false;
    for (int r = 0; r < R; ++r) {
        memcpy(&hh[(size_t)r], allw.data() + (size_t)(hw + 1) * r, sizeof(hipIpcMemHandle_t));
        if (r != ctx->rank && allw[(size_t)(hw + 1) * r + hw] == mine_w[(size_t)hw]) ctx->peer_same_dev = true;
    }
    ctx->peer_map.assign((size_t)R, nullptr);
    for (int r = 0; r < R && !bad; ++r) {   // (a mapping may fail: no peer access between these devices)
        if (r == ctx->rank) {
            ctx->peer_map[(size_t)r] = ctx->peer_region;
            continue;
        }
        hipError_t e = hipIpcOpenMemHandle(&ctx->peer_map[(size_t)r], hh[(size_t)r], hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            ctx->peer_map[(size_t)r] = nullptr;
            snprintf(why, sizeof why, "hipIpcOpenMemHandle(rank %d): %s", r, hipGetErrorString(e));
            bad = 1;
        }
    }
    if (!bad && (hipMalloc((void**)&ctx->peer_dev, sizeof(void*) * R) != hipSuccess ||
                 hipMemcpy(ctx->peer_dev, ctx->peer_map.data(), sizeof(void*) * R, hipMemcpyHostToDevice) != hipSuccess)) {
        snprintf(why, sizeof why, "peer pointer table");
        bad = 1;
    }
    // every rank's region is mapped before anyone pushes into it, and the ranks agree on whether
    // every mapping succeeded: a rank that failed alone would otherwise leave the others waiting in
    // their next all-reduce for pushes that never come.  On failure every rank drops the peer path
    // (MR_ERR_STATE: the callers take the RCCL / host collective instead).
    DBuf<int32_t> one;
    MR_TRY(one.upload(ctx, &bad, 1));
    MR_TRY(mr_coll_allreduce(ctx, one.p, 1, MR_DT_I32, 1));
    MR_TRY(one.download(ctx, &bad, 1));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (bad) {
        peer_retire(ctx);
        ctx->peer_on = false;
        if (why[0]) fprintf(stderr, "[microrank] peer collectives off on rank %d: %s\n", ctx->rank, why);
        return MR_ERR_STATE;
    }
    return MR_OK;
}

// MR_PEER_TIMEOUT_MS: the bounded spins' limit (default 2000 ms)
unsigned long long mr_peer_timeout_ticks() {
    static const unsigned long long t = [] {
        const char* e = getenv("MR_PEER_TIMEOUT_MS");
        const long long ms = e ? atoll(e) : 0;
        return ms > 0 ? (unsigned long long)ms * 100000ull : PEER_TIMEOUT;
    }();
    return t;
}

template <class T>
static int peer_allreduce(mr_ctx* ctx, T* dbuf, int64_t n) {
    if (!ctx->peer_on || ctx->nranks < 2 || !mr_coll_ready(ctx)) return MR_ERR_STATE;
    MR_TRY(peer_ensure(ctx, n));
    const int nb = cdiv(n, PEER_T);
    const uint64_t seq = ctx->peer_seq++;
    // a source's flag counts every block it has pushed into this region since the region was made;
    // n (hence nb) changes between calls (2N + R on the fused path, N + R on the tile path, N per
    // graph), so the round's target is the running total, not nb * rounds.  Every rank runs the
    // same sequence of all-reduces with the same n (a collective), so every source's flag reaches
    // exactly this total when it has pushed this round.
    ctx->peer_arrived += (uint64_t)nb;
    hipLaunchKernelGGL(k_peer_push, dim3(nb), dim3(PEER_T), 0, ctx->stream, (const unsigned long long*)dbuf, n,
                       ctx->peer_dev, ctx->nranks, ctx->rank, ctx->peer_words, seq);
    hipLaunchKernelGGL(k_peer_reduce<T>, dim3(nb), dim3(PEER_T), 0, ctx->stream, dbuf, n,
                       (unsigned long long*)ctx->peer_region, ctx->nranks, ctx->peer_words, seq,
                       (unsigned long long)ctx->peer_arrived, mr_peer_timeout_ticks());
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}
int mr_peer_allreduce_u64(mr_ctx* ctx, unsigned long long* dbuf, int64_t n) { return peer_allreduce(ctx, dbuf, n); }
int mr_peer_allreduce_f64(mr_ctx* ctx, double* dbuf, int64_t n) { return peer_allreduce(ctx, dbuf, n); }

// (collective) a peer that never arrived (a k_peer_reduce / k_peer_wait timeout) on ANY rank:
// the ranks agree on it through the fallback collective (RCCL or the host callback, never the
// regions themselves), and then every rank drops its region -- the error word and the arrival
// counts of an aborted round are stale -- so the next peer operation maps fresh, zeroed regions
// everywhere.  A rank whose own rounds completed still reports the failure: its peers' did not.
int mr_peer_check(mr_ctx* ctx, const char* what) {
    if (!ctx->peer_region) return MR_OK;   // (created and dropped collectively: the same on every rank)
    unsigned long long w = 0;
    MR_TRY_HIP(ctx, hipMemcpyAsync(&w, (unsigned long long*)ctx->peer_region + PEER_ERR, 8,
                                   hipMemcpyDeviceToHost, ctx->stream));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    int32_t any = w != 0 ? 1 : 0;
    DBuf<int32_t> f;
    MR_TRY(f.upload(ctx, &any, 1));
    MR_TRY(mr_coll_allreduce(ctx, f.p, 1, MR_DT_I32, 1));
    MR_TRY(f.download(ctx, &any, 1));
    MR_TRY_HIP(ctx, hipStreamSynchronize(ctx->stream));
    if (!any) return MR_OK;
    peer_retire(ctx);
    return mr_fail(ctx, MR_ERR_COMM, "%s: a rank did not arrive within the peer timeout (regions reset)", what);
}

// ---- exchanges (all-to-all) through the regions' areas A and B: a round is a set of puts into
// other ranks' areas, then one signal per destination; a rank waits for every source's signal
constexpr int PUT_B = 64;   // blocks of a put kernel (grid-stride): each counts once at its destination
__global__ void __launch_bounds__(PEER_T) k_peer_put(const unsigned long long* __restrict__ src, int64_t n,
                                                     unsigned long long* dst) {
    for (int64_t j = (int64_t)blockIdx.x * PEER_T + threadIdx.x; j < n; j += (int64_t)PUT_B * PEER_T)
        __hip_atomic_store((GLBP unsigned long long*)dst + j, src[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// after the round's puts (earlier launches on this stream, complete): one signal per destination
__global__ void k_peer_signal(unsigned long long* const* __restrict__ peers, int nranks, int rank) {
    if ((int)threadIdx.x < nranks) {
        __atomic_thread_fence(__ATOMIC_RELEASE);
        __hip_atomic_fetch_add((GLBP unsigned long long*)peers[threadIdx.x] + PEER_XF + rank, 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
__global__ void k_peer_wait(unsigned long long* region, int nranks, unsigned long long need,
                            unsigned long long timeout) {
    GLBP unsigned long long* reg = (GLBP unsigned long long*)region;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (int r = 0; r < nranks; ++r)
        while (__hip_atomic_load(reg + PEER_XF + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < need) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
                __hip_atomic_store(reg + PEER_ERR, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return;
            }
        }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
}

// ---- the exchange fused into k_fx_b (mr_pagerank.hip): mode 1 blocks push their ops' limbs into
// every rank's slot for this rank and then store the round number (seq + 1) in a per-(source,
// block) flag; mode 2 block b waits for flag (src, b) of every source -- only the words it sums --
// and sums the R slots in rank order.  A flag holds the number of the last round its block pushed
// (a store, not a count), so graphs of different sizes on one context need no bookkeeping.
// (collective) px for words per slot (2N + R) and nbf k_fx_b blocks; MR_ERR_STATE when the peer path
// is off or the ranks could not map each other's regions.
int mr_peer_fx_prepare(mr_ctx* ctx, int64_t words, int32_t nbf, MrPeerX* px) {
    if (!ctx->peer_on || ctx->nranks < 2 || !mr_coll_ready(ctx)) return MR_ERR_STATE;
    const int rc = peer_ensure(ctx, words, 0, 0, nbf);
    if (rc != MR_OK) return rc;
    const int R = ctx->nranks;
    px->peers = ctx->peer_dev;
    px->region = (unsigned long long*)ctx->peer_region;
    px->R = R;
    px->rank = ctx->rank;
    px->nbf = (int32_t)ctx->peer_nbf;
    px->W = ctx->peer_words;
    px->slots = PEER_FLAGS;
    px->bflags = (int64_t)PEER_FLAGS + 2 * (int64_t)R * ctx->peer_words + ctx->peer_xa + ctx->peer_xb;
    px->err = PEER_ERR;
    px->seq = ctx->peer_seq;
    px->timeout = mr_peer_timeout_ticks();
    px->spin = 1;
    // (tests, read per call) MR_PEER_TEST_MUTE=<rank>: that rank pushes its limbs but never stores
    // its round flags -- every rank's wait then runs into the timeout (a peer that never arrives)
    const char* me = getenv("MR_PEER_TEST_MUTE");
    px->mute = me && atoi(me) == ctx->rank ? 1 : 0;
    return MR_OK;
}
void mr_peer_fx_round_done(mr_ctx* ctx, MrPeerX* px) {
    ++ctx->peer_seq;
    px->seq = ctx->peer_seq;
}
bool mr_peer_same_device(const mr_ctx* ctx) { return ctx->peer_same_dev; }

// one block waits for every (source, block) flag of round seq (ranks sharing a device: mode-2
// blocks spinning beside a peer's k_tr_a would hold the CUs its 160-KB blocks need)
__global__ void __launch_bounds__(PEER_T) k_peer_bwait(const MrPeerX px, int32_t nb) {
    GLBP unsigned long long* reg = (GLBP unsigned long long*)px.region;
    const unsigned long long need = px.seq + 1, t0 = __builtin_amdgcn_s_memrealtime();
    for (int64_t i = threadIdx.x; i < (int64_t)px.R * nb; i += PEER_T) {
        const int64_t w = px.bflags + (i / nb) * px.nbf + i % nb;
        while (__hip_atomic_load(reg + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < need) {
            __builtin_amdgcn_s_sleep(2);
            // (a round of this call that already timed out: stop at once)
            if (__builtin_amdgcn_s_memrealtime() - t0 > px.timeout ||
                __hip_atomic_load(reg + px.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0ull) {
                __hip_atomic_store(reg + px.err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return;
            }
        }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
}
int mr_peer_fx_wait(mr_ctx* ctx, const MrPeerX& px, int32_t nb) {
    hipLaunchKernelGGL(k_peer_bwait, dim3(1), dim3(PEER_T), 0, ctx->stream, px, nb);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}

bool mr_peer_ready(const mr_ctx* ctx) { return ctx->peer_on && ctx->nranks >= 2 && mr_coll_ready(ctx); }

int mr_peer_xensure(mr_ctx* ctx, int64_t xa, int64_t xb) { return peer_ensure(ctx, 1, xa, xb); }

unsigned long long* mr_peer_area(mr_ctx* ctx, int rank, int area) {
    unsigned long long* base = (unsigned long long*)ctx->peer_map[(size_t)rank];
    return base + PEER_FLAGS + 2 * (size_t)ctx->nranks * (size_t)ctx->peer_words + (area ? (size_t)ctx->peer_xa : 0);
}

int mr_peer_put(mr_ctx* ctx, const unsigned long long* d_src, int64_t n, int rank, int area, int64_t offset) {
    if (n <= 0) return MR_OK;
    hipLaunchKernelGGL(k_peer_put, dim3(PUT_B), dim3(PEER_T), 0, ctx->stream, d_src, n,
                       mr_peer_area(ctx, rank, area) + offset);
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}

// the round's signals, then the wait for every rank's
int mr_peer_round(mr_ctx* ctx) {
    const uint64_t x = ctx->peer_xseq++;
    hipLaunchKernelGGL(k_peer_signal, dim3(1), dim3(64), 0, ctx->stream, ctx->peer_dev, ctx->nranks, ctx->rank);
    hipLaunchKernelGGL(k_peer_wait, dim3(1), dim3(1), 0, ctx->stream, (unsigned long long*)ctx->peer_region,
                       ctx->nranks, (unsigned long long)(x + 1), mr_peer_timeout_ticks());
    MR_TRY_HIP(ctx, hipGetLastError());
    return MR_OK;
}

unsigned long long* const* mr_peer_map_dev(mr_ctx* ctx) { return ctx->peer_dev; }

extern "C" int mr_comm_peer_enable(mr_ctx* ctx, int enable) {
    if (!ctx) return MR_ERR_ARG;
    if (!enable) mr_comm_peer_destroy(ctx);
    ctx->peer_on = enable != 0;
    return MR_OK;
}

extern "C" int mr_comm_peer_active(mr_ctx* ctx, int* active) {
    if (!ctx || !active) return MR_ERR_ARG;
    *active = ctx->peer_on && ctx->peer_region ? 1 : 0;
    return MR_OK;
}
