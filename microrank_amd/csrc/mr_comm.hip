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
