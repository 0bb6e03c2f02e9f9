// RCCL (over xGMI) for the trace-sharded PageRank: one process per GPU, the score-vector
// all-reduce per iteration.  librccl is dlopen'ed on first use so the library itself loads on
// machines (and CPU test containers) without it.
#include <dlfcn.h>
#include <cstring>
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
