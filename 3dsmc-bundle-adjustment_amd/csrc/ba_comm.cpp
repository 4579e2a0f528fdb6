// ba_comm.cpp — RCCL and host-callback backends of ba_comm.h.
#include "ba_comm.h"

#include <rccl/rccl.h>

#include <cstring>
#include <string>

namespace miba {

static thread_local std::string g_comm_err;

static ncclRedOp_t to_op(CommOp op) { return op == COMM_SUM ? ncclSum : (op == COMM_MAX ? ncclMax : ncclMin); }

// Host collective: device -> pinned stage, the callback reduces in place, stage -> device. The stage is
// reused by the next collective only after this one's upload (same stream) and a synchronisation.
static hipError_t host_allreduce(const Comm& cc, const void* send, void* recv, size_t count, CommType t, CommOp op,
                                 hipStream_t s) {
    Comm& c = const_cast<Comm&>(cc);
    const size_t bytes = count * (t == COMM_F64 ? 8 : 4);
    hipError_t e = hipSuccess;
    if (bytes > c.stage_cap) {
        if (c.stage) (void)hipHostFree(c.stage);
        c.stage = nullptr;
        c.stage_cap = 0;
        e = hipHostMalloc(&c.stage, bytes, hipHostMallocDefault);
        if (e != hipSuccess) { g_comm_err = "pinned staging allocation failed"; return e; }
        c.stage_cap = bytes;
    }
    e = hipMemcpyAsync(c.stage, send, bytes, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) return e;
    const int rc = c.host_fn(c.stage, (int64_t)count, t == COMM_F64 ? 0 : 1, (int32_t)op, c.host_user);
    if (rc != 0) {
        g_comm_err = "host all-reduce callback failed (" + std::to_string(rc) + ")";
        return hipErrorUnknown;
    }
    e = hipMemcpyAsync(recv, c.stage, bytes, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);  // the stage is host memory the next call rewrites
    return e;
}

hipError_t comm_allreduce(const Comm& c, const void* send, void* recv, size_t count, CommType t, CommOp op,
                          hipStream_t s) {
    if (!c.on() || count == 0) {
        if (send != recv && count)
            return hipMemcpyAsync(recv, send, count * (t == COMM_F64 ? 8 : 4), hipMemcpyDeviceToDevice, s);
        return hipSuccess;
    }
    if (c.host_fn) return host_allreduce(c, send, recv, count, t, op, s);
    const ncclResult_t r = ncclAllReduce(send, recv, count, t == COMM_F64 ? ncclFloat64 : ncclInt32, to_op(op),
                                         static_cast<ncclComm_t>(c.nccl), s);
    if (r != ncclSuccess) {
        g_comm_err = std::string("ncclAllReduce: ") + ncclGetErrorString(r);
        return hipErrorUnknown;
    }
    return hipSuccess;
}

int comm_unique_id(void* out, size_t n) {
    if (n < sizeof(ncclUniqueId)) {
        g_comm_err = "unique id buffer too small";
        return -1;
    }
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) {
        g_comm_err = std::string("ncclGetUniqueId: ") + ncclGetErrorString(r);
        return -1;
    }
    std::memcpy(out, &id, sizeof(id));
    return 0;
}

int comm_init(Comm& c, int nranks, int rank, const void* id) {
    comm_destroy(c);
    if (nranks < 1 || rank < 0 || rank >= nranks) {
        g_comm_err = "invalid rank / nranks";
        return -1;
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        g_comm_err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
        return -1;
    }
    c.nccl = comm;
    c.rank = rank;
    c.nranks = nranks;
    return 0;
}

int comm_init_host(Comm& c, int nranks, int rank, HostAllreduceFn fn, void* user) {
    comm_destroy(c);
    if (nranks < 1 || rank < 0 || rank >= nranks || !fn) {
        g_comm_err = !fn ? "null host all-reduce callback" : "invalid rank / nranks";
        return -1;
    }
    c.host_fn = fn;
    c.host_user = user;
    c.rank = rank;
    c.nranks = nranks;
    return 0;
}

void comm_destroy(Comm& c) {
    if (c.nccl) ncclCommDestroy(static_cast<ncclComm_t>(c.nccl));
    if (c.stage) (void)hipHostFree(c.stage);
    c.stage = nullptr;
    c.stage_cap = 0;
    c.host_fn = nullptr;
    c.host_user = nullptr;
    c.nccl = nullptr;
    c.rank = 0;
    c.nranks = 1;
}

const char* comm_last_error() { return g_comm_err.c_str(); }

}  // namespace miba
