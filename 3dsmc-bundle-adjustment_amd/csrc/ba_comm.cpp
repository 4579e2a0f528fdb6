// ba_comm.cpp — RCCL backend of ba_comm.h.
#include "ba_comm.h"

#include <rccl/rccl.h>

#include <cstring>
#include <string>

namespace miba {

static thread_local std::string g_comm_err;

static ncclRedOp_t to_op(CommOp op) { return op == COMM_SUM ? ncclSum : (op == COMM_MAX ? ncclMax : ncclMin); }

hipError_t comm_allreduce(const Comm& c, const void* send, void* recv, size_t count, CommType t, CommOp op,
                          hipStream_t s) {
    if (!c.on() || count == 0) {
        if (send != recv && count)
            return hipMemcpyAsync(recv, send, count * (t == COMM_F64 ? 8 : 4), hipMemcpyDeviceToDevice, s);
        return hipSuccess;
    }
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

void comm_destroy(Comm& c) {
    if (c.nccl) ncclCommDestroy(static_cast<ncclComm_t>(c.nccl));
    c.nccl = nullptr;
    c.rank = 0;
    c.nranks = 1;
}

const char* comm_last_error() { return g_comm_err.c_str(); }

}  // namespace miba
