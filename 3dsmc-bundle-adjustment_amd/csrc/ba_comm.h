// ba_comm.h — landmark-shard communicator of a ba_context.
//
// One process per GPU; every rank holds the same window cameras / intrinsics and its
// own block of landmarks (points with all their observations). Per LM iteration the
// ranks exchange (out-of-place, on the solver stream, always in the same order):
//   1. [camdata | intrinsics partials] after the camera-side linearisation (sum),
//   2. the packed envelope of the reduced camera system S + rhs (sum),
//   3. the step scalars (sum) and the point-side maxima (max).
// RCCL over xGMI, or a caller-supplied host collective (ba_comm_init_host: the device buffer is
// copied to pinned host memory, reduced by the callback and copied back, in stream order). A context
// without a communicator runs the unsharded solver (no collective); with one (any nranks,
// including 1) it runs the sharded path.
#ifndef MIBA_BA_COMM_H
#define MIBA_BA_COMM_H

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace miba {

// Host-side collective supplied by the caller (ba_comm_init_host): in-place all-reduce of count
// elements of a host buffer; dtype 0 = f64, 1 = i32; op 0 = sum, 1 = max, 2 = min; returns 0 on success.
typedef int32_t (*HostAllreduceFn)(void* buf, int64_t count, int32_t dtype, int32_t op, void* user);

struct Comm {
    void* nccl = nullptr;  // ncclComm_t (RCCL over xGMI: the product backend)
    HostAllreduceFn host_fn = nullptr;  // or a host collective (MPI, gloo, ...), staged through pinned memory
    void* host_user = nullptr;
    void* stage = nullptr;  // pinned staging buffer of the host collective
    size_t stage_cap = 0;
    int rank = 0;
    int nranks = 1;
    bool on() const { return nccl != nullptr || host_fn != nullptr; }
};

enum CommOp { COMM_SUM = 0, COMM_MAX = 1, COMM_MIN = 2 };
enum CommType { COMM_F64 = 0, COMM_I32 = 1 };

// all-reduce of count elements on stream s (in place when send == recv); a copy when !c.on()
hipError_t comm_allreduce(const Comm& c, const void* send, void* recv, size_t count, CommType t, CommOp op,
                          hipStream_t s);
int comm_unique_id(void* out, size_t n);                       // 0 = ok
int comm_init(Comm& c, int nranks, int rank, const void* id);  // 0 = ok (collective over the ranks)
int comm_init_host(Comm& c, int nranks, int rank, HostAllreduceFn fn, void* user);  // 0 = ok (local)
void comm_destroy(Comm& c);
const char* comm_last_error();

}  // namespace miba

#endif  // MIBA_BA_COMM_H
