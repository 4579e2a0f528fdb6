// ba_comm.h — landmark-shard communicator of a ba_context.
//
// One process per GPU; every rank holds the same window cameras / intrinsics and its
// own block of landmarks (points with all their observations). Per LM iteration the
// ranks exchange (out-of-place, on the solver stream, always in the same order):
//   1. [camdata | intrinsics partials] after the camera-side linearisation (sum),
//   2. the packed envelope of the reduced camera system S + rhs (sum),
//   3. the step scalars (sum) and the point-side maxima (max).
// RCCL over xGMI. A context without a communicator runs the unsharded solver (no
// collective); with one (any nranks, including 1) it runs the sharded path.
#ifndef MIBA_BA_COMM_H
#define MIBA_BA_COMM_H

#include <hip/hip_runtime.h>

#include <cstddef>

namespace miba {

struct Comm {
    void* nccl = nullptr;  // ncclComm_t
    int rank = 0;
    int nranks = 1;
    bool on() const { return nccl != nullptr; }
};

enum CommOp { COMM_SUM = 0, COMM_MAX = 1, COMM_MIN = 2 };
enum CommType { COMM_F64 = 0, COMM_I32 = 1 };

// all-reduce of count elements on stream s (in place when send == recv); a copy when !c.on()
hipError_t comm_allreduce(const Comm& c, const void* send, void* recv, size_t count, CommType t, CommOp op,
                          hipStream_t s);
int comm_unique_id(void* out, size_t n);                       // 0 = ok
int comm_init(Comm& c, int nranks, int rank, const void* id);  // 0 = ok (collective over the ranks)
void comm_destroy(Comm& c);
const char* comm_last_error();

}  // namespace miba

#endif  // MIBA_BA_COMM_H
