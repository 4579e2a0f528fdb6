// Read-request calibration for the TCC EA counters on gfx950 (settles the request size behind FETCH_SIZE for
// the access forms libmiba's kernels use). Each kernel reads a fresh 64 MiB buffer exactly once:
//   k_plain8   8 B per lane, plain global_load_dwordx2           (the Jacobian / Schur record loads)
//   k_plain16 16 B per lane, plain global_load_dwordx4           (the guide's calibrated streaming form)
//   k_agent8   8 B per lane, relaxed agent-scope atomic loads     (k_bcr_split's ld_pub / tail_ld)
//   k_store8   8 B per lane, relaxed agent-scope atomic stores    (st_pub) of 64 MiB
// Run under rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum (and WRREQ / WRREQ_64B) and divide the
// known bytes by the request count.
// build: hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/_build/pmc_calib
#include <hip/hip_runtime.h>

#include <cstdio>

static constexpr size_t NBYTES = 64ull << 20;

__global__ void k_plain8(const double* __restrict__ p, double* out, size_t n) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
    if (s == 12345.0) out[0] = s;
}
__global__ void k_plain16(const double2* __restrict__ p, double* out, size_t n) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = p[i];
        s += v.x + v.y;
    }
    if (s == 12345.0) out[0] = s;
}
__global__ void k_agent8(const unsigned long long* p, double* out, size_t n) {
    unsigned long long s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s == 12345ull) out[0] = (double)s;
}
__global__ void k_store8(unsigned long long* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __hip_atomic_store(p + i, (unsigned long long)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
            return 1;                                                          \
        }                                                                      \
    } while (0)

int main() {
    void* buf[4];
    double* out;
    for (auto& b : buf) {
        CK(hipMalloc(&b, NBYTES));
        CK(hipMemset(b, 0, NBYTES));
    }
    CK(hipMalloc(&out, 64));
    // flush the Infinity Cache between kernels with a 512 MiB sweep (its hits count as EA requests too)
    void* sweep;
    CK(hipMalloc(&sweep, 512ull << 20));
    const size_t n8 = NBYTES / 8;
    const dim3 g(4096), b(256);
    CK(hipMemset(sweep, 1, 512ull << 20));
    k_plain8<<<g, b>>>((const double*)buf[0], out, n8);
    CK(hipMemset(sweep, 2, 512ull << 20));
    k_plain16<<<g, b>>>((const double2*)buf[1], out, n8 / 2);
    CK(hipMemset(sweep, 3, 512ull << 20));
    k_agent8<<<g, b>>>((const unsigned long long*)buf[2], out, n8);
    CK(hipMemset(sweep, 4, 512ull << 20));
    k_store8<<<g, b>>>((unsigned long long*)buf[3], n8);
    CK(hipDeviceSynchronize());
    std::printf("each kernel moved %zu bytes\n", NBYTES);
    return 0;
}
