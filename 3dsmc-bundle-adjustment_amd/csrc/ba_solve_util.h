// ba_solve_util.h — small device helpers shared by the reduced-camera-system solvers (ba_bcr.hip, ba_band.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

namespace miba {

// chol_flag is raised by several workgroups at once: fetch-or, so a timeout is never overwritten
__device__ __forceinline__ void raise_flag(int* flag, int bit) {
    __hip_atomic_fetch_or(flag, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// shader clock (100 MHz real-time counter) for the diagnostic phase stamps
__device__ __forceinline__ unsigned long long realtime_now() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// v from lane l to every lane (v_readlane on both halves of the f64)
__device__ __forceinline__ double bcast_b(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// 4x4 border system (C - sum B^T V) y_k = b_k - sum B^T u on one thread: bk = [b_k | S_kk lower packed],
// red[m * 5 + c] = (B^T [u | V])[m][c]. bad: a non-positive pivot (replaced by 1).
__device__ __forceinline__ void border_solve4(const double* bk, const double* red, double* yk, bool& bad) {
    double Cm[16], bp[4];
    int q = 0;
    for (int mm = 0; mm < 4; ++mm)
        for (int l = 0; l <= mm; ++l, ++q) {
            const double v = bk[4 + q];
            Cm[mm * 4 + l] = v - red[mm * 5 + 1 + l];
            Cm[l * 4 + mm] = v - red[l * 5 + 1 + mm];
        }
    for (int mm = 0; mm < 4; ++mm) bp[mm] = bk[mm] - red[mm * 5];
    double Lm[16] = {0};
    for (int j = 0; j < 4; ++j) {
        double d = Cm[j * 4 + j];
        for (int k = 0; k < j; ++k) d -= Lm[j * 4 + k] * Lm[j * 4 + k];
        if (!(d > 0.0)) { bad = true; d = 1.0; }
        Lm[j * 4 + j] = sqrt(d);
        for (int r = j + 1; r < 4; ++r) {
            double v = Cm[r * 4 + j];
            for (int k = 0; k < j; ++k) v -= Lm[r * 4 + k] * Lm[j * 4 + k];
            Lm[r * 4 + j] = v / Lm[j * 4 + j];
        }
    }
    double z[4];
    for (int r = 0; r < 4; ++r) {
        double v = bp[r];
        for (int k = 0; k < r; ++k) v -= Lm[r * 4 + k] * z[k];
        z[r] = v / Lm[r * 4 + r];
    }
    for (int r = 3; r >= 0; --r) {
        double v = z[r];
        for (int k = r + 1; k < 4; ++k) v -= Lm[k * 4 + r] * z[k];
        z[r] = v / Lm[r * 4 + r];
    }
    for (int mm = 0; mm < 4; ++mm) yk[mm] = z[mm];
}

}  // namespace miba
