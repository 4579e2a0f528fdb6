// ba_solve_util.h — small device helpers shared by the reduced-camera-system solvers (ba_bcr.hip, ba_band.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <type_traits>

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

// Wave reductions by DPP moves (gfx9 DPP controls, two 32-bit moves per f64) instead of __shfl_xor, which HIP
// lowers to ds_bpermute: an LDS-crossbar round trip per step and half, on the critical path of every workgroup-wide
// sum (a 5-value block sum took ~1 us in the band tail's back-substitution chunks, MIBA_BCR_STAMPS). Called in
// uniform control flow with all 64 lanes active. Every lane of a row ends with the bitwise same value (the pairings
// are symmetric and f64 addition commutes), so the order is fixed per lane and run to run.
enum : int {
    DPP_QP_X1 = 0xB1,       // quad_perm [1,0,3,2]: lane ^ 1
    DPP_QP_X2 = 0x4E,       // quad_perm [2,3,0,1]: lane ^ 2
    DPP_ROW_MIRROR = 0x140, // lane 15 - i within the row of 16
    DPP_ROW_HMIRROR = 0x141,  // lane 7 - i within each half row of 8
    DPP_ROW_BCAST15 = 0x142,  // lane 15 of row r -> row r + 1 (row_mask selects the rows written)
    DPP_ROW_BCAST31 = 0x143,  // lane 31 -> rows 2, 3
};
// x from the DPP source lane; lanes of rows outside ROW_MASK get `old`
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_f64(double x, double old) {
    const long long u = __double_as_longlong(x), o = __double_as_longlong(old);
    const int lo = __builtin_amdgcn_update_dpp((int)o, (int)u, CTRL, ROW_MASK, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(u >> 32), CTRL, ROW_MASK, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// the sum over each row of 16 lanes, in every lane of the row
// (fp contract off: the adds must not fuse with a caller's product into an FMA, whose rounding would then depend on
// the inlining context — the obs32 and f64 instantiations of a kernel must sum bit for bit alike)
__device__ __forceinline__ double dpp_row_sum(double x) {
#pragma clang fp contract(off)
    x += dpp_f64<DPP_QP_X1>(x, 0.0);
    x += dpp_f64<DPP_QP_X2>(x, 0.0);
    x += dpp_f64<DPP_ROW_HMIRROR>(x, 0.0);
    x += dpp_f64<DPP_ROW_MIRROR>(x, 0.0);
    return x;
}
__device__ __forceinline__ double readlane_f64(double x, int l) {
    const long long u = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)u, l), hi = __builtin_amdgcn_readlane((int)(u >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// the sum over the wave, in every lane: the row sums r0..r3 by DPP, then the rows combined by two xor exchanges
// ((r0 + r1) + (r2 + r3), the same bits in every lane). (A lane-63 total by row_bcast:15 / row_bcast:31 and a
// v_readlane broadcast made the obs32 and f64 instantiations of a kernel differ in the last bit:
// test_obs32_records_match_f64_arrays_bitwise.)
__device__ __forceinline__ double dpp_wave_sum(double x) {
#pragma clang fp contract(off)
    x = dpp_row_sum(x);
    x += __shfl_xor(x, 16);
    x += __shfl_xor(x, 32);
    return x;
}
__device__ __forceinline__ double dpp_wave_max(double x) {
    x = fmax(x, dpp_f64<DPP_QP_X1>(x, x));
    x = fmax(x, dpp_f64<DPP_QP_X2>(x, x));
    x = fmax(x, dpp_f64<DPP_ROW_HMIRROR>(x, x));
    x = fmax(x, dpp_f64<DPP_ROW_MIRROR>(x, x));
    x = fmax(x, dpp_f64<DPP_ROW_BCAST15, 0xa>(x, x));
    x = fmax(x, dpp_f64<DPP_ROW_BCAST31, 0xc>(x, x));
    return readlane_f64(x, 63);
}
// v from lane l to every lane (v_readlane on both halves of the f64)
__device__ __forceinline__ double bcast_b(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// compile-time loop (a DPP lane select is an immediate)
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        sfor<B + 1, E>(f);
    }
}

// a -= lr[lane K of this lane's 16-lane row] * l in ONE v_fmac_f64_dpp: row_newbcast (the DPP64 control of gfx90a+)
// hands src0 from lane K of the row to every lane of it. NOP: two wait states first — a DPP read of a VGPR that a VALU
// wrote in the previous two cycles is a hazard the compiler's hazard recognizer does not see through inline assembly
// (callers put it on the first DPP read after the source was produced; the later reads of the same source follow
// other DPP instructions).
template <int K, bool NOP>
__device__ __forceinline__ void fnma_row_bcast(double& a, double lr, double l) {
    static_assert(K >= 0 && K < 16, "row_newbcast selects a lane of the 16-lane row");
    if constexpr (NOP)
        asm("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
            : "+v"(a) : "v"(lr), "v"(l), "i"(K));
    else
        asm("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(a) : "v"(lr), "v"(l), "i"(K));
}

// w += w[lane K of this lane's 16-lane row] * c (one v_fmac_f64_dpp reading its own destination through row_newbcast);
// the two wait states first: w was written by the VALU instruction just before (the previous step of the caller's chain)
template <int K>
__device__ __forceinline__ void fmac_self_row_bcast(double& w, double c) {
    static_assert(K >= 0 && K < 16, "row_newbcast selects a lane of the 16-lane row");
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "+v"(w) : "v"(c), "i"(K));
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
