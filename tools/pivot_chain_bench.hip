// Pivot-chain micro-benchmark for the BCR's 64x64 block Cholesky (k_bcr_split's wave-0 chain): one wave factors
// a tall 64 x 16 column panel in registers (lane r holds row r), 16 pivots, repeated. Variants:
//   0  the kernel's chain: y = rsq(d) + one Newton step folded into l = a y (1 + e/2); next pivot
//      dn = a_{j+1,j+1} - l^2 on lane j+1, broadcast by v_readlane; trailing updates a[k] -= l bcast(l, k)
//   1  the next pivot from the reciprocal: dn = a_{j+1,j+1} - a_{j+1,j}^2 / d_j with r = rcp(d) + one Newton
//      step (rcp + 3 dependent ops + readlane on the chain instead of rsq + 4); l and the trailing updates as 0
//   2  variant 0 without the trailing updates (the chain alone: a lower bound)
//   3  variant 0 with the trailing updates of columns j + 2.. fed by an LDS broadcast of the multipliers
//   4  variant 0 with pivot j - 1's trailing updates issued inside pivot j's chain (sched_barrier fences; same L)
//   5  variant 4 without the fences
//   6  variant 0 with the trailing updates of columns j + 2.. as one v_fmac_f64_dpp each: the multipliers of lanes
//      0-15 copied to every 16-lane row (ds_bpermute), then row_newbcast:k hands lane k's l to the FMA (no v_readlane)
//   7  variant 6 with column j + 1 by DPP as well (only the next pivot's value by v_readlane)
// Reports ns and shader cycles per pivot and the max |L L^T - A| of the last repetition.
// build: hipcc --offload-arch=gfx950 -O3 tools/pivot_chain_bench.hip -o /tmp/pcb && /tmp/pcb
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

__device__ __forceinline__ double bcast(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ unsigned long long rt() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ unsigned long long clk() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

// a -= lr[lane K of this lane's 16-lane row] * l  (one v_fmac_f64_dpp; the DPP64 control row_newbcast); NOP: the two
// wait states a DPP read needs after a VALU write of its source (lr comes from ds_bpermute, but a copy may intervene)
template <int K, bool NOP>
__device__ __forceinline__ void fnma_row_bcast(double& a, double lr, double l) {
    if constexpr (NOP)
        asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                     : "+v"(a) : "v"(lr), "v"(l), "i"(K));
    else
        asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                     : "+v"(a) : "v"(lr), "v"(l), "i"(K));
}
template <int J, int K>
__device__ __forceinline__ void trail_dpp(double (&a)[16], double lr, double l) {
    if constexpr (K < 16) {
        fnma_row_bcast<K, K == J>(a[K], lr, l);
        trail_dpp<J, K + 1>(a, lr, l);
    }
}
template <int J, int V>
__device__ __forceinline__ void chain_dpp_step(double (&a)[16], double& my_inv, double& dn) {
    const int r = threadIdx.x & 63;
    const double d = dn;
    const double y = __builtin_amdgcn_rsq(d);
    const double e = __builtin_fma(-d * y, y, 1.0);
    const double l = __builtin_fma(0.5 * a[J] * y, e, a[J] * y);
    my_inv = (r == J) ? __builtin_fma(0.5 * y, e, y) : my_inv;
    a[J] = l;
    if constexpr (J < 15) {
        dn = bcast(__builtin_fma(-l, l, a[J + 1]), J + 1);
        const double lr = __shfl(l, r & 15);  // row 0's multipliers in every row
        if constexpr (V == 6) {
            a[J + 1] = __builtin_fma(-l, bcast(l, J + 1), a[J + 1]);
            trail_dpp<J + 2, J + 2>(a, lr, l);
        } else {
            trail_dpp<J + 1, J + 1>(a, lr, l);
        }
    }
}
template <int J, int V>
__device__ __forceinline__ void chain_dpp(double (&a)[16], double& my_inv, double& dn) {
    if constexpr (J < 16) {
        chain_dpp_step<J, V>(a, my_inv, dn);
        chain_dpp<J + 1, V>(a, my_inv, dn);
    }
}

template <int V>
__device__ __forceinline__ void chain(double (&a)[16], double& my_inv, double* lb) {
    const int r = threadIdx.x & 63;
    if constexpr (V == 6 || V == 7) {
        double dn = bcast(a[0], 0);
        chain_dpp<0, V>(a, my_inv, dn);
        return;
    }
    if constexpr (V == 3) {
        // the next column by v_readlane (on the chain); columns j + 2.. by an LDS broadcast of the multipliers
        // (lanes 0-15 store l, every lane reads l_k two at a time with uniform-address ds_read_b128): the
        // trailing updates cost one FMA per column instead of two v_readlane_b32 + one FMA
        double dn = bcast(a[0], 0);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const double d = dn;
            const double y = __builtin_amdgcn_rsq(d);
            const double e = __builtin_fma(-d * y, y, 1.0);
            const double l = __builtin_fma(0.5 * a[j] * y, e, a[j] * y);
            my_inv = (r == j) ? __builtin_fma(0.5 * y, e, y) : my_inv;
            a[j] = l;
            if (j < 15) {
                dn = bcast(__builtin_fma(-l, l, a[j + 1]), j + 1);
                a[j + 1] = __builtin_fma(-l, bcast(l, j + 1), a[j + 1]);
                if (j < 14) {
                    if (r < 16) lb[r] = l;
                    __builtin_amdgcn_wave_barrier();
                    int k = j + 2;
                    if (k & 1) {
                        a[k] = __builtin_fma(-l, lb[k], a[k]);
                        ++k;
                    }
#pragma unroll
                    for (; k < 16; k += 2) {
                        const double2 lk = *reinterpret_cast<const double2*>(lb + k);
                        a[k] = __builtin_fma(-l, lk.x, a[k]);
                        a[k + 1] = __builtin_fma(-l, lk.y, a[k + 1]);
                    }
                    __builtin_amdgcn_wave_barrier();
                }
            }
        }
    } else if constexpr (V == 0 || V == 2) {
        double dn = bcast(a[0], 0);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const double d = dn;
            const double y = __builtin_amdgcn_rsq(d);
            const double e = __builtin_fma(-d * y, y, 1.0);
            const double l = __builtin_fma(0.5 * a[j] * y, e, a[j] * y);
            my_inv = (r == j) ? __builtin_fma(0.5 * y, e, y) : my_inv;
            a[j] = l;
            if (j < 15) {
                dn = bcast(__builtin_fma(-l, l, a[j + 1]), j + 1);
                if constexpr (V == 0) {
#pragma unroll
                    for (int k = j + 1; k < 16; ++k) a[k] = __builtin_fma(-l, bcast(l, k), a[k]);
                } else {
                    a[j + 1] = __builtin_fma(-l, bcast(l, j + 1), a[j + 1]);
                }
            }
        }
    } else {
        // d_{j+1} = a_{j+1,j+1} - a_{j+1,j}^2 / d_j on lane j + 1: the chain is rcp + e + r' + dn + readlane
        double dn = bcast(a[0], 0);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const double d = dn;
            if (j < 15) {
                const double q = a[j] * a[j];  // lane j + 1: a_{j+1,j}^2 (current before pivot j)
                const double rc = __builtin_amdgcn_rcp(d);
                const double er = __builtin_fma(-d, rc, 1.0);
                const double rr = __builtin_fma(rc, er, rc);
                dn = bcast(__builtin_fma(-q, rr, a[j + 1]), j + 1);
            }
            const double y = __builtin_amdgcn_rsq(d);
            const double e = __builtin_fma(-d * y, y, 1.0);
            const double l = __builtin_fma(0.5 * a[j] * y, e, a[j] * y);
            my_inv = (r == j) ? __builtin_fma(0.5 * y, e, y) : my_inv;
            a[j] = l;
            if (j < 15) {
#pragma unroll
                for (int k = j + 1; k < 16; ++k) a[k] = __builtin_fma(-l, bcast(l, k), a[k]);
            }
        }
    }
}


template <int V>
__device__ __forceinline__ void chain_pipe(double (&a)[16], double& my_inv) {
    // variant 4 / 5: the trailing updates of pivot j - 1 (columns j + 1..15) issue inside pivot j's chain, which
    // does not read them (column j + 1 first: the next pivot needs it). Every element still receives its updates
    // in pivot order, so L is bitwise the kernel's. 5: the same code order without scheduling fences.
    const int r = threadIdx.x & 63;
    double dn = bcast(a[0], 0);
    double lp = 0.0;  // this lane's multiplier of the previous pivot
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const double d = dn;
        const double y = __builtin_amdgcn_rsq(d);
        if (j >= 1 && j + 1 < 16) a[j + 1] = __builtin_fma(-lp, bcast(lp, j + 1), a[j + 1]);
        if constexpr (V == 4) __builtin_amdgcn_sched_barrier(0);
        const double dy = d * y;
        constexpr int dummy = 0; (void)dummy;
        // the deferred trailing updates, split over the chain's dependent steps
        const int k0 = j + 2, n = 16 - k0 > 0 ? 16 - k0 : 0;
        const int c1 = k0 + n / 3, c2 = k0 + (2 * n) / 3;
        if (j >= 1)
#pragma unroll
            for (int k = k0; k < c1; ++k) a[k] = __builtin_fma(-lp, bcast(lp, k), a[k]);
        if constexpr (V == 4) __builtin_amdgcn_sched_barrier(0);
        const double e = __builtin_fma(-dy, y, 1.0);
        const double ay = a[j] * y;
        if (j >= 1)
#pragma unroll
            for (int k = c1; k < c2; ++k) a[k] = __builtin_fma(-lp, bcast(lp, k), a[k]);
        if constexpr (V == 4) __builtin_amdgcn_sched_barrier(0);
        const double l = __builtin_fma(0.5 * ay, e, ay);
        my_inv = (r == j) ? __builtin_fma(0.5 * y, e, y) : my_inv;
        a[j] = l;
        if (j >= 1)
#pragma unroll
            for (int k = c2; k < 16; ++k) a[k] = __builtin_fma(-lp, bcast(lp, k), a[k]);
        if constexpr (V == 4) __builtin_amdgcn_sched_barrier(0);
        if (j < 15) {
            dn = bcast(__builtin_fma(-l, l, a[j + 1]), j + 1);
            a[j + 1] = __builtin_fma(-l, bcast(l, j + 1), a[j + 1]);
        }
        lp = l;
    }
}

template <int V>
__global__ __launch_bounds__(64) void k_bench(const double* __restrict__ A, double* __restrict__ L,
                                              unsigned long long* __restrict__ t, int reps) {
    const int r = threadIdx.x;
    double a0[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) a0[c] = A[r * 16 + c];
    __shared__ __attribute__((aligned(16))) double lb[16];
    double a[16], my_inv = 0.0, sink = 0.0;
    const unsigned long long t0 = rt(), c0 = clk();
    for (int it = 0; it < reps; ++it) {
#pragma unroll
        for (int c = 0; c < 16; ++c) a[c] = a0[c] + sink * 1e-300;  // depends on the previous repetition
        if constexpr (V == 4 || V == 5) chain_pipe<V>(a, my_inv); else chain<V>(a, my_inv, lb);
        sink = bcast(a[15], 63);
    }
    const unsigned long long c1 = clk(), t1 = rt();
#pragma unroll
    for (int c = 0; c < 16; ++c) L[r * 16 + c] = a[c];
    if (r == 0) { t[0] = t1 - t0; t[1] = c1 - c0; }
}

int main() {
    // tall panel: rows 0..63 of column block 0 of an SPD 64 x 64 matrix A = B B^T + 64 I (rows 16..63: below)
    const int n = 64;
    std::vector<double> B(n * n), Af(n * n), A(64 * 16);
    unsigned long long s = 12345;
    for (auto& v : B) { s = s * 6364136223846793005ull + 1442695040888963407ull; v = ((s >> 11) * (1.0 / 9007199254740992.0)) - 0.5; }
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) {
            double acc = i == j ? 64.0 : 0.0;
            for (int k = 0; k < n; ++k) acc += B[i * n + k] * B[j * n + k];
            Af[i * n + j] = acc;
        }
    for (int r = 0; r < 64; ++r)
        for (int c = 0; c < 16; ++c) A[r * 16 + c] = Af[r * n + c];
    double *dA, *dL;
    unsigned long long* dt;
    (void)hipMalloc(&dA, 8 * A.size()); (void)hipMalloc(&dL, 8 * A.size()); (void)hipMalloc(&dt, 16);
    (void)hipMemcpy(dA, A.data(), 8 * A.size(), hipMemcpyHostToDevice);
    const int reps = 2000;
    const char* names[8] = {"rsq chain (kernel)", "rcp next-pivot chain", "chain only (lower bound)",
                            "LDS-broadcast trailing", "deferred trailing, fenced", "deferred trailing, unfenced",
                            "DPP64 trailing (j+2..)", "DPP64 trailing (j+1..)"};
    for (int round = 0; round < 2; ++round)
        for (int v = 0; v < 8; ++v) {
            if (v == 0) hipLaunchKernelGGL(k_bench<0>, dim3(1), dim3(64), 0, 0, dA, dL, dt, reps);
            if (v == 1) hipLaunchKernelGGL(k_bench<1>, dim3(1), dim3(64), 0, 0, dA, dL, dt, reps);
            if (v == 2) hipLaunchKernelGGL(k_bench<2>, dim3(1), dim3(64), 0, 0, dA, dL, dt, reps);
            if (v == 3) hipLaunchKernelGGL(k_bench<3>, dim3(1), dim3(64), 0, 0, dA, dL, dt, reps);
            if (v == 4) hipLaunchKernelGGL(k_bench<4>, dim3(1), dim3(64), 0, 0, dA, dL, dt, reps);
            if (v == 5) hipLaunchKernelGGL(k_bench<5>, dim3(1), dim3(64), 0, 0, dA, dL, dt, reps);
            if (v == 6) hipLaunchKernelGGL(k_bench<6>, dim3(1), dim3(64), 0, 0, dA, dL, dt, reps);
            if (v == 7) hipLaunchKernelGGL(k_bench<7>, dim3(1), dim3(64), 0, 0, dA, dL, dt, reps);
            unsigned long long t[2];
            std::vector<double> L(64 * 16);
            (void)hipMemcpy(t, dt, 16, hipMemcpyDeviceToHost);
            (void)hipMemcpy(L.data(), dL, 8 * L.size(), hipMemcpyDeviceToHost);
            // residual of the leading 16 x 16 block and the panel rows: (L L^T)[r][c] vs A[r][c], c <= min(r, 15)
            double err = 0.0;
            for (int r = 0; r < 64; ++r)
                for (int c = 0; c <= (r < 16 ? r : 15); ++c) {
                    double acc = 0.0;
                    for (int k = 0; k <= c; ++k) acc += L[r * 16 + k] * L[c * 16 + k];
                    err = std::fmax(err, std::fabs(acc - A[r * 16 + c]) / std::fabs(A[c * 16 + c]));
                }
            const double ns = t[0] * 10.0 / (reps * 16.0);  // s_memrealtime: 100 MHz
            printf("round %d  %-26s %7.1f ns/pivot  %7.1f clk/pivot  rel.err %.2e\n", round, names[v], ns,
                   (double)t[1] / (reps * 16.0), v == 2 ? 0.0 : err);
        }
    return 0;
}
