// ba_bcr.hip — block cyclic reduction (BCR) solver for the reduced camera system.
//
// With the active cameras grouped in blocks of G = BCR_CAMS consecutive cameras and the
// camera co-visibility band < G, the camera part A of S is exactly block-tridiagonal
// (64x64 blocks, 6G = 60 dofs + 4 identity pad rows); the intrinsics rows form a dense
// border B (6nac x 4) and corner C (4x4):
//     S = [A  B; B^T C],  A y_a + B y_k = b_a,  B^T y_a + C y_k = b_k.
// We solve A [u | V] = [b_a | B] (5 right-hand sides) by odd-even block elimination.
// At level m (stride s = 2^m) every block i with i % 2s == s is eliminated in parallel,
// one workgroup each (k_bcr_elim):
//   - its diagonal block D_i, rhs R_i and couplings A[i][i-s], A[i][i+s] are assembled:
//     level 0 reads them straight from S; deeper levels subtract the Schur contributions
//     that blocks eliminated at levels l < m left for it (UR of i-2^l, UL of i+2^l) and
//     take the fill couplings F of i -+ 2^(m-1);
//   - Cf = chol(D_i) (LDS, MFMA trailing updates), [XL | XR | x] = Cf^-1 [A_l | A_r | R];
//   - it emits its own contributions for the survivors, all from LDS operands:
//       UL = XL^T XL, rL = XL^T x  -> left survivor i-s
//       UR = XR^T XR, rR = XR^T x  -> right survivor i+s
//       F  = -XR^T XL              -> new coupling A[i+s][i-s]
//     Survivors sum these in a fixed order when they are eliminated (deterministic, no
//     atomics, no separate update pass).
// Block 0 is factored last (the root); back-substitution runs the levels in reverse
// (k_bcr_back: y_i = Cf^-T (x_i - XL y_{i-s} - XR y_{i+s})). Finally the 4x4 border system
// C' = C - B^T V, b' = b_k - B^T u gives y_k and y_a = u - V y_k (k_bcr_border).
// Sequential depth: (levels + 1) block factorizations instead of the n = 6*nac + 4 pivots
// of the band Cholesky; exact elimination, only the rounding order differs.
#include <hip/hip_runtime.h>

#include "ba_device.h"
#include "ba_kernels.h"

namespace miba {

static constexpr int TPB_B = 512;        // 8 waves per block workgroup
static constexpr int NWB = TPB_B / 64;
static constexpr int BB = 64;            // block size (dofs)
static constexpr int BLD = 66;           // LDS row stride of 64x64 blocks
static constexpr int RC = 8;             // rhs columns: u, V(4), 3 pad
static constexpr int LDX = 2 * BB + RC;  // [XL | XR | x]
static constexpr int G_DOF = 6 * BCR_CAMS;
static constexpr int BSZ = BB * BB;
typedef double d4b __attribute__((ext_vector_type(4)));

// Diagnostic phase stamps (MIBA_BCR_STAMPS=1 launches the STAMP=true variants).
__device__ __forceinline__ unsigned long long bcr_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define BCR_STAMP(k)                                                             \
    do {                                                                         \
        if constexpr (STAMP) {                                                   \
            __syncthreads();                                                     \
            if (threadIdx.x == 0) stamps[(m * 64 + blockIdx.x % 64) * 8 + (k)] = bcr_stamp(); \
        }                                                                        \
    } while (0)

__device__ __forceinline__ double bcast_b(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double rsqrt_nr_b(double x) {
    double y = __builtin_amdgcn_rsq(x);
    y = y * (1.5 - 0.5 * x * y * y);
    y = y * (1.5 - 0.5 * x * y * y);
    return y;
}

// 16x16 Cholesky of the tile at T (LDS, stride ld) by one wave; rdiag[16] = 1/L_jj.
__device__ __forceinline__ void potrf16_tile(double* T, int ld, double* rdiag, int lane, bool& bad) {
    const int r = lane & 15;
    double a[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = T[r * ld + j];
    double my_inv = 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        double djj = bcast_b(a[j], j);
        const bool ok = (djj > 0.0) && (djj < INFINITY);
        bad = bad || !ok;
        djj = ok ? djj : 1.0;
        const double inv = rsqrt_nr_b(djj);
        const double lrj = a[j] * inv;
        a[j] = lrj;
        my_inv = (r == j) ? inv : my_inv;
#pragma unroll
        for (int k = j + 1; k < 16; ++k) a[k] -= lrj * bcast_b(lrj, k);
    }
    if (lane < 16) {
#pragma unroll
        for (int j = 0; j < 16; ++j) T[r * ld + j] = (j <= r) ? a[j] : 0.0;
        rdiag[r] = my_inv;
    }
}

// In-LDS Cholesky of a 64x64 SPD block (lower triangle of T, stride BLD), whole workgroup.
__device__ void potrf64(double* T, double* rdiag64, bool& bad) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rr = lane & 15, kk = lane >> 4;
    for (int kb = 0; kb < 4; ++kb) {
        double* Tkk = T + (16 * kb) * BLD + 16 * kb;
        if (wave == 0) potrf16_tile(Tkk, BLD, rdiag64 + 16 * kb, lane, bad);
        __syncthreads();
        const int nrow = 64 - 16 * (kb + 1);
        if (tid < nrow) {
            const int r = 16 * (kb + 1) + tid;
            double x[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) x[j] = T[r * BLD + 16 * kb + j];
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                x[m] *= rdiag64[16 * kb + m];
#pragma unroll
                for (int j = m + 1; j < 16; ++j) x[j] -= x[m] * Tkk[j * BLD + m];
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) T[r * BLD + 16 * kb + j] = x[j];
        }
        __syncthreads();
        const int nt = 3 - kb;
        const int npairs = nt * (nt + 1) / 2;
        for (int t = wave; t < npairs; t += NWB) {
            int p = 0, rem = t;
            while (rem > p) { rem -= p + 1; ++p; }
            const int i = kb + 1 + p, j = kb + 1 + rem;
            const double* Li = T + (16 * i) * BLD + 16 * kb;
            const double* Lj = T + (16 * j) * BLD + 16 * kb;
            d4b acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Li[rr * BLD + 4 * s4 + kk], Lj[rr * BLD + 4 * s4 + kk], acc, 0, 0, 0);
            double* C = T + (16 * i) * BLD + 16 * j;
#pragma unroll
            for (int g = 0; g < 4; ++g) C[(kk + 4 * g) * BLD + rr] -= acc[g];
        }
        __syncthreads();
    }
}

// X <- L^-1 X, L 64x64 lower (LDS, stride BLD), X 64 x ncol (LDS, stride ldx).
__device__ void trsm_lower64(const double* L, const double* rdiag64, double* X, int ldx, int ncol) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rr = lane & 15, kk = lane >> 4;
    for (int kb = 0; kb < 4; ++kb) {
        const double* Lkk = L + (16 * kb) * BLD + 16 * kb;
        for (int c = tid; c < ncol; c += TPB_B) {
            double x[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) x[j] = X[(16 * kb + j) * ldx + c];
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                x[m] *= rdiag64[16 * kb + m];
#pragma unroll
                for (int j = m + 1; j < 16; ++j) x[j] -= Lkk[j * BLD + m] * x[m];
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) X[(16 * kb + j) * ldx + c] = x[j];
        }
        __syncthreads();
        const int ncb = (ncol + 15) / 16;
        const int ntile = (3 - kb) * ncb;
        for (int t = wave; t < ntile; t += NWB) {
            const int i = kb + 1 + t / ncb, cb = t % ncb;
            const double* A = L + (16 * i) * BLD + 16 * kb;
            d4b acc = {0.0, 0.0, 0.0, 0.0};
            const int col = 16 * cb + rr;
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const double bv = (col < ncol) ? X[(16 * kb + 4 * s4 + kk) * ldx + col] : 0.0;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[rr * BLD + 4 * s4 + kk], bv, acc, 0, 0, 0);
            }
            if (col < ncol)
#pragma unroll
                for (int g = 0; g < 4; ++g) X[(16 * i + kk + 4 * g) * ldx + col] -= acc[g];
        }
        __syncthreads();
    }
}

// X <- L^-T X (backward), L 64x64 lower in LDS, X (64 x ncol) in LDS.
__device__ void trsm_lower64_t(const double* L, const double* rdiag64, double* X, int ldx, int ncol) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rr = lane & 15, kk = lane >> 4;
    for (int kb = 3; kb >= 0; --kb) {
        const double* Lkk = L + (16 * kb) * BLD + 16 * kb;
        for (int c = tid; c < ncol; c += TPB_B) {
            double x[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) x[j] = X[(16 * kb + j) * ldx + c];
#pragma unroll
            for (int m = 15; m >= 0; --m) {
                x[m] *= rdiag64[16 * kb + m];
#pragma unroll
                for (int j = 0; j < m; ++j) x[j] -= Lkk[m * BLD + j] * x[m];  // (L^T)[j][m] = L[m][j]
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) X[(16 * kb + j) * ldx + c] = x[j];
        }
        __syncthreads();
        const int ncb = (ncol + 15) / 16;
        const int ntile = kb * ncb;
        for (int t = wave; t < ntile; t += NWB) {
            const int i = t / ncb, cb = t % ncb;
            const double* A = L + (16 * kb) * BLD + 16 * i;  // L[kb][i]; operand (L^T)[r][k] = L[kb][i][k][r]
            d4b acc = {0.0, 0.0, 0.0, 0.0};
            const int col = 16 * cb + rr;
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const double av = A[(4 * s4 + kk) * BLD + rr];
                const double bv = (col < ncol) ? X[(16 * kb + 4 * s4 + kk) * ldx + col] : 0.0;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
            }
            if (col < ncol)
#pragma unroll
                for (int g = 0; g < 4; ++g) X[(16 * i + kk + 4 * g) * ldx + col] -= acc[g];
        }
        __syncthreads();
    }
}

// 64x64 block copy global -> LDS with every load issued before any LDS store
// (one round trip per block instead of one per element row).
template <bool TRANS>
__device__ __forceinline__ void stage64(double* dst, int ldd, const double* __restrict__ src) {
    double v[BSZ / TPB_B];
#pragma unroll
    for (int q = 0; q < BSZ / TPB_B; ++q) v[q] = src[threadIdx.x + TPB_B * q];
#pragma unroll
    for (int q = 0; q < BSZ / TPB_B; ++q) {
        const int e = threadIdx.x + TPB_B * q, r = e >> 6, c = e & 63;
        if (TRANS) dst[c * ldd + r] = v[q];
        else dst[r * ldd + c] = v[q];
    }
}
__device__ __forceinline__ void zero64(double* dst, int ldd) {
#pragma unroll
    for (int q = 0; q < BSZ / TPB_B; ++q) {
        const int e = threadIdx.x + TPB_B * q;
        dst[(e >> 6) * ldd + (e & 63)] = 0.0;
    }
}
__device__ __forceinline__ void store64(double* __restrict__ dst, const double* src, int lds_) {
#pragma unroll
    for (int q = 0; q < BSZ / TPB_B; ++q) {
        const int e = threadIdx.x + TPB_B * q;
        dst[e] = src[(e >> 6) * lds_ + (e & 63)];
    }
}

struct ElimLds {
    double T[BB * BLD];   // D_i -> Cf
    double X[BB * LDX];   // [A_l | A_r | R] -> [XL | XR | x]
    double rdiag[BB];
};

// ---- level-m elimination of the blocks i = s + 2s*b (s = 2^m); m == levels: root (block 0).
template <bool STAMP>
__global__ __launch_bounds__(TPB_B) void k_bcr_elim(const LmState* __restrict__ st, DevProblem P,
                                                    const double* __restrict__ S, const double* __restrict__ rhs,
                                                    BcrWork Bw, int m, int* __restrict__ flag,
                                                    unsigned long long* __restrict__ stamps) {
    if (st->done) return;
    BCR_STAMP(0);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    ElimLds& L = *reinterpret_cast<ElimLds*>(smem);
    const int nblk = Bw.nblk;
    const bool root = m >= Bw.levels;
    const int s = 1 << m;
    const int i = root ? 0 : s + 2 * s * (int)blockIdx.x;
    if (i >= nblk) return;
    const bool has_r = !root && i + s < nblk;
    const size_t ld = P.npad;
    const int nd = 6 * P.nac;
    const int b0 = i * G_DOF;
    const int tid = threadIdx.x;

    // D_i: lower triangle of S (identity on pad / missing dofs) minus pending contributions
    {
        double v[BSZ / TPB_B];
#pragma unroll
        for (int q = 0; q < BSZ / TPB_B; ++q) {
            const int e = tid + TPB_B * q, r = e >> 6, c = e & 63;
            const int gr = b0 + r;
            const bool ok = c <= r && r < G_DOF && gr < nd;
            v[q] = ok ? S[(size_t)gr * ld + b0 + c] : (r == c ? 1.0 : 0.0);
        }
        for (int l = 0; l < m; ++l) {
            const int a = i - (1 << l), b = i + (1 << l);
            const double* pa = Bw.UR + (size_t)(a >= 0 ? a : 0) * BSZ;
            const double* pb = Bw.UL + (size_t)(b < nblk ? b : 0) * BSZ;
            double ua[BSZ / TPB_B], ub[BSZ / TPB_B];
#pragma unroll
            for (int q = 0; q < BSZ / TPB_B; ++q) {
                ua[q] = a >= 0 ? pa[tid + TPB_B * q] : 0.0;
                ub[q] = b < nblk ? pb[tid + TPB_B * q] : 0.0;
            }
#pragma unroll
            for (int q = 0; q < BSZ / TPB_B; ++q) v[q] = (v[q] - ua[q]) - ub[q];
        }
#pragma unroll
        for (int q = 0; q < BSZ / TPB_B; ++q) {
            const int e = tid + TPB_B * q;
            L.T[(e >> 6) * BLD + (e & 63)] = v[q];
        }
    }
    // R_i = [b_a | B] rows of block i (one element per thread)
    {
        const int r = tid >> 3, c = tid & 7, gr = b0 + r;
        double v = 0.0;
        if (r < G_DOF && gr < nd) {
            if (c == 0) v = rhs[gr];
            else if (c <= 4) v = S[(size_t)(P.kb + c - 1) * ld + gr];
        }
        for (int l = 0; l < m; ++l) {
            const int a = i - (1 << l), b = i + (1 << l);
            const double va = a >= 0 ? Bw.rR[(size_t)a * BB * RC + tid] : 0.0;
            const double vb = b < nblk ? Bw.rL[(size_t)b * BB * RC + tid] : 0.0;
            v = (v - va) - vb;
        }
        L.X[r * LDX + 2 * BB + c] = v;
    }
    if (!root) {
        // left coupling A[i][i-s]
        if (m == 0) {
#pragma unroll
            for (int q = 0; q < BSZ / TPB_B; ++q) {
                const int e = tid + TPB_B * q, r = e >> 6, c = e & 63;
                const int gr = b0 + r;
                const bool ok = r < G_DOF && gr < nd && c < G_DOF;
                L.X[r * LDX + c] = ok ? S[(size_t)gr * ld + b0 - G_DOF + c] : 0.0;
            }
        } else {
            stage64<false>(L.X, LDX, Bw.F + (size_t)(i - s / 2) * BSZ);
        }
        // right coupling A[i][i+s] = A[i+s][i]^T
        if (!has_r) {
            zero64(L.X + BB, LDX);
        } else if (m == 0) {
            const int b1 = b0 + G_DOF;
#pragma unroll
            for (int q = 0; q < BSZ / TPB_B; ++q) {
                const int e = tid + TPB_B * q, r = e >> 6, c = e & 63;
                const bool ok = r < G_DOF && b1 + r < nd && c < G_DOF;
                L.X[c * LDX + BB + r] = ok ? S[(size_t)(b1 + r) * ld + b0 + c] : 0.0;
            }
        } else {
            stage64<true>(L.X + BB, LDX, Bw.F + (size_t)(i + s / 2) * BSZ);
        }
    }
    __syncthreads();
    BCR_STAMP(1);
    bool bad = false;
    potrf64(L.T, L.rdiag, bad);
    if (bad) *flag = 1;
    BCR_STAMP(2);
    if (root) {
        trsm_lower64(L.T, L.rdiag, L.X + 2 * BB, LDX, RC);
        trsm_lower64_t(L.T, L.rdiag, L.X + 2 * BB, LDX, RC);
        const int r = tid >> 3, c = tid & 7;
        Bw.Y[tid] = L.X[r * LDX + 2 * BB + c];
        return;
    }
    trsm_lower64(L.T, L.rdiag, L.X, LDX, LDX);
    BCR_STAMP(3);
    // factor and solved blocks for the back-substitution
    store64(Bw.Cf + (size_t)i * BSZ, L.T, BLD);
    store64(Bw.XL + (size_t)i * BSZ, L.X, LDX);
    if (has_r) store64(Bw.XR + (size_t)i * BSZ, L.X + BB, LDX);
    {
        const int r = tid >> 3, c = tid & 7;
        Bw.x[(size_t)i * BB * RC + tid] = L.X[r * LDX + 2 * BB + c];
    }
    if (tid < BB) Bw.rd[(size_t)i * BB + tid] = L.rdiag[tid];
    BCR_STAMP(4);
    // Schur contributions for the survivors (operands in LDS):
    //   t in [0,10) UL lower tiles, [10,20) UR lower tiles, [20,36) F, [36,40) rL, [40,44) rR
    const int lane = tid & 63, wave = tid >> 6, rr = lane & 15, kk = lane >> 4;
    for (int t = wave; t < 44; t += NWB) {
        int ib, cb, aoff, boff;
        double* dst;
        int ldd = BB;
        double sign = 1.0;
        bool rhs_tile = false;
        if (t < 20) {
            if (t >= 10 && !has_r) continue;
            int p = 0, rem = t % 10;
            while (rem > p) { rem -= p + 1; ++p; }
            ib = p; cb = rem;
            aoff = boff = (t < 10) ? 0 : BB;
            dst = (t < 10 ? Bw.UL : Bw.UR) + (size_t)i * BSZ;
        } else if (t < 36) {
            if (!has_r) continue;
            ib = (t - 20) >> 2; cb = (t - 20) & 3;
            aoff = BB; boff = 0; sign = -1.0;
            dst = Bw.F + (size_t)i * BSZ;
        } else {
            if (t >= 40 && !has_r) continue;
            ib = (t - 36) & 3; cb = 0;
            aoff = (t < 40) ? 0 : BB; boff = 2 * BB;
            dst = (t < 40 ? Bw.rL : Bw.rR) + (size_t)i * BB * RC;
            ldd = RC;
            rhs_tile = true;
        }
        const bool bcol_ok = !rhs_tile || rr < RC;
        d4b acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
        for (int s4 = 0; s4 < 16; ++s4) {
            const double* row = L.X + (4 * s4 + kk) * LDX;
            const double bv = bcol_ok ? row[boff + 16 * cb + rr] : 0.0;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(row[aoff + 16 * ib + rr], bv, acc, 0, 0, 0);
        }
        if (bcol_ok)
#pragma unroll
            for (int g = 0; g < 4; ++g) dst[(size_t)(16 * ib + kk + 4 * g) * ldd + 16 * cb + rr] = sign * acc[g];
    }
    BCR_STAMP(5);
}

struct BackLds {
    double T[BB * BLD];   // Cf_i
    double U1[BB * BLD];  // XL_i
    double U2[BB * BLD];  // XR_i
    double t[BB * RC], yl[BB * RC], yr[BB * RC];
    double rdiag[BB];
};

// ---- back-substitution for the blocks eliminated at level m:
// y_i = Cf_i^-T (x_i - XL_i y_{i-s} - XR_i y_{i+s})
template <bool STAMP>
__global__ __launch_bounds__(TPB_B) void k_bcr_back(const LmState* __restrict__ st, BcrWork Bw, int m,
                                                    unsigned long long* __restrict__ stamps) {
    if (st->done) return;
    BCR_STAMP(6);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    BackLds& L = *reinterpret_cast<BackLds*>(smem);
    const int s = 1 << m;
    const int i = s + 2 * s * (int)blockIdx.x;
    const int nblk = Bw.nblk;
    if (i >= nblk) return;
    const bool has_r = i + s < nblk;
    const int tid = threadIdx.x;
    stage64<false>(L.T, BLD, Bw.Cf + (size_t)i * BSZ);
    stage64<false>(L.U1, BLD, Bw.XL + (size_t)i * BSZ);
    if (has_r) stage64<false>(L.U2, BLD, Bw.XR + (size_t)i * BSZ);
    {
        const double xv = Bw.x[(size_t)i * BB * RC + tid];
        const double yl = Bw.Y[(size_t)(i - s) * BB * RC + tid];
        const double yr = has_r ? Bw.Y[(size_t)(i + s) * BB * RC + tid] : 0.0;
        L.t[tid] = xv;
        L.yl[tid] = yl;
        L.yr[tid] = yr;
        if (tid < BB) L.rdiag[tid] = Bw.rd[(size_t)i * BB + tid];
    }
    __syncthreads();
    const int lane = tid & 63, wave = tid >> 6, rr = lane & 15, kk = lane >> 4;
    if (wave < 4) {
        d4b acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
        for (int s4 = 0; s4 < 16; ++s4) {
            const double bv = rr < RC ? L.yl[(4 * s4 + kk) * RC + rr] : 0.0;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(L.U1[(16 * wave + rr) * BLD + 4 * s4 + kk], bv, acc, 0, 0, 0);
        }
        if (has_r) {
#pragma unroll 4
            for (int s4 = 0; s4 < 16; ++s4) {
                const double bv = rr < RC ? L.yr[(4 * s4 + kk) * RC + rr] : 0.0;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(L.U2[(16 * wave + rr) * BLD + 4 * s4 + kk], bv, acc, 0, 0, 0);
            }
        }
        if (rr < RC)
#pragma unroll
            for (int g = 0; g < 4; ++g) L.t[(16 * wave + kk + 4 * g) * RC + rr] -= acc[g];
    }
    __syncthreads();
    BCR_STAMP(7);
    trsm_lower64_t(L.T, L.rdiag, L.t, RC, RC);
    Bw.Y[(size_t)i * BB * RC + tid] = L.t[tid];
    if constexpr (STAMP) {
        __syncthreads();
        if (threadIdx.x == 0) stamps[(m * 64 + blockIdx.x % 64) * 8 + 6] = bcr_stamp() - stamps[(m * 64 + blockIdx.x % 64) * 8 + 6];
        if (threadIdx.x == 0) stamps[(m * 64 + blockIdx.x % 64) * 8 + 7] = bcr_stamp() - stamps[(m * 64 + blockIdx.x % 64) * 8 + 7];
    }
}

// ---- border: C' = S_kk - B^T V, b' = b_k - B^T u ; y_k = C'^-1 b' ; y_a = u - V y_k -> rhs (dense)
static constexpr int TPB_BD = 256;
__global__ __launch_bounds__(TPB_BD) void k_bcr_border(const LmState* __restrict__ st, DevProblem P,
                                                      const double* __restrict__ S, double* __restrict__ rhs,
                                                      BcrWork Bw, int* __restrict__ flag) {
    if (st->done) return;
    __shared__ double red[TPB_BD][20];
    __shared__ double yk[4];
    const size_t ld = P.npad;
    const int nd = 6 * P.nac;
    const int kb = P.kb;
    double acc[20];
#pragma unroll
    for (int q = 0; q < 20; ++q) acc[q] = 0.0;
    for (int g = threadIdx.x; g < nd; g += TPB_BD) {
        const int blk = g / G_DOF, r = g % G_DOF;
        const double* y = Bw.Y + ((size_t)blk * BB + r) * RC;
        double bm[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) bm[m] = S[(size_t)(kb + m) * ld + g];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
#pragma unroll
            for (int l = 0; l < 4; ++l) acc[m * 4 + l] += bm[m] * y[1 + l];  // (B^T V)[m][l]
            acc[16 + m] += bm[m] * y[0];                                    // (B^T u)[m]
        }
    }
#pragma unroll
    for (int q = 0; q < 20; ++q) red[threadIdx.x][q] = acc[q];
    __syncthreads();
    for (int w = TPB_BD / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
#pragma unroll
            for (int q = 0; q < 20; ++q) red[threadIdx.x][q] += red[threadIdx.x + w][q];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        double Cm[16], bp[4];
        for (int m = 0; m < 4; ++m) {
            for (int l = 0; l < 4; ++l) {
                const double s_ml = (m >= l) ? S[(size_t)(kb + m) * ld + kb + l] : S[(size_t)(kb + l) * ld + kb + m];
                Cm[m * 4 + l] = s_ml - red[0][m * 4 + l];
            }
            bp[m] = rhs[kb + m] - red[0][16 + m];
        }
        // 4x4 Cholesky solve
        bool bad = false;
        double Lm[16] = {0};
        for (int j = 0; j < 4; ++j) {
            double d = Cm[j * 4 + j];
            for (int k = 0; k < j; ++k) d -= Lm[j * 4 + k] * Lm[j * 4 + k];
            if (!(d > 0.0)) { bad = true; d = 1.0; }
            Lm[j * 4 + j] = sqrt(d);
            for (int i = j + 1; i < 4; ++i) {
                double v = Cm[i * 4 + j];
                for (int k = 0; k < j; ++k) v -= Lm[i * 4 + k] * Lm[j * 4 + k];
                Lm[i * 4 + j] = v / Lm[j * 4 + j];
            }
        }
        double z[4];
        for (int i = 0; i < 4; ++i) {
            double v = bp[i];
            for (int k = 0; k < i; ++k) v -= Lm[i * 4 + k] * z[k];
            z[i] = v / Lm[i * 4 + i];
        }
        for (int i = 3; i >= 0; --i) {
            double v = z[i];
            for (int k = i + 1; k < 4; ++k) v -= Lm[k * 4 + i] * z[k];
            z[i] = v / Lm[i * 4 + i];
        }
        for (int m = 0; m < 4; ++m) yk[m] = z[m];
        if (bad) *flag = 1;
    }
    __syncthreads();
    for (int g = threadIdx.x; g < nd; g += TPB_BD) {
        const int blk = g / G_DOF, r = g % G_DOF;
        const double* y = Bw.Y + ((size_t)blk * BB + r) * RC;
        rhs[g] = y[0] - (y[1] * yk[0] + y[2] * yk[1] + y[3] * yk[2] + y[4] * yk[3]);
    }
    if (threadIdx.x < 4) rhs[kb + threadIdx.x] = yk[threadIdx.x];
}

#define CKB(x)                            \
    do {                                  \
        hipError_t e_ = (x);              \
        if (e_ != hipSuccess) return e_;  \
    } while (0)

template <bool STAMP>
static hipError_t launch_bcr_t(const DevProblem& P, DevWork& W, const BcrWork& Bw, hipStream_t s,
                               unsigned long long* stamps) {
    const int nblk = Bw.nblk;
    for (int m = 0; m < Bw.levels; ++m) {
        const int st = 1 << m;
        const int nel = (nblk - st + 2 * st - 1) / (2 * st);
        hipLaunchKernelGGL(k_bcr_elim<STAMP>, dim3(nel), dim3(TPB_B), sizeof(ElimLds), s, W.st, P, W.S, W.rhs, Bw, m,
                           W.chol_flag, stamps);
        CKB(hipGetLastError());
    }
    hipLaunchKernelGGL(k_bcr_elim<STAMP>, dim3(1), dim3(TPB_B), sizeof(ElimLds), s, W.st, P, W.S, W.rhs, Bw, Bw.levels,
                       W.chol_flag, stamps);
    CKB(hipGetLastError());
    for (int m = Bw.levels - 1; m >= 0; --m) {
        const int st = 1 << m;
        const int nel = (nblk - st + 2 * st - 1) / (2 * st);
        hipLaunchKernelGGL(k_bcr_back<STAMP>, dim3(nel), dim3(TPB_B), sizeof(BackLds), s, W.st, Bw, m, stamps);
        CKB(hipGetLastError());
    }
    hipLaunchKernelGGL(k_bcr_border, dim3(1), dim3(TPB_BD), 0, s, W.st, P, W.S, W.rhs, Bw, W.chol_flag);
    CKB(hipGetLastError());
    return hipSuccess;
}

hipError_t launch_bcr(const DevProblem& P, DevWork& W, const BcrWork& Bw, hipStream_t s, Prof* pf) {
    static bool attr = false;
    static unsigned long long* stamps = nullptr;
    if (!attr) {
        const int le = (int)sizeof(ElimLds), lb = (int)sizeof(BackLds);
        CKB(hipFuncSetAttribute((const void*)k_bcr_elim<false>, hipFuncAttributeMaxDynamicSharedMemorySize, le));
        CKB(hipFuncSetAttribute((const void*)k_bcr_elim<true>, hipFuncAttributeMaxDynamicSharedMemorySize, le));
        CKB(hipFuncSetAttribute((const void*)k_bcr_back<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lb));
        CKB(hipFuncSetAttribute((const void*)k_bcr_back<true>, hipFuncAttributeMaxDynamicSharedMemorySize, lb));
        const char* e = getenv("MIBA_BCR_STAMPS");
        if (e && e[0] == '1') CKB(hipMalloc(&stamps, sizeof(unsigned long long) * 16 * 64 * 8));
        attr = true;
    }
    if (pf) pf->begin(K_CHOL, s);
    if (stamps) {
        CKB(hipMemsetAsync(stamps, 0, sizeof(unsigned long long) * 16 * 64 * 8, s));
        CKB(launch_bcr_t<true>(P, W, Bw, s, stamps));
        static unsigned long long h[16 * 64 * 8];
        CKB(hipMemcpyAsync(h, stamps, sizeof(h), hipMemcpyDeviceToHost, s));
        CKB(hipStreamSynchronize(s));
        for (int m = 0; m <= Bw.levels; ++m) {
            const unsigned long long* q = h + (size_t)m * 64 * 8;
            if (!q[0]) continue;
            fprintf(stderr, "bcr level %d blk0 cycles: load %llu potrf %llu trsm %llu store %llu contrib %llu | back %llu (trsm %llu)\n", m,
                    q[1] - q[0], q[2] - q[1], q[3] - q[2], q[4] - q[3], q[5] ? q[5] - q[4] : 0ull, q[6], q[7]);
        }
    } else {
        CKB(launch_bcr_t<false>(P, W, Bw, s, nullptr));
    }
    if (pf) pf->end(s);
    return hipSuccess;
}

}  // namespace miba
