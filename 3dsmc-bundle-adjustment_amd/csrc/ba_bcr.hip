// ba_bcr.hip — block cyclic reduction (BCR) solver for the reduced camera system.
//
// With the active cameras grouped in blocks of G = BCR_CAMS consecutive cameras and the
// camera co-visibility band < G, the camera part A of S is exactly block-tridiagonal
// (64x64 blocks, 6G = 60 dofs + 4 identity pad rows); the intrinsics rows form a dense
// border B (6nac x 4) and corner C (4x4):
//     S = [A  B; B^T C],  A y_a + B y_k = b_a,  B^T y_a + C y_k = b_k.
// We solve A [u | V] = [b_a | B] (5 right-hand sides) by odd-even block elimination.
// Level m (stride s = 2^m) eliminates every block i with i % 2s == s:
//   k_bcr_elim  (critical path, one workgroup per block) assembles D_i, R_i and the
//               couplings A[i][i-s], A[i][i+s] in ONE load round, then factors
//               Cf = chol(D_i) fused with the forward solve X = Cf^-1 [A_l | A_r | R_i].
//               Level 0 reads S directly; level m >= 1 subtracts the level m-1 Schur
//               contributions of its neighbours i -+ s/2 from Dacc_i, which already holds
//               all earlier levels: extra "accumulator" workgroups of the same launch fold
//               level m-1 into Dacc_j of every block j that survives level m.
//   k_bcr_contrib (11 workgroups per eliminated block, MFMA operands straight from L2)
//               emits UL = XL^T XL, UR = XR^T XR, F = -XR^T XL, rL = XL^T x, rR = XR^T x.
// Block 0 is the root (factor + solve). Back-substitution runs the levels in reverse
// (k_bcr_back: y_i = Cf^-T (x_i - XL y_{i-s} - XR y_{i+s}), plus the border partial
// B_i^T y_i). k_bcr_border sums the partials in block order, solves the 4x4 system
// C' y_k = b' (C' = C - B^T V, b' = b_k - B^T u) and writes y_a = u - V y_k.
// All sums run in a fixed order (deterministic, no atomics). Sequential depth:
// (levels + 1) block factorizations instead of the n = 6*nac + 4 pivots of the band
// Cholesky; exact elimination, only the rounding order differs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ba_device.h"
#include "ba_kernels.h"
#include "ba_solve_util.h"

namespace miba {

static constexpr int TPB_E = 512;        // elimination workgroup: 8 waves
static constexpr int NWE = TPB_E / 64;
static constexpr int TPB_C = 256;        // contrib / back workgroups: 4 waves
static constexpr int BB = 64;            // block size (dofs)
static constexpr int BLD = 66;           // LDS row stride of 64x64 blocks
static constexpr int RC = 8;             // rhs columns: u, V(4), 3 pad
static constexpr int XW = BCR_XW;        // [XL | XR | x] row stride (global and LDS)
static constexpr int XC = 2 * BB + RC;   // [XL | XR | x] columns
static constexpr int G_DOF = 6 * BCR_CAMS;
static constexpr int BSZ = BB * BB;
static constexpr int XSZ = BB * XW;
static constexpr int RSZ = BB * RC;
static constexpr int NCONTRIB_WG = 11;  // 44 contribution tiles / 4 waves
typedef double d4b __attribute__((ext_vector_type(4)));


// Diagnostic phase stamps (MIBA_BCR_STAMPS=1 launches the STAMP=true variants).
__device__ __forceinline__ unsigned long long bcr_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define BCR_STAMP(slot, k)                                                                       \
    do {                                                                                         \
        if constexpr (STAMP) {                                                                   \
            __syncthreads();                                                                     \
            if (threadIdx.x == 0 && blockIdx.x == 0) stamps[(slot) * 8 + (k)] = bcr_stamp();     \
        }                                                                                        \
    } while (0)

// 1/sqrt(x): v_rsq_f64 (~2^-24) + one Newton step in FMA form (rel. error ~4e-15,
// measured by tools/rsq_f64_check.hip) — three dependent f64 ops on the pivot path.
__device__ __forceinline__ double rsqrt_1nr(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    const double e = __builtin_fma(-x * y, y, 1.0);
    return __builtin_fma(0.5 * y, e, y);
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
        const double inv = rsqrt_1nr(djj);
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

// Forward substitution of a 16-vector against the 16x16 lower tile Lkk:
// v[m] = (v[m] - sum_{j<m} L[m][j] v[j]) / L[m][m]. Serves both panel rows
// (l = a L^-T) and right-hand-side columns (z = L^-1 b).
__device__ __forceinline__ void fwd16(double v[16], const double* Lkk, const double* rd) {
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        v[m] *= rd[m];
#pragma unroll
        for (int j = m + 1; j < 16; ++j) v[j] -= Lkk[j * BLD + m] * v[m];
    }
}

// In-LDS Cholesky of the 64x64 SPD block T (lower, stride BLD) fused with the forward
// solve X <- L^-1 X of ncol right-hand columns (X stride XW): per 16-column panel,
// (1) wave 0 factors the diagonal tile, (2) the panel rows below it and the X columns
// run their 16-step substitution in the same phase, (3) the trailing updates of T and
// of X share one MFMA phase.
template <bool STAMP = false>
__device__ void potrf64_fwd(double* T, double* rdiag64, double* X, int ncol, bool& bad,
                            unsigned long long* pst = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    unsigned long long tp = 0;
    if constexpr (STAMP) if (tid == 0 && pst) tp = bcr_stamp();
#define PF_STAMP(k)                                                        \
    do {                                                                   \
        if constexpr (STAMP) if (tid == 0 && pst) {                        \
            const unsigned long long t_ = bcr_stamp();                     \
            pst[k] += t_ - tp;                                             \
            tp = t_;                                                       \
        }                                                                  \
    } while (0)
    const int rr = lane & 15, kk = lane >> 4;
    const int ncb = (ncol + 15) >> 4;
    for (int kb = 0; kb < 4; ++kb) {
        double* Tkk = T + (16 * kb) * BLD + 16 * kb;
        const double* rd = rdiag64 + 16 * kb;
        if (wave == 0) potrf16_tile(Tkk, BLD, rdiag64 + 16 * kb, lane, bad);
        __syncthreads();
        PF_STAMP(0);
        const int nrow = 48 - 16 * kb;
        if (tid < nrow) {
            double* row = T + (16 * (kb + 1) + tid) * BLD + 16 * kb;
            double v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = row[j];
            fwd16(v, Tkk, rd);
#pragma unroll
            for (int j = 0; j < 16; ++j) row[j] = v[j];
        } else if (tid < nrow + ncol) {
            double* col = X + (16 * kb) * XW + (tid - nrow);
            double v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = col[j * XW];
            fwd16(v, Tkk, rd);
#pragma unroll
            for (int j = 0; j < 16; ++j) col[j * XW] = v[j];
        }
        __syncthreads();
        PF_STAMP(1);
        // trailing: T tiles (i, j), kb < j <= i, then X tiles (i > kb, cb)
        const int nt = 3 - kb;
        const int npairs = nt * (nt + 1) / 2;
        const int ntile = npairs + nt * ncb;
        for (int t = wave; t < ntile; t += NWE) {
            const double *Ap, *Bp;
            double* C;
            int ldb, ldc;
            bool colok = true;
            if (t < npairs) {
                int p = 0, rem = t;
                while (rem > p) { rem -= p + 1; ++p; }
                const int i = kb + 1 + p, j = kb + 1 + rem;
                Ap = T + (16 * i + rr) * BLD + 16 * kb;  // L[i][kb] row rr
                Bp = T + (16 * j + rr) * BLD + 16 * kb;  // L[j][kb] row rr  (B = L[j][kb]^T)
                C = T + (16 * i) * BLD + 16 * j;
                ldb = 1;
                ldc = BLD;
            } else {
                const int u = t - npairs, i = kb + 1 + u / ncb, cb = u % ncb;
                Ap = T + (16 * i + rr) * BLD + 16 * kb;
                Bp = X + (16 * kb) * XW + 16 * cb + rr;  // X[kb rows][cols]
                C = X + (16 * i) * XW + 16 * cb;
                ldb = XW;
                ldc = XW;
                colok = 16 * cb + rr < ncol;
            }
            double av[4], bv[4];
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                av[s4] = Ap[4 * s4 + kk];
                bv[s4] = colok ? Bp[(4 * s4 + kk) * ldb] : 0.0;
            }
            d4b acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc, 0, 0, 0);
            if (colok)
#pragma unroll
                for (int g = 0; g < 4; ++g) C[(kk + 4 * g) * ldc + rr] -= acc[g];
        }
        __syncthreads();
        PF_STAMP(2);
    }
#undef PF_STAMP
}

// ---- look-ahead variant: the 16x16 diagonal tiles are inverted right after they are factored,
// so every substitution becomes an MFMA product, and wave 0 runs the pivot chain while the other
// waves do the previous panel's trailing update. Per panel kb (two barrier phases):
//   phase 1  wave 0: potrf16(kb) and W_kb = L_kk^-1 (lanes 0..15, one column each)
//            waves 1-7: trailing update of panel kb-1 on every tile except (kb,kb)
//   phase 2  wave 0: L(kb+1,kb) = A(kb+1,kb) W^T, then (kb+1,kb+1) -= L(kb+1,kb) L(kb+1,kb)^T
//            waves 1-7: L(i,kb) = A(i,kb) W^T for i >= kb+2, and X_kb <- W X_kb
// Each tile receives its panel updates in panel order, as in potrf64_fwd.
// acc = A * B^T over k = 0..15: A rows from a (stride lda), B rows from b (stride ldb)
__device__ __forceinline__ d4b mfma16_abt(const double* a, int lda, const double* b, int ldb, int rr, int kk) {
    double av[4], bv[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
        av[s4] = a[rr * lda + 4 * s4 + kk];
        bv[s4] = b[rr * ldb + 4 * s4 + kk];
    }
    d4b acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc, 0, 0, 0);
    return acc;
}
// acc = A * B over k = 0..15: A rows from a (stride lda), B rows (k) from b (stride ldb), columns rr
__device__ __forceinline__ d4b mfma16_ab(const double* a, int lda, const double* b, int ldb, int rr, int kk,
                                         bool colok) {
    double av[4], bv[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
        av[s4] = a[rr * lda + 4 * s4 + kk];
        bv[s4] = colok ? b[(4 * s4 + kk) * ldb + rr] : 0.0;
    }
    d4b acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc, 0, 0, 0);
    return acc;
}

// Schur contributions of an eliminated block, accumulated k-block by k-block inside the
// factorization: X's row block kb is final after phase 2 of panel kb, so waves 1-7 add
// X_kb^T X_kb to their contribution tiles during phase 1 of panel kb + 1 (beside the trailing
// update, while wave 0 runs the pivot chain); the caller adds the last row block. Tile map of
// k_bcr_contrib: [0,10) UL lower, [10,20) UR lower, [20,36) F = -XR^T XL, [36,40) rL, [40,44) rR.
static constexpr int NCONTRIB = 44;
static constexpr int NCT = (NCONTRIB + NWE - 2) / (NWE - 1);  // tiles per helper wave
struct ContribTile {
    int ib, cb, aoff, boff, ldd;
    double sign;
    bool valid, rhs, gram;
};
// Tile GRAM_TILE (k_bcr_split only, past the k_bcr_contrib map): the Gram x^T x of the block's
// forward-solved right-hand sides x = [b_a | B] (5 of the 8 x columns). Summed over all blocks it is
// [b_a | B]^T A^-1 [b_a | B] (A = L L^T in elimination order, x_i = (L^-1 [b_a | B])_i), which is all
// the 4x4 border system needs: (C - B^T A^-1 B) y_k = b_k - B^T A^-1 b_a.
static constexpr int GRAM_TILE = NCONTRIB;
__device__ __forceinline__ ContribTile contrib_tile(int t, bool has_r) {
    ContribTile c{0, 0, 0, 0, BB, 1.0, true, false, false};
    if (t == GRAM_TILE) {
        c.aoff = c.boff = 2 * BB;
        c.ldd = RC;
        c.rhs = c.gram = true;
    } else if (t < 20) {
        c.valid = t < 10 || has_r;
        int p = 0, rem = t % 10;
        while (rem > p) { rem -= p + 1; ++p; }
        c.ib = p; c.cb = rem;
        c.aoff = c.boff = (t < 10) ? 0 : BB;
    } else if (t < 36) {
        c.valid = has_r;
        c.ib = (t - 20) >> 2; c.cb = (t - 20) & 3;
        c.aoff = BB; c.boff = 0; c.sign = -1.0;
    } else {
        c.valid = t < 40 || has_r;
        c.ib = (t - 36) & 3; c.cb = 0;
        c.aoff = (t < 40) ? 0 : BB; c.boff = 2 * BB;
        c.ldd = RC;
        c.rhs = true;
    }
    return c;
}
__device__ __forceinline__ void contrib_accumulate(const double* X, int kbk, d4b (&cacc)[NCT], bool has_r, int wave,
                                                   int rr, int kk) {
    if (wave == 0) return;  // the pivot wave owns no contribution tile
#pragma unroll
    for (int q = 0; q < NCT; ++q) {
        const int t = (wave - 1) + (NWE - 1) * q;
        if (t >= NCONTRIB) continue;
        const ContribTile ct = contrib_tile(t, has_r);
        if (!ct.valid) continue;
        const bool bok = !ct.rhs || rr < RC;
        double av[4], bv[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            const double* row = X + (16 * kbk + 4 * s4 + kk) * XW;
            av[s4] = row[ct.aoff + 16 * ct.ib + rr];
            bv[s4] = bok ? row[ct.boff + 16 * ct.cb + rr] : 0.0;
        }
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) cacc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], cacc[q], 0, 0, 0);
    }
}

template <bool CONTRIB>
__device__ __forceinline__ void potrf64_fwd_la(double* T, double* rdiag64, double* Wb, double* X, int ncol, bool& bad,
                                               d4b (&cacc)[NCT], bool has_r, unsigned long long* pst = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rr = lane & 15, kk = lane >> 4;
    const int ncb = (ncol + 15) >> 4;
    for (int kb = 0; kb < 4; ++kb) {
        double* Tkk = T + (16 * kb) * BLD + 16 * kb;
        // ---- phase 1
        if (wave == 0) {
            potrf16_tile(Tkk, BLD, rdiag64 + 16 * kb, lane, bad);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < 16) {
                double v[16];
#pragma unroll
                for (int m = 0; m < 16; ++m) v[m] = (m == lane) ? 1.0 : 0.0;
                fwd16(v, Tkk, rdiag64 + 16 * kb);
#pragma unroll
                for (int m = 0; m < 16; ++m) Wb[m * 16 + lane] = v[m];
            }
        } else if (kb > 0) {
            const int p = kb - 1, nt = 4 - kb;
            const int npairs = nt * (nt + 1) / 2 - 1;  // tiles (i,j), kb <= j <= i, minus (kb,kb)
            const int ntile = npairs + nt * ncb;
            for (int t = wave - 1; t < ntile; t += NWE - 1) {
                if (t < npairs) {
                    int q = t + 1, a = 0;
                    while (q > a) { q -= a + 1; ++a; }
                    const int i = kb + a, j = kb + q;
                    const d4b acc = mfma16_abt(T + (16 * i) * BLD + 16 * p, BLD, T + (16 * j) * BLD + 16 * p, BLD, rr, kk);
#pragma unroll
                    for (int g = 0; g < 4; ++g) T[(16 * i + kk + 4 * g) * BLD + 16 * j + rr] -= acc[g];
                } else {
                    const int u = t - npairs, i = kb + u / ncb, cb = u % ncb;
                    const bool colok = 16 * cb + rr < ncol;
                    const d4b acc = mfma16_ab(T + (16 * i) * BLD + 16 * p, BLD, X + (16 * p) * XW + 16 * cb, XW, rr, kk,
                                              colok);
                    if (colok)
#pragma unroll
                        for (int g = 0; g < 4; ++g) X[(16 * i + kk + 4 * g) * XW + 16 * cb + rr] -= acc[g];
                }
            }
            if constexpr (CONTRIB) contrib_accumulate(X, kb - 1, cacc, has_r, wave, rr, kk);
        }
        __syncthreads();
        if (pst && tid == 0) pst[2 * kb] = realtime_now();
        // ---- phase 2
        const int nrow = 3 - kb;  // row tiles below the panel
        if (wave == 0) {
            if (kb < 3) {
                const int i = kb + 1;
                double* Ai = T + (16 * i) * BLD + 16 * kb;
                const d4b acc = mfma16_abt(Ai, BLD, Wb, 16, rr, kk);
#pragma unroll
                for (int g = 0; g < 4; ++g) Ai[(kk + 4 * g) * BLD + rr] = acc[g];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const d4b acc2 = mfma16_abt(Ai, BLD, Ai, BLD, rr, kk);
#pragma unroll
                for (int g = 0; g < 4; ++g) T[(16 * i + kk + 4 * g) * BLD + 16 * i + rr] -= acc2[g];
            }
        } else {
            const int ntile = (nrow > 0 ? nrow - 1 : 0) + ncb;
            for (int t = wave - 1; t < ntile; t += NWE - 1) {
                if (t < nrow - 1) {
                    double* Ai = T + (16 * (kb + 2 + t)) * BLD + 16 * kb;
                    const d4b acc = mfma16_abt(Ai, BLD, Wb, 16, rr, kk);
#pragma unroll
                    for (int g = 0; g < 4; ++g) Ai[(kk + 4 * g) * BLD + rr] = acc[g];
                } else {
                    const int cb = t - (nrow > 0 ? nrow - 1 : 0);
                    const bool colok = 16 * cb + rr < ncol;
                    double* Xc = X + (16 * kb) * XW + 16 * cb;
                    const d4b acc = mfma16_ab(Wb, 16, Xc, XW, rr, kk, colok);
                    if (colok)
#pragma unroll
                        for (int g = 0; g < 4; ++g) Xc[(kk + 4 * g) * XW + rr] = acc[g];
                }
            }
        }
        __syncthreads();
        if (pst && tid == 0) pst[2 * kb + 1] = realtime_now();
    }
}

// X <- L^-T X (backward), L 64x64 lower in LDS (stride BLD), X 64 x ncol (LDS, stride ldx).
__device__ void trsm_lower64_t(const double* L, const double* rdiag64, double* X, int ldx, int ncol) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rr = lane & 15, kk = lane >> 4;
    const int nw = blockDim.x >> 6;
    for (int kb = 3; kb >= 0; --kb) {
        const double* Lkk = L + (16 * kb) * BLD + 16 * kb;
        if (tid < ncol) {
            double* col = X + (16 * kb) * ldx + tid;
            double x[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) x[j] = col[j * ldx];
#pragma unroll
            for (int m = 15; m >= 0; --m) {
                x[m] *= rdiag64[16 * kb + m];
#pragma unroll
                for (int j = 0; j < m; ++j) x[j] -= Lkk[m * BLD + j] * x[m];  // (L^T)[j][m] = L[m][j]
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) col[j * ldx] = x[j];
        }
        __syncthreads();
        const int ncb = (ncol + 15) / 16;
        const int ntile = kb * ncb;
        for (int t = wave; t < ntile; t += nw) {
            const int i = t / ncb, cb = t % ncb;
            const double* A = L + (16 * kb) * BLD + 16 * i;  // L[kb][i]; operand (L^T)[r][k] = L[kb][i][k][r]
            const int col = 16 * cb + rr;
            double av[4], bv[4];
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                av[s4] = A[(4 * s4 + kk) * BLD + rr];
                bv[s4] = (col < ncol) ? X[(16 * kb + 4 * s4 + kk) * ldx + col] : 0.0;
            }
            d4b acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc, 0, 0, 0);
            if (col < ncol)
#pragma unroll
                for (int g = 0; g < 4; ++g) X[(16 * i + kk + 4 * g) * ldx + col] -= acc[g];
        }
        __syncthreads();
    }
}

// Y <- L^-T Y for the 8 right-hand columns of Y (LDS, 64 x RC), L = Cf (LDS, stride BLD,
// upper triangle zero), rd = 1/diag(L). Lane-per-row layout: waves 0..3 each own columns
// (w, w+4); lane r holds row r. Step R = 63..0 finalises row R (y_R = x_R / L_RR) and
// broadcasts x_R by v_readlane; rows r < R subtract (L[R][r] / L_RR) x_R. The row
// L[R][*] is one conflict-free LDS read, issued a step ahead; no barriers inside.
__device__ __forceinline__ double readlane_d(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}
__device__ void trsm_t_lanes(const double* L, const double* rd, double* Y) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (wave < 4) {
        double x0 = Y[lane * RC + wave], x1 = Y[lane * RC + wave + 4];
        // rows of L prefetched PF steps ahead: one step of the chain (FMA -> v_readlane -> FMA) is shorter than an
        // LDS round trip, so a one-step prefetch left every step waiting on its row
        constexpr int PF = 4;
        double lq[PF];
#pragma unroll
        for (int p = 0; p < PF; ++p) lq[p] = L[(63 - p) * BLD + lane] * rd[63 - p];
#pragma unroll
        for (int R = 63; R >= 0; --R) {
            const double lt = lane < R ? lq[(63 - R) % PF] : 0.0;
            if (R - PF >= 0) lq[(63 - R) % PF] = L[(R - PF) * BLD + lane] * rd[R - PF];
            const double xr0 = readlane_d(x0, R), xr1 = readlane_d(x1, R);
            x0 = __builtin_fma(-lt, xr0, x0);
            x1 = __builtin_fma(-lt, xr1, x1);
        }
        const double rdl = rd[lane];
        Y[lane * RC + wave] = x0 * rdl;
        Y[lane * RC + wave + 4] = x1 * rdl;
    }
    __syncthreads();
}

// agent-scope (sc1) 8-byte payload store / load of the in-launch hand-offs (below)
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ void st_pub(double* p, double v) {
    __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_pub(const double* p) {
    return __longlong_as_double(
        (long long)__hip_atomic_load((gu64*)const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Border rows B_i (4 x 60, S rows kb..kb+3 at the block's columns) -> LDS Bl[4][BB]
// (zero past the last dof); one element per thread, issued with the block's other loads.
__device__ __forceinline__ double border_load(const DevProblem& P, const double* __restrict__ S, int i, int e) {
    const int m = e >> 6, r = e & 63;
    const int b0 = i * G_DOF, nd = 6 * P.nac;
    return (e < 4 * BB && r < G_DOF && b0 + r < nd) ? S[(size_t)(P.kb + m) * P.npad + b0 + r] : 0.0;
}
// Border partial B_i^T Y_i (4 x 5) from Bl (LDS) and Y (LDS, stride RC): 80 threads
// = 20 outputs x 4 row quarters, then a fixed-order 4-term sum.
__device__ __forceinline__ void border_partial(const double* Bl, const double* Yl, double* red, int i,
                                               double* __restrict__ Bp) {
    const int t = threadIdx.x;
    if (t < 80) {
        const int q = t >> 2, part = t & 3, m = q / 5, c = q % 5;
        double acc = 0.0;
#pragma unroll
        for (int r = 16 * part; r < 16 * part + 16; ++r) acc += Bl[m * BB + r] * Yl[r * RC + c];
        red[t] = acc;
    }
    __syncthreads();
    if (t < 20) st_pub(Bp + (size_t)i * 32 + t, ((red[4 * t] + red[4 * t + 1]) + red[4 * t + 2]) + red[4 * t + 3]);
}

struct ElimLds {
    double T[BB * BLD];  // D_i -> Cf
    double X[BB * XW];   // [A_l | A_r | R] -> [XL | XR | x]
    double rdiag[BB];
    double Wb[256];      // inverse of the current 16x16 diagonal tile
    double Bl[4 * BB];   // root: border rows
    double red[80];
};

// ---- launch m: eliminate the blocks of level m (workgroups [0, nel)) and fold the level
// m-1 contributions into the accumulators of the level-m survivors (workgroups [nel, ...)).
// m == levels: the root (block 0; one workgroup).
template <bool STAMP>
__global__ __launch_bounds__(TPB_E) void k_bcr_elim(const LmState* __restrict__ st, DevProblem P,
                                                    const double* __restrict__ S, const double* __restrict__ rhs,
                                                    BcrWork Bw, int m, int nel, int* __restrict__ flag,
                                                    unsigned long long* __restrict__ stamps) {
    if (skip_step(st)) return;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    ElimLds& L = *reinterpret_cast<ElimLds*>(smem);
    const int nblk = Bw.nblk;
    const bool root = m >= Bw.levels;
    const int s = 1 << m, h = s >> 1;
    const int tid = threadIdx.x;
    const size_t ld = P.npad;
    const int nd = 6 * P.nac;
    constexpr int NQ = BSZ / TPB_E;  // 64x64 elements per thread
    BCR_STAMP(m, 0);
    if (!root && (int)blockIdx.x >= nel) {
        // accumulator for survivor j (m >= 1): Dacc_j = base - UR_{j-h} - UL_{j+h}
        const int j = ((int)blockIdx.x - nel) << (m + 1);
        if (j >= nblk) return;
        const int a = j - h, b = j + h;
        const int b0 = j * G_DOF;
        double v[NQ], ua[NQ], ub[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = tid + TPB_E * q, r = e >> 6, c = e & 63;
            const bool ok = c <= r && r < G_DOF && b0 + r < nd;
            v[q] = m >= 2 ? Bw.Dacc[(size_t)j * BSZ + e] : (ok ? S[(size_t)(b0 + r) * ld + b0 + c] : (r == c ? 1.0 : 0.0));
            ua[q] = a >= 0 ? Bw.UR[(size_t)a * BSZ + e] : 0.0;
            ub[q] = b < nblk ? Bw.UL[(size_t)b * BSZ + e] : 0.0;
        }
        const int r = tid >> 3, c = tid & 7, gr = b0 + r;
        double rv = 0.0;
        if (m >= 2) rv = Bw.Racc[(size_t)j * RSZ + tid];
        else if (r < G_DOF && gr < nd) rv = c == 0 ? rhs[gr] : (c <= 4 ? S[(size_t)(P.kb + c - 1) * ld + gr] : 0.0);
        const double ra = a >= 0 ? Bw.rR[(size_t)a * RSZ + tid] : 0.0;
        const double rb = b < nblk ? Bw.rL[(size_t)b * RSZ + tid] : 0.0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) Bw.Dacc[(size_t)j * BSZ + tid + TPB_E * q] = (v[q] - ua[q]) - ub[q];
        Bw.Racc[(size_t)j * RSZ + tid] = (rv - ra) - rb;
        return;
    }
    const int i = root ? 0 : s + 2 * s * (int)blockIdx.x;
    if (i >= nblk) return;
    const bool has_r = !root && i + s < nblk;
    const int b0 = i * G_DOF;
    const int a = i - h, b = i + h;  // level m-1 neighbours (m >= 1)
    // ---- one load round: D, R, contributions, couplings
    {
        double v[NQ], ua[NQ], ub[NQ], al[NQ], ar[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = tid + TPB_E * q, r = e >> 6, c = e & 63;
            const bool ok = c <= r && r < G_DOF && b0 + r < nd;
            v[q] = m >= 2 ? Bw.Dacc[(size_t)i * BSZ + e] : (ok ? S[(size_t)(b0 + r) * ld + b0 + c] : (r == c ? 1.0 : 0.0));
            ua[q] = (m >= 1 && a >= 0) ? Bw.UR[(size_t)a * BSZ + e] : 0.0;
            ub[q] = (m >= 1 && b < nblk) ? Bw.UL[(size_t)b * BSZ + e] : 0.0;
            if (root) {
                al[q] = ar[q] = 0.0;
            } else if (m == 0) {
                const bool okl = r < G_DOF && b0 + r < nd && c < G_DOF;
                al[q] = okl ? S[(size_t)(b0 + r) * ld + b0 - G_DOF + c] : 0.0;
                const int b1 = b0 + G_DOF;  // element (r, c) of A[i+1][i] -> A[i][i+1][c][r]
                const bool okr = has_r && r < G_DOF && b1 + r < nd && c < G_DOF;
                ar[q] = okr ? S[(size_t)(b1 + r) * ld + b0 + c] : 0.0;
            } else {
                al[q] = Bw.F[(size_t)(i - h) * BSZ + e];
                ar[q] = has_r ? Bw.F[(size_t)(i + h) * BSZ + e] : 0.0;
            }
        }
        const int r = tid >> 3, c = tid & 7, gr = b0 + r;
        double rv = 0.0;
        if (m >= 2) rv = Bw.Racc[(size_t)i * RSZ + tid];
        else if (r < G_DOF && gr < nd) rv = c == 0 ? rhs[gr] : (c <= 4 ? S[(size_t)(P.kb + c - 1) * ld + gr] : 0.0);
        const double ra = (m >= 1 && a >= 0) ? Bw.rR[(size_t)a * RSZ + tid] : 0.0;
        const double rb = (m >= 1 && b < nblk) ? Bw.rL[(size_t)b * RSZ + tid] : 0.0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = tid + TPB_E * q, rr_ = e >> 6, cc = e & 63;
            L.T[rr_ * BLD + cc] = (v[q] - ua[q]) - ub[q];
            L.X[rr_ * XW + cc] = al[q];
            L.X[cc * XW + BB + rr_] = ar[q];  // A[i][i+s] = (A[i+s][i])^T
        }
        L.X[r * XW + 2 * BB + c] = (rv - ra) - rb;
        if (root && tid < 4 * BB) L.Bl[tid] = border_load(P, S, 0, tid);
    }
    __syncthreads();
    BCR_STAMP(m, 1);
    bool bad = false;
    if (STAMP)
        potrf64_fwd<STAMP>(L.T, L.rdiag, root ? L.X + 2 * BB : L.X, root ? RC : XC, bad,
                           blockIdx.x == 0 ? stamps + 8 * 24 + 4 * m : nullptr);
    else {
        d4b none[NCT];
        potrf64_fwd_la<false>(L.T, L.rdiag, L.Wb, root ? L.X + 2 * BB : L.X, root ? RC : XC, bad, none, false);
    }
    if (bad) raise_flag(flag, FLAG_NOT_PD);
    BCR_STAMP(m, 2);
    if (root) {
        // compact the 8 solved columns (stride RC) next to the factor, backward solve
        double* Yl = L.X;  // rows of X are consumed: reuse its head as Y_0 (stride RC)
        const int r = tid >> 3, c = tid & 7;
        const double z = L.X[r * XW + 2 * BB + c];
        __syncthreads();
        Yl[tid] = z;
        __syncthreads();
        trsm_t_lanes(L.T, L.rdiag, Yl);
        Bw.Y[tid] = Yl[tid];
        if (tid < 4) Bw.bk[tid] = rhs[P.kb + tid];
        if (tid >= 4 && tid < 14) {
            int q = tid - 4, mm = 0;
            while (q > mm) { q -= mm + 1; ++mm; }
            Bw.bk[tid] = S[(size_t)(P.kb + mm) * ld + P.kb + q];  // (mm, q), q <= mm
        }
        __syncthreads();
        border_partial(L.Bl, Yl, L.red, 0, Bw.Bp);
        BCR_STAMP(m, 3);
        return;
    }
    // ---- store factor and solved blocks
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int e = tid + TPB_E * q;
        Bw.Cf[(size_t)i * BSZ + e] = L.T[(e >> 6) * BLD + (e & 63)];
    }
    for (int e = tid; e < XSZ; e += TPB_E) Bw.X[(size_t)i * XSZ + e] = L.X[e];
    if (tid < BB) Bw.rd[(size_t)i * BB + tid] = L.rdiag[tid];
    BCR_STAMP(m, 3);
}

// ---- Schur contributions of the blocks eliminated at level m: 44 tiles per block,
// one per wave, MFMA operands loaded straight from X (L2-resident):
//   t in [0,10) UL lower tiles, [10,20) UR lower tiles, [20,36) F, [36,40) rL, [40,44) rR
__global__ __launch_bounds__(TPB_C) void k_bcr_contrib(const LmState* __restrict__ st, BcrWork Bw, int m) {
    if (skip_step(st)) return;
    const int s = 1 << m;
    const int bi = (int)blockIdx.x / NCONTRIB_WG, r = (int)blockIdx.x % NCONTRIB_WG;
    const int i = s + 2 * s * bi;
    const int nblk = Bw.nblk;
    if (i >= nblk) return;
    const bool has_r = i + s < nblk;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, rr = lane & 15, kq = lane >> 4;
    const int t = 4 * r + wave;
    int ib, cb, aoff, boff, ldd = BB;
    double* dst;
    double sign = 1.0;
    bool rhs_tile = false;
    if (t < 20) {
        if (t >= 10 && !has_r) return;
        int p = 0, rem = t % 10;
        while (rem > p) { rem -= p + 1; ++p; }
        ib = p; cb = rem;
        aoff = boff = (t < 10) ? 0 : BB;
        dst = (t < 10 ? Bw.UL : Bw.UR) + (size_t)i * BSZ;
    } else if (t < 36) {
        if (!has_r) return;
        ib = (t - 20) >> 2; cb = (t - 20) & 3;
        aoff = BB; boff = 0; sign = -1.0;
        dst = Bw.F + (size_t)i * BSZ;
    } else {
        if (t >= 40 && !has_r) return;
        ib = (t - 36) & 3; cb = 0;
        aoff = (t < 40) ? 0 : BB; boff = 2 * BB;
        dst = (t < 40 ? Bw.rL : Bw.rR) + (size_t)i * RSZ;
        ldd = RC;
        rhs_tile = true;
    }
    const bool bcol_ok = !rhs_tile || rr < RC;
    const double* X = Bw.X + (size_t)i * XSZ;
    double av[16], bv[16];
#pragma unroll
    for (int s4 = 0; s4 < 16; ++s4) {
        const double* row = X + (4 * s4 + kq) * XW;
        av[s4] = row[aoff + 16 * ib + rr];
        bv[s4] = bcol_ok ? row[boff + 16 * cb + rr] : 0.0;
    }
    d4b acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s4 = 0; s4 < 16; s4 += 2) {
        acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4 + 1], bv[s4 + 1], acc1, 0, 0, 0);
    }
    if (bcol_ok)
#pragma unroll
        for (int g = 0; g < 4; ++g) dst[(size_t)(16 * ib + kq + 4 * g) * ldd + 16 * cb + rr] = sign * (acc0[g] + acc1[g]);
}

struct BackLds {
    double T[BB * BLD];  // Cf_i
    double t[RSZ], yl[RSZ], yr[RSZ];
    double rdiag[BB];
    double Bl[4 * BB];   // border rows of the block
    double red[80];
};

// ---- back-substitution for the blocks eliminated at level m:
// y_i = Cf_i^-T (x_i - XL_i y_{i-s} - XR_i y_{i+s});  plus the border partial B_i^T y_i.
template <bool STAMP>
__global__ __launch_bounds__(TPB_C) void k_bcr_back(const LmState* __restrict__ st, DevProblem P,
                                                    const double* __restrict__ S, BcrWork Bw, int m,
                                                    unsigned long long* __restrict__ stamps) {
    if (skip_step(st)) return;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    BackLds& L = *reinterpret_cast<BackLds*>(smem);
    const int s = 1 << m;
    const int i = s + 2 * s * (int)blockIdx.x;
    const int nblk = Bw.nblk;
    if (i >= nblk) return;
    BCR_STAMP(16 + m, 0);
    const bool has_r = i + s < nblk;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, rr = lane & 15, kq = lane >> 4;
    constexpr int NQ = BSZ / TPB_C;
    const double* X = Bw.X + (size_t)i * XSZ;
    // ---- one load round: Cf, x, y_{i-s}, y_{i+s}, and the MFMA A-operands XL / XR
    double cf[NQ], xv[2], ylv[2], yrv[2], al[16], ar[16];
#pragma unroll
    for (int q = 0; q < NQ; ++q) cf[q] = Bw.Cf[(size_t)i * BSZ + tid + TPB_C * q];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int e = tid + TPB_C * q, r = e >> 3, c = e & 7;
        xv[q] = X[r * XW + 2 * BB + c];
        ylv[q] = Bw.Y[(size_t)(i - s) * RSZ + e];
        yrv[q] = has_r ? Bw.Y[(size_t)(i + s) * RSZ + e] : 0.0;
    }
#pragma unroll
    for (int s4 = 0; s4 < 16; ++s4) {
        const double* row = X + (16 * wave + rr) * XW + 4 * s4 + kq;  // XL[16w + rr][4 s4 + kq]
        al[s4] = row[0];
        ar[s4] = has_r ? row[BB] : 0.0;
    }
    const double rdv = tid < BB ? Bw.rd[(size_t)i * BB + tid] : 0.0;
    const double blv = border_load(P, S, i, tid);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int e = tid + TPB_C * q;
        L.T[(e >> 6) * BLD + (e & 63)] = cf[q];
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int e = tid + TPB_C * q;
        L.t[e] = xv[q];
        L.yl[e] = ylv[q];
        L.yr[e] = yrv[q];
    }
    if (tid < BB) L.rdiag[tid] = rdv;
    L.Bl[tid] = blv;
    __syncthreads();
    BCR_STAMP(16 + m, 1);
    // t -= XL y_l + XR y_r  (wave w: rows 16w..16w+15)
    {
        d4b acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s4 = 0; s4 < 16; ++s4) {
            const double bl = rr < RC ? L.yl[(4 * s4 + kq) * RC + rr] : 0.0;
            const double br = rr < RC ? L.yr[(4 * s4 + kq) * RC + rr] : 0.0;
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(al[s4], bl, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[s4], br, acc1, 0, 0, 0);
        }
        if (rr < RC)
#pragma unroll
            for (int g = 0; g < 4; ++g) L.t[(16 * wave + kq + 4 * g) * RC + rr] -= acc0[g] + acc1[g];
    }
    __syncthreads();
    BCR_STAMP(16 + m, 2);
    trsm_t_lanes(L.T, L.rdiag, L.t);
#pragma unroll
    for (int q = 0; q < 2; ++q) Bw.Y[(size_t)i * RSZ + tid + TPB_C * q] = L.t[tid + TPB_C * q];
    border_partial(L.Bl, L.t, L.red, i, Bw.Bp);
    BCR_STAMP(16 + m, 3);
}

// ---- border: every workgroup sums the border partials in block order and solves the
// 4x4 system C' y_k = b' (C' = S_kk - B^T V, b' = b_k - B^T u); workgroup i then writes
// y_a = u - V y_k for the rows of block i into rhs (workgroup 0 also y_k) and applies the camera
// step of its cameras (was k_update_cams): lanes < BCR_CAMS, workgroup 0 also the intrinsics; one
// partial per workgroup of the step scalars for k_final. PUB: inside k_bcr_split, after every
// block's back-substitution flag, so Bp and Y are read with sc1 loads; bk = [b_k | S_kk packed].

static constexpr int TPB_BD = 64;
static constexpr int BP_CHUNK = 32;  // blocks' border partials (20 doubles) / Grams (25) staged in LDS per round
template <bool PUB>
__device__ __forceinline__ void border_apply(const LmState* __restrict__ st, const DevProblem& P, double* __restrict__ rhs,
                                             const BcrWork& Bw, int* __restrict__ flag, const BaConsts& c,
                                             const double* __restrict__ scale, const double* __restrict__ camdata,
                                             const double* __restrict__ lin, double* __restrict__ delta,
                                             double* __restrict__ part, int i, const double* bk, double* red,
                                             double* yk, double* ybl, double* bpl) {
    const int tid = threadIdx.x;
    // sum of the blocks' border partials in block order: BP_CHUNK blocks' partials are loaded by all
    // threads at once into LDS (one round trip), then lanes < 20 add them in order
    double bsum = 0.0;
    for (int b0 = 0; b0 < Bw.nblk; b0 += BP_CHUNK) {
        const int nb = Bw.nblk - b0 < BP_CHUNK ? Bw.nblk - b0 : BP_CHUNK;
        for (int e = tid; e < 20 * nb; e += blockDim.x) {
            const double* q = Bw.Bp + (size_t)(b0 + e / 20) * 32 + e % 20;
            bpl[e] = PUB ? ld_pub(q) : *q;
        }
        __syncthreads();
        if (tid < 20)
            for (int b = 0; b < nb; ++b) bsum += bpl[20 * b + tid];
        __syncthreads();
    }
    if (tid < 20) red[tid] = bsum;
    __syncthreads();
    if (tid == 0) {
        bool bad = false;
        border_solve4(bk, red, yk, bad);
        if (bad && i == 0) raise_flag(flag, FLAG_NOT_PD);
    }
    __syncthreads();
    const int b0 = i * G_DOF, nd = 6 * P.nac;
    if (tid < G_DOF && b0 + tid < nd) {
        const double* y = Bw.Y + (size_t)i * RSZ + tid * RC;
        double yv[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) yv[k] = PUB ? ld_pub(y + k) : y[k];
        const double ya = yv[0] - (yv[1] * yk[0] + yv[2] * yk[1] + yv[3] * yk[2] + yv[4] * yk[3]);
        rhs[b0 + tid] = ya;
        ybl[tid] = ya;
    }
    if (i == 0 && tid < 4) rhs[P.kb + tid] = yk[tid];
    if (i == 0 && tid == 0) Bw.flags[0] += 1;  // next call's epoch (persistent / split kernels)
    __syncthreads();
    if (tid >= 64) return;  // the camera step is wave 0's
    const int cur = st->cur;
    const double radius = st->radius;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};  // sn2, mcc, cand cost, |x_cand|^2
    const int ac = i * BCR_CAMS + tid;
    if (tid < BCR_CAMS && ac < P.nac)
        update_camera(P, c, cur, radius, scale, camdata, ac, ybl + 6 * tid, delta, acc);
    else if (i == 0 && tid == BCR_CAMS)
        update_intrinsics(P, c, cur, radius, scale, lin, yk, delta, acc);
    // (only lanes < 16 hold a term: the row-0 sum by DPP is the total)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = dpp_row_sum(acc[k]);
    if (tid == 0) {
        part[PART_UPD_SN2 * P.part_stride + i] = acc[0];
        part[PART_UPD_MCC * P.part_stride + i] = acc[1];
        part[PART_UPD_COST * P.part_stride + i] = acc[2];
        part[PART_UPD_XN2 * P.part_stride + i] = acc[3];
    }
}
// k_bcr_split's step of block i once its y rows [u | V] (LDS, stride RC) and y_k (LDS) are known:
// y_a = u - V y_k into rhs, the block's camera steps (wave 0) and their model-cost / norm terms
// (part[*][i]); the root block also y_k itself and the intrinsics step. No wait for other blocks.
__device__ __forceinline__ void block_step(const LmState* __restrict__ st, const DevProblem& P, double* __restrict__ rhs,
                                           const BaConsts& c, const double* __restrict__ scale,
                                           const double* __restrict__ camdata, const double* __restrict__ lin,
                                           double* __restrict__ delta, double* __restrict__ part, int i, bool intr,
                                           const double* Yrows, const double* yk, double* ybl) {
    const int tid = threadIdx.x;
    const int b0 = i * G_DOF, nd = 6 * P.nac;
    if (tid < G_DOF && b0 + tid < nd) {
        const double* y = Yrows + tid * RC;
        const double ya = y[0] - (y[1] * yk[0] + y[2] * yk[1] + y[3] * yk[2] + y[4] * yk[3]);
        rhs[b0 + tid] = ya;
        ybl[tid] = ya;
    }
    if (intr && tid < 4) rhs[P.kb + tid] = yk[tid];
    __syncthreads();
    if (tid >= 64) return;  // the camera step is wave 0's
    const int cur = st->cur;
    const double radius = st->radius;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};  // sn2, mcc, cand cost, |x_cand|^2
    const int ac = i * BCR_CAMS + tid;
    if (tid < BCR_CAMS && ac < P.nac)
        update_camera(P, c, cur, radius, scale, camdata, ac, ybl + 6 * tid, delta, acc);
    else if (intr && tid == BCR_CAMS)
        update_intrinsics(P, c, cur, radius, scale, lin, yk, delta, acc);
    // (only lanes < 16 hold a term: the row-0 sum by DPP is the total)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = dpp_row_sum(acc[k]);
    if (tid == 0) {
        part[PART_UPD_SN2 * P.part_stride + i] = acc[0];
        part[PART_UPD_MCC * P.part_stride + i] = acc[1];
        part[PART_UPD_COST * P.part_stride + i] = acc[2];
        part[PART_UPD_XN2 * P.part_stride + i] = acc[3];
    }
}
__global__ __launch_bounds__(TPB_BD) void k_bcr_border(const LmState* __restrict__ st, DevProblem P,
                                                       double* __restrict__ rhs, BcrWork Bw, int* __restrict__ flag,
                                                       BaConsts c, const double* __restrict__ scale,
                                                       const double* __restrict__ camdata,
                                                       const double* __restrict__ lin, double* __restrict__ delta,
                                                       double* __restrict__ part) {
    if (skip_step(st)) return;
    __shared__ double red[20];
    __shared__ double yk[4];
    __shared__ double ybl[G_DOF];
    __shared__ double bpl[20 * BP_CHUNK];
    border_apply<false>(st, P, rhs, Bw, flag, c, scale, camdata, lin, delta, part, blockIdx.x, Bw.bk, red, yk, ybl,
                        bpl);
}

// ---- persistent path: one resident workgroup per block for the whole solve -------------------
// Workgroup i keeps D_i -> Cf_i and [A_l | A_r | R] -> [XL | XR | x] in LDS from its first load to
// its back-substitution, so nothing of its own is stored or re-read. It folds the contributions of
// its neighbours i -+ 2^m for every level m it survives (waiting on their "eliminated" flags),
// eliminates at level ctz(i) (block 0: root) and publishes UL/UR/F/rL/rR, then waits for the
// "back-substituted" flags of i -+ 2^ctz(i) and publishes y_i. The arithmetic and its order are
// those of the per-level launches (k_bcr_elim / k_bcr_contrib / k_bcr_back): same results bit for bit.
// Hand-offs follow the gfx950 inter-workgroup recipe: payload written and read with agent-scope
// (sc1) 8-byte accesses, every storing wave drains (s_waitcnt vmcnt(0)) before the workgroup barrier
// behind which ONE lane stores the flag; ONE lane polls (relaxed, s_sleep), the others read after a
// barrier. Flags hold the call epoch (flags[0] + 1; k_bcr_border advances flags[0]), so nothing is
// reset per call. Every spin is bounded: a timeout raises FLAG_TIMEOUT in chol_flag, which ends the solve
// with BA_E_INTERNAL (the context then falls back to the per-level launches).
__device__ __forceinline__ void publish_flag(unsigned* f, unsigned epoch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store((gu32*)f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// polls before a hand-off wait gives up (bcr_set_spin_limit; tests force a tiny bound)
__device__ unsigned g_spin_limit = 1u << 22;
// read once per function into spin_lim (a load of g_spin_limit inside a poll loop puts a memory round trip
// on every retry)
#define SPIN_LIMIT spin_lim
// ONE lane polls fa and fb together (either may be null: both loads in flight per round trip, so two
// flags that are already set cost one round trip, not two); uniform result, false on timeout.
__device__ bool wait_flags(const unsigned* fa, const unsigned* fb, unsigned epoch, int* lds_ok) {
    if (threadIdx.x == 0) {
        const unsigned spin_lim = g_spin_limit;
        int ok = 1;
        unsigned n = 0;
        for (;;) {
            const unsigned va =
                fa ? __hip_atomic_load((gu32*)const_cast<unsigned*>(fa), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : epoch;
            const unsigned vb =
                fb ? __hip_atomic_load((gu32*)const_cast<unsigned*>(fb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : epoch;
            if (va == epoch && vb == epoch) break;
            __builtin_amdgcn_s_sleep(2);
            if (++n > SPIN_LIMIT) { ok = 0; break; }
        }
        *lds_ok = ok;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the payload loads below the poll
    __syncthreads();
    return *lds_ok != 0;
}

struct PersistLds {
    double T[BB * BLD];  // D_i -> Cf_i
    double X[BB * XW];   // [A_l | A_r | R] -> [XL | XR | x]
    double rdiag[BB];
    double Wb[256];      // inverse of the current 16x16 diagonal tile
    double Bl[4 * BB];   // border rows of block i
    double red[80];
    double yl[RSZ], yr[RSZ], yt[RSZ];
    int ok;
};

// timeline stamps (100 MHz realtime, comparable across XCDs): tl[32 i + k]
#define TL(k)                                                                 \
    do {                                                                      \
        if constexpr (STAMP) if (threadIdx.x == 0) tl[32 * blockIdx.x + (k)] = realtime_now(); \
    } while (0)

template <bool STAMP>
__global__ __launch_bounds__(TPB_E) void k_bcr_persist(const LmState* __restrict__ st, DevProblem P,
                                                       const double* __restrict__ S, const double* __restrict__ rhs,
                                                       BcrWork Bw, int* __restrict__ flag,
                                                       unsigned long long* __restrict__ tl) {
    if (skip_step(st)) return;
    TL(0);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    PersistLds& L = *reinterpret_cast<PersistLds*>(smem);
    const int nblk = Bw.nblk;
    const int i = blockIdx.x;
    const bool root = i == 0;
    const int mi = root ? Bw.levels : __builtin_ctz(i);  // elimination level of block i
    const int tid = threadIdx.x;
    const size_t ld = P.npad;
    const int nd = 6 * P.nac;
    const int b0 = i * G_DOF;
    const unsigned epoch = Bw.flags[0] + 1;
    unsigned* elim_f = Bw.flags + 16;
    unsigned* back_f = Bw.flags + 16 + nblk;
    constexpr int NQ = BSZ / TPB_E;
    // ---- level-0 state (and the level-0 couplings of blocks eliminated at level 0)
    {
        double v[NQ], al[NQ], ar[NQ];
        const bool has_r0 = i + 1 < nblk;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = tid + TPB_E * q, r = e >> 6, c = e & 63;
            const bool ok = c <= r && r < G_DOF && b0 + r < nd;
            v[q] = ok ? S[(size_t)(b0 + r) * ld + b0 + c] : (r == c ? 1.0 : 0.0);
            if (mi == 0) {
                const bool okl = r < G_DOF && b0 + r < nd && c < G_DOF;
                al[q] = okl ? S[(size_t)(b0 + r) * ld + b0 - G_DOF + c] : 0.0;
                const int b1 = b0 + G_DOF;
                const bool okr = has_r0 && r < G_DOF && b1 + r < nd && c < G_DOF;
                ar[q] = okr ? S[(size_t)(b1 + r) * ld + b0 + c] : 0.0;
            }
        }
        const int r = tid >> 3, c = tid & 7, gr = b0 + r;
        double rv = 0.0;
        if (r < G_DOF && gr < nd) rv = c == 0 ? rhs[gr] : (c <= 4 ? S[(size_t)(P.kb + c - 1) * ld + gr] : 0.0);
        const double blv = tid < 4 * BB ? border_load(P, S, i, tid) : 0.0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = tid + TPB_E * q, rr_ = e >> 6, cc = e & 63;
            L.T[rr_ * BLD + cc] = v[q];
            if (mi == 0) {
                L.X[rr_ * XW + cc] = al[q];
                L.X[cc * XW + BB + rr_] = ar[q];
            }
        }
        L.X[r * XW + 2 * BB + c] = rv;
        if (tid < 4 * BB) L.Bl[tid] = blv;
    }
    TL(1);
    // ---- survive levels 0 .. mi-1: fold the neighbours' contributions (same order as Dacc/Racc)
    for (int m = 0; m < mi; ++m) {
        const int s = 1 << m, a = i - s, b = i + s;
        const bool last = m == mi - 1 && !root;
        const bool has_r = i + 2 * s < nblk;  // right coupling at elimination level m + 1 = mi
        if (!wait_flags(a >= 0 ? elim_f + a : nullptr, b < nblk ? elim_f + b : nullptr, epoch, &L.ok)) {
            if (tid == 0) raise_flag(flag, FLAG_TIMEOUT);
            return;
        }
        TL(2 + m);
        double ua[NQ], ub[NQ], fl[NQ], fr[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = tid + TPB_E * q;
            const bool lower = ((e & 63) >> 4) <= ((e >> 6) >> 4);  // UR / UL upper tiles are zero and unread
            ua[q] = a >= 0 && lower ? ld_pub(Bw.UR + (size_t)a * BSZ + e) : 0.0;
            ub[q] = b < nblk && lower ? ld_pub(Bw.UL + (size_t)b * BSZ + e) : 0.0;
            if (last) {
                fl[q] = ld_pub(Bw.F + (size_t)a * BSZ + e);
                fr[q] = has_r ? ld_pub(Bw.F + (size_t)b * BSZ + e) : 0.0;
            }
        }
        const double ra = a >= 0 ? ld_pub(Bw.rR + (size_t)a * RSZ + tid) : 0.0;
        const double rb = b < nblk ? ld_pub(Bw.rL + (size_t)b * RSZ + tid) : 0.0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = tid + TPB_E * q, rr_ = e >> 6, cc = e & 63;
            L.T[rr_ * BLD + cc] = (L.T[rr_ * BLD + cc] - ua[q]) - ub[q];
            if (last) {
                L.X[rr_ * XW + cc] = fl[q];
                L.X[cc * XW + BB + rr_] = fr[q];
            }
        }
        const int r = tid >> 3, c = tid & 7;
        L.X[r * XW + 2 * BB + c] = (L.X[r * XW + 2 * BB + c] - ra) - rb;
    }
    __syncthreads();
    // ---- eliminate: Cf = chol(D), X <- Cf^-1 X
    bool bad = false;
    __syncthreads();
    TL(9);
    const int s = 1 << mi;
    const bool has_r = !root && i + s < nblk;
    d4b cacc[NCT];
#pragma unroll
    for (int q = 0; q < NCT; ++q) cacc[q] = d4b{0.0, 0.0, 0.0, 0.0};
    unsigned long long* pst = nullptr;
    if constexpr (STAMP) pst = tl + 32 * i + 16;
    if (root)
        potrf64_fwd_la<false>(L.T, L.rdiag, L.Wb, L.X + 2 * BB, RC, bad, cacc, false, pst);
    else
        potrf64_fwd_la<true>(L.T, L.rdiag, L.Wb, L.X, XC, bad, cacc, has_r, pst);
    if (bad) raise_flag(flag, FLAG_NOT_PD);
    TL(10);
    if (root) {
        double* Yl = L.yt;
        {
            const int r = tid >> 3, c = tid & 7;
            Yl[tid] = L.X[r * XW + 2 * BB + c];
        }
        __syncthreads();
        trsm_t_lanes(L.T, L.rdiag, Yl);
        st_pub(Bw.Y + tid, Yl[tid]);
        if (tid < 4) Bw.bk[tid] = rhs[P.kb + tid];
        if (tid >= 4 && tid < 14) {
            int q = tid - 4, mm = 0;
            while (q > mm) { q -= mm + 1; ++mm; }
            Bw.bk[tid] = S[(size_t)(P.kb + mm) * ld + P.kb + q];
        }
        __syncthreads();
        border_partial(L.Bl, Yl, L.red, 0, Bw.Bp);
        publish_flag(back_f, epoch);
        TL(14);
        return;
    }
    const int lane = tid & 63, wave = tid >> 6, rr = lane & 15, kq = lane >> 4;
    // ---- Schur contributions: add the last row block of X, then publish (sc1)
    contrib_accumulate(L.X, 3, cacc, has_r, wave, rr, kq);
#pragma unroll
    for (int q = 0; q < NCT; ++q) {
        const int t = (wave - 1) + (NWE - 1) * q;
        if (wave == 0 || t >= NCONTRIB) continue;
        const ContribTile ct = contrib_tile(t, has_r);
        if (!ct.valid || (ct.rhs && rr >= RC)) continue;
        double* dst = (t < 10 ? Bw.UL : t < 20 ? Bw.UR : t < 36 ? Bw.F : t < 40 ? Bw.rL : Bw.rR) +
                      (size_t)i * (ct.rhs ? RSZ : BSZ);
#pragma unroll
        for (int g = 0; g < 4; ++g)
            st_pub(dst + (size_t)(16 * ct.ib + kq + 4 * g) * ct.ldd + 16 * ct.cb + rr, ct.sign * cacc[q][g]);
    }
    publish_flag(elim_f + i, epoch);
    TL(11);
    // ---- off the critical path, while the higher levels finish: [P | Q | u] = Cf^-T [XL | XR | x]
    trsm_lower64_t(L.T, L.rdiag, L.X, XW, XC);
    TL(13);
    // ---- back-substitution: y_i = u - P y_{i-s} - Q y_{i+s}  (= Cf^-T (x_i - XL y_{i-s} - XR y_{i+s}))
    if (!wait_flags(back_f + (i - s), has_r ? back_f + (i + s) : nullptr, epoch, &L.ok)) {
        if (tid == 0) raise_flag(flag, FLAG_TIMEOUT);
        return;
    }
    TL(12);
    L.yl[tid] = ld_pub(Bw.Y + (size_t)(i - s) * RSZ + tid);
    L.yr[tid] = has_r ? ld_pub(Bw.Y + (size_t)(i + s) * RSZ + tid) : 0.0;
    L.yt[tid] = L.X[(tid >> 3) * XW + 2 * BB + (tid & 7)];
    __syncthreads();
    if (wave < 4) {
        double al[16], ar[16];
#pragma unroll
        for (int s4 = 0; s4 < 16; ++s4) {
            const double* row = L.X + (16 * wave + rr) * XW + 4 * s4 + kq;
            al[s4] = row[0];
            ar[s4] = has_r ? row[BB] : 0.0;
        }
        d4b acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s4 = 0; s4 < 16; ++s4) {
            const double bl = rr < RC ? L.yl[(4 * s4 + kq) * RC + rr] : 0.0;
            const double br = rr < RC ? L.yr[(4 * s4 + kq) * RC + rr] : 0.0;
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(al[s4], bl, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[s4], br, acc1, 0, 0, 0);
        }
        if (rr < RC)
#pragma unroll
            for (int g = 0; g < 4; ++g) L.yt[(16 * wave + kq + 4 * g) * RC + rr] -= acc0[g] + acc1[g];
    }
    __syncthreads();
    st_pub(Bw.Y + (size_t)i * RSZ + tid, L.yt[tid]);
    border_partial(L.Bl, L.yt, L.red, i, Bw.Bp);
    publish_flag(back_f + i, epoch);
    TL(14);
}
#undef TL

// ---- split persistent path: two resident workgroups per block --------------------------------
// F(i) ("factor") holds D_i and runs only the pivot side of the 64x64 Cholesky (potrf16 + W per
// panel, the T trailing updates and row panels), publishing each finished column panel (L tiles,
// W_kb, 1/diag) to global memory. H(i) ("helper", another CU) holds [A_l | A_r | R] and applies the
// panels as they arrive: X_kb <- W_kb X_kb, X_i -= L(i,kb) X_kb, and the Schur contributions of row
// block kb; it publishes the contributions, then runs the back-substitution from its copy of L.
// F's pivot chain thus no longer shares its CU's f64 pipes with the 136-column MFMA work.
// Hand-offs as in k_bcr_persist; panel flags hold 4 * epoch + kb (monotone, polled with >=).
static constexpr int SG_LD = 66;         // LDS row stride of pulled 64-column row blocks (Pull)
static constexpr int SG_W = 16 * SG_LD;  // one staged 16 x 64 row block
struct FLds {
    double T[BB * BLD];
    double rdiag[BB];
    double Lcm[4][256];  // panel kb's diagonal tile, column-major (wave 0 -> wave 5: W_kb = L_kk^-1)
    double sg[2 * SG_W];  // pulled row blocks XR_a, XL_b of the survived levels
    int ok;
    int sync[12];  // look-ahead flags of the factor workgroup (k_bcr_split)
};
struct HLds {
    double X[BB * XW];
    double L[BB * BLD];   // copy of Cf, filled panel by panel
    double rdiag[BB];
    double W[4][256];
    double Bl[4 * BB];
    double red[100];  // border partials / the root's Gram quarters
    double yl[RSZ], yr[RSZ], yt[RSZ];
    double bk[16], bred[25], byk[4], bybl[G_DOF];  // border: S_kk / b_k, sums / Gram, y_k, the block's y rows
    double bpl[25 * 32];                            // staged border partials / Grams (BP_CHUNK blocks)
    int ok;
    int pre;  // next panel's flags already set (prefetch)
};
static constexpr int PANEL_DOUBLES = BB * BB + 4 * 256 + BB;  // per block: L tiles | W_0..3 | 1/diag

// ONE lane polls f (>= target) and, if given, f2 (>= target2); uniform result, false on timeout.
__device__ bool wait_ge(const unsigned* f, unsigned target, int* lds_ok, const unsigned* f2 = nullptr,
                        unsigned target2 = 0) {
    if (threadIdx.x == 0) {
        const unsigned spin_lim = g_spin_limit;
        int ok = 1;
        unsigned n = 0;
        for (;;) {  // both loads in flight per round trip
            const unsigned v = __hip_atomic_load((gu32*)const_cast<unsigned*>(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned v2 =
                f2 ? __hip_atomic_load((gu32*)const_cast<unsigned*>(f2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : target2;
            if (v >= target && v2 >= target2) break;
            __builtin_amdgcn_s_sleep(2);
            if (++n > SPIN_LIMIT) { ok = 0; break; }
        }
        *lds_ok = ok;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __syncthreads();
    return *lds_ok != 0;
}
// Wave 0 polls every block's flag (lane j: blocks j, j + 64, ...; relaxed, bounded); uniform result.
// The payload behind these flags is read with sc1 loads only (ld_pub), so no acquire fence.
__device__ bool wait_all_eq(const unsigned* f, int n, unsigned epoch, int* lds_ok, int skip = -1) {
    if (threadIdx.x < 64) {
        const unsigned spin_lim = g_spin_limit;
        int ok = 1;
        for (int j = threadIdx.x; j < n && ok; j += 64) {
            if (j == skip) continue;
            unsigned cnt = 0;
            while (__hip_atomic_load((gu32*)const_cast<unsigned*>(f + j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                   epoch) {
                __builtin_amdgcn_s_sleep(2);
                if (++cnt > SPIN_LIMIT) { ok = 0; break; }
            }
        }
        ok = __all(ok);
        if (threadIdx.x == 0) *lds_ok = ok;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the payload loads below the poll
    __syncthreads();
    return *lds_ok != 0;
}

// k_bcr_split's back-substitution hand-off without flags: block i's y rows for epoch e live in
// ybuf(e) (Y / Racc by parity); the producer stores them (agent scope) with no drain, barrier or flag,
// and resets its slot of ybuf(e + 1) to BCR_Y_EMPTY at the start of the launch; a consumer polls the
// 8-byte values themselves, so a hop costs one store-to-load latency instead of drain + flag + poll +
// load. The root carries y_k in its rows 0..3, column 5 (a pad column of [u | V]).
__device__ __forceinline__ double* ybuf(const BcrWork& Bw, unsigned epoch) { return (epoch & 1) ? Bw.Racc : Bw.Y; }
__device__ __forceinline__ unsigned long long ld_u64(const double* p) {
    return __hip_atomic_load((gu64*)const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The same protocol carries the factor workgroup's published panels to its helpers (Cf | X slots, two
// epochs).
// lower 16 x 16 tiles of a column-major 64 x 64 slot (element e = column * 64 + row)
__device__ __forceinline__ bool lower_tile_cm(int e) { return ((e & 63) >> 4) >= ((e >> 6) >> 4); }

// Pull hand-off between the levels (k_bcr_split). The eliminated block's helpers publish every finished row
// block kb of their forward-substituted columns — XL and XR (16 x 64 each), x (16 x 8) — into epoch-parity
// slots, flag-free (no drain: consumers poll the values, an empty slot holds BCR_Y_EMPTY). Each survivor's
// workgroups then form the Schur terms they need themselves, row block by row block, as the rows arrive
// (a = j - s, b = j + s are eliminated at level m):
//   factor F(j):  D_j -= XR_a^T XR_a + XL_b^T XL_b
//   helpers:      x_j -= XR_a^T x_a + XL_b^T x_b; at j's last survived level the couplings of its own level,
//                 XL_j = -XR_a^T XL_a (helper A) and XR_j = -XL_b^T XR_b (helper B) (the fills)
// The eliminated block's helpers thus run only the forward substitution (at the factor's pace), and the
// next level's factor starts one row-block hand-off after the last panel instead of after the contribution
// tiles, their publication and their flag.
__device__ __forceinline__ double* pub_xl(const BcrWork& Bw, unsigned e) { return (e & 1) ? Bw.F : Bw.UL; }
__device__ __forceinline__ double* pub_xr(const BcrWork& Bw, unsigned e) { return (e & 1) ? Bw.F2 : Bw.UR; }
__device__ __forceinline__ double* pub_x(const BcrWork& Bw, unsigned e) { return (e & 1) ? Bw.rR : Bw.rL; }
template <int NW, int NX>
struct PullSrc {
    const double* w[NW];               // 64-column sources (64 x 64 row-major); nullptr: staged as zeros
    const double* x[NX > 0 ? NX : 1];  // 8-column sources (64 x 8)
};
// Row block kb of every source -> LDS sg (64-column sources at sg + k SG_W, row stride SG_LD, then the
// 8-column ones, 128 each). issue(kb) puts this thread's loads in flight (the caller issues row block kb + 1
// right after committing kb, so the loads overlap its MFMAs); commit(kb) re-polls the values still empty and
// stores the row block to LDS. With `probe`, while some value is still empty ONE lane first waits for each
// live source's last entry of the row block (all in flight per round trip), so a long wait does not load the
// memory path the producers store through. commit's first barrier also ends the previous row block's reads of
// sg. Uniform result; false on timeout.
template <int NW, int NX>
struct Pull {
    static constexpr int NE = NW * 1024 + NX * 128, NU = (NE + TPB_E - 1) / TPB_E;
    unsigned long long v[NU];
    // the source of entry u is uniform over the workgroup (64-column part: source u / 2, rows 8 (u & 1) + wave)
    // or a wave (8-column part, u == 2 NW: source wave / 2). Written with the source index a compile-time
    // constant (u is one in the unrolled loops) or a select, so the sources stay in registers: indexed by
    // (threadIdx.x + TPB_E u) >> 10 they went to scratch, one extra memory round trip in front of every pull.
    __device__ __forceinline__ const double* gaddr(const PullSrc<NW, NX>& ps, int kb, int u) const {
        static_assert(TPB_E == 512 && NX <= 4, "row-block split assumes 512 threads");
        const int tid = threadIdx.x;
        if (u < 2 * NW) {
            const double* p = ps.w[u >> 1];
            return p ? p + (16 * kb + 8 * (u & 1) + (tid >> 6)) * BB + (tid & 63) : nullptr;
        }
        if constexpr (NX > 0) {
            if (u == 2 * NW && tid < NX * 128) {
                const int k = tid >> 7;
                const double* p = ps.x[0];
#pragma unroll
                for (int q = 1; q < NX; ++q) p = k == q ? ps.x[q] : p;
                return p ? p + (16 * kb + ((tid >> 3) & 15)) * RC + (tid & 7) : nullptr;
            }
        }
        return nullptr;
    }
    __device__ __forceinline__ void issue(const PullSrc<NW, NX>& ps, int kb) {
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const double* a = gaddr(ps, kb, u);
            v[u] = a ? ld_u64(a) : 0ull;
        }
    }
    __device__ bool commit(const PullSrc<NW, NX>& ps, int kb, double* sg, int* lds_ok, unsigned spin_lim, bool probe) {
        const int tid = threadIdx.x;
        bool pend = false;
#pragma unroll
        for (int u = 0; u < NU; ++u) pend = pend || v[u] == BCR_Y_EMPTY;
        if (__syncthreads_or(pend) && probe) {
            if (tid == 0) {
                const double* pp[NW + NX];
                unsigned long long pv[NW + NX];
#pragma unroll
                for (int k = 0; k < NW + NX; ++k) {
                    const double* p = k < NW ? ps.w[k] : ps.x[k - NW];
                    pp[k] = p ? p + (k < NW ? (16 * kb + 15) * BB + BB - 1 : (16 * kb + 15) * RC + RC - 1) : nullptr;
                    pv[k] = pp[k] ? ld_u64(pp[k]) : 0ull;
                }
                int ok = 1;
                for (unsigned n = 0;; ++n) {
                    bool pw = false;
#pragma unroll
                    for (int k = 0; k < NW + NX; ++k) pw = pw || pv[k] == BCR_Y_EMPTY;
                    if (!pw) break;
                    if (n > SPIN_LIMIT) { ok = 0; break; }
                    __builtin_amdgcn_s_sleep(2);
#pragma unroll
                    for (int k = 0; k < NW + NX; ++k)
                        if (pv[k] == BCR_Y_EMPTY) pv[k] = ld_u64(pp[k]);
                }
                *lds_ok = ok;
            }
            __syncthreads();
            if (!*lds_ok) return false;
        }
        int ok = 1;
        for (unsigned n = 0;; ++n) {
            bool pe = false;
#pragma unroll
            for (int u = 0; u < NU; ++u) pe = pe || v[u] == BCR_Y_EMPTY;
            if (!pe) break;
            if (n > SPIN_LIMIT) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int u = 0; u < NU; ++u)
                if (v[u] == BCR_Y_EMPTY) v[u] = ld_u64(gaddr(ps, kb, u));
        }
#pragma unroll
        for (int u = 0; u < NU; ++u) {
            const int e = tid + TPB_E * u;
            const double d = __longlong_as_double((long long)v[u]);
            if (e < NW * 1024) sg[(e >> 10) * SG_W + ((e >> 6) & 15) * SG_LD + (e & 63)] = d;
            else if (e < NE) sg[NW * SG_W + (e - NW * 1024)] = d;
        }
        return __syncthreads_and(ok);
    }
};

#define TLS(k)                                                                                     \
    do {                                                                                           \
        if constexpr (STAMP) if (threadIdx.x == 0) tl[32 * blockIdx.x + (k)] = realtime_now();      \
    } while (0)
// Helper roles: NH = 1 -> one helper H per block owning all of [XL | XR | x]; NH = 2 -> helper A owns
// [XL | x], helper B owns [XR | x], the Gram of x and the back-substitution data [P | Q | u] and y_i.
// x (8 columns) is forward-substituted by both (same arithmetic, bitwise identical copies): its row
// block r lives in LDS and belongs to wave 4 + r (waves 0-3 hold the four XL / XR column tiles, one
// per SIMD), so x_kb <- W_kb x_kb runs beside the column tiles and x_ii -= L(ii,kb) x_kb after them.
// Column tile of [XL | XR | x] (16 columns) a helper wave keeps in registers (-1: none); NH = 1 also keeps
// the x columns (tile 8) on wave 0. The root has only the x columns (NH = 1: wave 0; NH = 2: LDS rows).
template <int NH>
__device__ __forceinline__ int helper_cb(bool roleB, int wave, bool root) {
    if (root) return (NH == 1 && wave == 0) ? 0 : -1;
    if (NH == 1) return wave;
    return wave < 4 ? (roleB ? 4 + wave : wave) : -1;
}

template <bool STAMP, int NH>
__global__ __launch_bounds__(TPB_E) void k_bcr_split(const LmState* __restrict__ st, DevProblem P,
                                                     const double* __restrict__ S, double* __restrict__ rhs,
                                                     BcrWork Bw, int* __restrict__ flag,
                                                     unsigned long long* __restrict__ tl, BaConsts c,
                                                     const double* __restrict__ scale,
                                                     const double* __restrict__ camdata,
                                                     const double* __restrict__ lin, double* __restrict__ delta,
                                                     double* __restrict__ part) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int nblk = Bw.nblk;
    // workgroup id (xmap: launch workgroup b on XCD b mod 8; only XCDs 0-3 take a role, densely numbered)
    int bid = blockIdx.x;
    if (Bw.xmap) {
        if ((bid & 7) >= 4) return;
        bid = (bid >> 3) * 4 + (bid & 7);
        if (bid >= (NH + 1) * nblk) return;
    }
    const int i = bid / (NH + 1);
    const int role = bid % (NH + 1);  // 0 factor, 1 helper (A), 2 helper B
    // elimination tree on virtual indices v = i + voff (balanced: the root is the middle block, depth
    // floor(log2 nblk) + 1 instead of ceil(log2 nblk) + 1 with block 0 as the root)
    const bool root = i == Bw.vroot;
    const int mi = root ? Bw.vlevels : __builtin_ctz(i + Bw.voff);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, rr = lane & 15, kk = lane >> 4;
    const size_t ld = P.npad;
    const int nd = 6 * P.nac;
    const int b0 = i * G_DOF;
    constexpr int NQ = BSZ / TPB_E;
    // The level-0 inputs from S (their addresses depend on kernel arguments only) are issued before the LM state
    // is read, so their memory round trip overlaps the state's instead of following it: the factor workgroup's
    // D_i, the helpers' couplings [A_l | A_r] (level-0 blocks) and rhs / border columns, the root's border inputs.
    constexpr int NQX = (NH == 1 ? 2 : 1) * NQ;
    double pre[NQX];
    double pre_r = 0.0, pre_bk = 0.0;
    const bool roleA0 = NH == 2 && role == 1;
    if (role == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = tid + TPB_E * q, r = e >> 6, c = e & 63;
            const bool ok = c <= r && r < G_DOF && b0 + r < nd;
            pre[q] = S[ok ? (size_t)(b0 + r) * ld + b0 + c : 0];
        }
    } else {
        if (mi == 0) {
            // straight-line: the role picks the address (a select, no branch), so the loads stay in flight together
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int e = tid + TPB_E * q, r = e >> 6, c = e & 63;
                const int b1 = b0 + G_DOF;
                const bool okl = i >= 1 && r < G_DOF && b0 + r < nd && c < G_DOF;
                const bool okr = i + 1 < nblk && r < G_DOF && b1 + r < nd && c < G_DOF;
                const size_t al = okl ? (size_t)(b0 + r) * ld + b0 - G_DOF + c : 0;
                const size_t ar = okr ? (size_t)(b1 + r) * ld + b0 + c : 0;
                if constexpr (NH == 1) {
                    pre[q] = S[al];
                    pre[NQ + q] = S[ar];
                } else {
                    pre[q] = S[roleA0 ? al : ar];
                }
            }
        }
        const int r = tid >> 3, c = tid & 7, gr = b0 + r;
        const bool rok = r < G_DOF && gr < nd && c <= 4;
        pre_r = rok ? (c == 0 ? rhs[gr] : S[(size_t)(P.kb + c - 1) * ld + gr]) : 0.0;
        if (root && tid < 14) {  // border inputs [b_k | S_kk packed]
            int q = tid - 4, mm = 0;
            while (q > mm) { q -= mm + 1; ++mm; }
            pre_bk = tid < 4 ? rhs[P.kb + tid] : S[(size_t)(P.kb + mm) * ld + P.kb + q];
        }
    }
    if (skip_step(st)) return;
    TLS(0);
    const unsigned spin_lim = g_spin_limit;
    const unsigned epoch = Bw.flags[0] + 1;
    // block i's Gram of x (Bp) published by helper B (NH = 2) / H (NH = 1): the root sums them all
    unsigned* gram_f = NH == 2 ? Bw.flags + 16 + 3 * nblk : Bw.flags + 16;
    // this block's published panels, by epoch parity (flag-free: F stores, the helpers poll the values)
    double* pg = Bw.Cf + ((epoch & 1) ? (size_t)nblk * PANEL_DOUBLES : 0) + (size_t)i * PANEL_DOUBLES;
    double* pg_next = Bw.Cf + ((epoch & 1) ? 0 : (size_t)nblk * PANEL_DOUBLES) + (size_t)i * PANEL_DOUBLES;
    const int s_i = 1 << mi;
    const bool has_r = !root && i + s_i < nblk;
    const bool has_l = !root && i - s_i >= 0;
    if (role == 0) {
        // ================= F: D_i, pivot side of the factorization
        FLds& L = *reinterpret_cast<FLds*>(smem);
        {
            // every load was issued before the first LDS store (clamped addresses, selects after): the level-0
            // factorization starts one memory round trip after the launch, not eight
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int e = tid + TPB_E * q, r = e >> 6, c = e & 63;
                const bool ok = c <= r && r < G_DOF && b0 + r < nd;
                L.T[r * BLD + c] = ok ? pre[q] : (r == c ? 1.0 : 0.0);
            }
        }
        if (tid < 12) L.sync[tid] = 0;
        {  // the next epoch's panel slot starts empty (the entries a panel writes: lower tiles, stored
           // column-major, W, 1/diag)
            unsigned long long* nx = reinterpret_cast<unsigned long long*>(pg_next);
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                if (lower_tile_cm(tid + TPB_E * q)) nx[tid + TPB_E * q] = BCR_Y_EMPTY;
            nx[BB * BB + tid] = BCR_Y_EMPTY;
            nx[BB * BB + TPB_E + tid] = BCR_Y_EMPTY;
            if (tid < BB) nx[BB * BB + 4 * 256 + tid] = BCR_Y_EMPTY;
        }
        // survived levels: D_i -= XR_a^T XR_a + XL_b^T XL_b, pulled row block by row block from the rows the
        // eliminated neighbours' helpers publish (Pull); lower tiles wq and wq + 8 on wave wq
        for (int m = 0; m < mi; ++m) {
            const int s = 1 << m, a = i - s, b = i + s;
            PullSrc<2, 0> ps;
            ps.w[0] = a >= 0 ? pub_xr(Bw, epoch) + (size_t)a * BSZ : nullptr;
            ps.w[1] = b < nblk ? pub_xl(Bw, epoch) + (size_t)b * BSZ : nullptr;
            ps.x[0] = nullptr;
            const int wq = __builtin_amdgcn_readfirstlane(wave);
            int tib[2], tjb[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                int t = wq + NWE * q, ib = 0;
                while (t > ib) { t -= ib + 1; ++ib; }
                tib[q] = ib;
                tjb[q] = t;
            }
            d4b acc[2] = {d4b{0.0, 0.0, 0.0, 0.0}, d4b{0.0, 0.0, 0.0, 0.0}};
            Pull<2, 0> pl;
            pl.issue(ps, 0);
            for (int kb = 0; kb < 4; ++kb) {
                // the probe only for the first row block (the level's long wait): the later ones arrive at the
                // producers' panel pace, and 4 values per thread are polled directly
                if (!pl.commit(ps, kb, L.sg, &L.ok, spin_lim, kb == 0)) {
                    if (tid == 0) raise_flag(flag, FLAG_TIMEOUT);
                    return;
                }
                if (kb < 3) pl.issue(ps, kb + 1);
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    if (wq + NWE * q >= 10) continue;
#pragma unroll
                    for (int src = 0; src < 2; ++src) {
                        if (!ps.w[src]) continue;
                        const double* sgs = L.sg + src * SG_W;
                        double av[4], bv[4];
#pragma unroll
                        for (int s4 = 0; s4 < 4; ++s4) {
                            av[s4] = sgs[(4 * s4 + kk) * SG_LD + 16 * tib[q] + rr];
                            bv[s4] = sgs[(4 * s4 + kk) * SG_LD + 16 * tjb[q] + rr];
                        }
#pragma unroll
                        for (int s4 = 0; s4 < 4; ++s4) acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc[q], 0, 0, 0);
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                if (wq + NWE * q >= 10) continue;
#pragma unroll
                for (int g = 0; g < 4; ++g) L.T[(16 * tib[q] + kk + 4 * g) * BLD + 16 * tjb[q] + rr] -= acc[q][g];
            }
        }
        __syncthreads();
        TLS(1);
        // Look-ahead factorization with wave roles and LDS flags instead of workgroup barriers:
        //   wave 0     pivot chain of the tall column block kb (rows 16 kb..63, all 64 lanes): the
        //              diagonal tile and the row panels below it in one pass (no L_kk^-1 on this path)
        //   waves 1-3  the critical update of column block kb + 1 by panel kb (one tile each), which
        //              wave 0 waits for before its next chain
        //   wave 5     W_kb = L_kk^-1 and the publication of panel kb (L tiles, W_kb, 1/diag) + flag
        //   waves 6-7  the non-critical trailing tiles (panel 0 on column blocks 2, 3; panel 1 on 3)
        //   wave 4     idle (it shares wave 0's SIMD: its f64 work would slow the pivot chain)
        // Every tile's updates run in panel order on one wave or behind a counter.
        double* T = L.T;
        int* const sync = L.sync;  // [0] panels factored, [1..4] crit[kb], [5..8] trailing done per column block
        auto lds_ld = [&](int k) { return __hip_atomic_load(sync + k, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); };
        auto spin_ge = [&](int k, int v) {
            unsigned n = 0;
            while (lds_ld(k) < v) {
                __builtin_amdgcn_s_sleep(1);
                if (++n > SPIN_LIMIT) return false;
            }
            return true;
        };
        auto tile_sub = [&](int ii, int jj, int p) {  // T(ii,jj) -= L(ii,p) L(jj,p)^T
            const d4b acc = mfma16_abt(T + (16 * ii) * BLD + 16 * p, BLD, T + (16 * jj) * BLD + 16 * p, BLD, rr, kk);
#pragma unroll
            for (int g = 0; g < 4; ++g) T[(16 * ii + kk + 4 * g) * BLD + 16 * jj + rr] -= acc[g];
        };
        auto signal = [&](int k) {  // one add per wave, after the wave's LDS stores
            if (lane == 0) __hip_atomic_fetch_add(sync + k, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        };
        bool ok = true;
        if (wave == 0) {
            bool bad = false;
            for (int kb = 0; kb < 4; ++kb) {
                if (kb > 0 && !spin_ge(1 + kb - 1, 4 - kb)) { ok = false; break; }  // column block kb updated
                TLS(17 + 3 * kb);
                const int r = lane, row = 16 * kb + r;
                const bool live = row < BB;
                double a[16];
#pragma unroll
                for (int c = 0; c < 16; ++c) a[c] = live ? T[row * BLD + 16 * kb + c] : 0.0;
                double my_inv = 0.0;
                double dn = bcast_b(a[0], 0);
                // shader-clock stamps around the first and last chains' pivots (slots 28-31): cycles per pivot in
                // the kernel, beside the micro-benchmark's (tools/pivot_chain_bench.hip)
                if constexpr (STAMP) if (lane == 0 && (kb == 0 || kb == 3)) tl[32 * bid + 28 + (kb ? 2 : 0)] = bcr_stamp();
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    // d = current pivot; y ~ d^-1/2 (v_rsq_f64), one Newton step folded into l = a y (1 + e/2)
                    const double d = dn;
                    bad = bad || !(d > 0.0 && d < INFINITY);
                    const double y = __builtin_amdgcn_rsq(d);
                    const double e = __builtin_fma(-d * y, y, 1.0);
                    const double l = __builtin_fma(0.5 * a[j] * y, e, a[j] * y);
                    my_inv = (r == j) ? __builtin_fma(0.5 * y, e, y) : my_inv;
                    a[j] = l;
                    if (j < 15) {
                        // next pivot first: on lane j + 1, bcast(l, j + 1) == l
                        dn = bcast_b(__builtin_fma(-l, l, a[j + 1]), j + 1);
#pragma unroll
                        for (int k = j + 1; k < 16; ++k) a[k] = __builtin_fma(-l, bcast_b(l, k), a[k]);
                    }
                }
                if constexpr (STAMP) if (lane == 0 && (kb == 0 || kb == 3)) tl[32 * bid + 29 + (kb ? 2 : 0)] = bcr_stamp();
                if (live)
#pragma unroll
                    for (int c = 0; c < 16; ++c) T[row * BLD + 16 * kb + c] = (r >= 16 || c <= r) ? a[c] : 0.0;
                if (r < 16) {
                    L.rdiag[16 * kb + r] = my_inv;
#pragma unroll
                    for (int c = 0; c < 16; ++c) L.Lcm[kb][c * 16 + r] = a[c];  // strictly-lower part is what W reads
                }
                if (lane == 0) __hip_atomic_store(sync, kb + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                // publish the panel's L tiles straight from the chain's registers (column-major: one
                // coalesced row of 64 per store); W_kb and 1/diag follow from wave 5
                if (live)
#pragma unroll
                    for (int c = 0; c < 16; ++c) st_pub(pg + (16 * kb + c) * BB + row, (r >= 16 || c <= r) ? a[c] : 0.0);
                TLS(16 + 3 * kb);
            }
            if (bad) raise_flag(flag, FLAG_NOT_PD);
        } else if (wave <= 3) {
            for (int kb = 0; kb + wave <= 3 && kb < 3; ++kb) {
                if (!spin_ge(0, kb + 1)) { ok = false; break; }
                // earlier panels' (trailing) updates of column block kb + 1: 2 tiles each for blocks 2, 3
                if (kb + 1 >= 2 && !spin_ge(5 + kb + 1, 2)) { ok = false; break; }
                tile_sub(kb + wave, kb + 1, kb);
                signal(1 + kb);
            }
        } else if (wave == 6) {  // tile (3,3): panel 0, then panel 1
            for (int p = 0; p < 2 && ok; ++p) {
                if (!spin_ge(0, p + 1)) { ok = false; break; }
                tile_sub(3, 3, p);
                signal(5 + 3);
            }
        } else if (wave == 7) {  // tiles (2,2), (3,2): panel 0
            if (!spin_ge(0, 1)) ok = false;
            else {
                tile_sub(2, 2, 0);
                tile_sub(3, 2, 0);
                __hip_atomic_fetch_add(sync + 5 + 2, lane == 0 ? 2 : 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        } else if (wave == 5) {
            for (int kb = 0; kb < 4; ++kb) {
                if (!spin_ge(0, kb + 1)) { ok = false; break; }
                // W_kb = L_kk^-1, column `lane` per lane (lanes 0-15): forward substitution of e_lane against the
                // column-major diagonal tile (uniform LDS reads, contiguous per column), published straight from
                // registers (row m of W_kb: 16 consecutive doubles), then 1/diag (the panel's L tiles: wave 0)
                if (lane < 16) {
                    const double* Lc = L.Lcm[kb];
                    const double* rd = L.rdiag + 16 * kb;
                    double v[16];
#pragma unroll
                    for (int m = 0; m < 16; ++m) v[m] = (m == lane) ? 1.0 : 0.0;
#pragma unroll
                    for (int m = 0; m < 16; ++m) {
                        v[m] *= rd[m];
#pragma unroll
                        for (int j = m + 1; j < 16; ++j) v[j] = __builtin_fma(-Lc[m * 16 + j], v[m], v[j]);
                    }
#pragma unroll
                    for (int m = 0; m < 16; ++m) st_pub(pg + BB * BB + kb * 256 + m * 16 + lane, v[m]);
                    st_pub(pg + BB * BB + 4 * 256 + 16 * kb + lane, rd[lane]);
                }
                if constexpr (STAMP) if (lane == 0) tl[32 * bid + 2 + kb] = realtime_now();
            }
        }
        if (!ok) raise_flag(flag, FLAG_TIMEOUT);
        return;
    }
    // ================= helpers: survived levels (pulls), panel application, back-substitution
    const bool roleA = NH == 2 && role == 1;  // NH = 2: XL side (exits after its forward substitution)
    const bool roleB = NH == 1 || role == 2;  // owns XR, the Gram and the back-substitution
    if (root && roleA) return;                // the root has only the x columns (helper B)
    HLds& L = *reinterpret_cast<HLds*>(smem);
    // the wave index as a scalar: role and tile branches below are uniform
    const int wu = __builtin_amdgcn_readfirstlane(wave);
    // rows this helper publishes for the next level (pull hand-off): XL if the block has a left neighbour,
    // XR if it has a right one, x if either (helper A / H; helper B's x is the same)
    const bool pubL = !root && (NH == 1 || roleA) && has_l;
    const bool pubR = !root && roleB && has_r;
    const bool pubX = !root && (NH == 1 || roleA) && (has_l || has_r);
    double* const xl_pub = pub_xl(Bw, epoch) + (size_t)i * BSZ;
    double* const xr_pub = pub_xr(Bw, epoch) + (size_t)i * BSZ;
    double* const x_pub = pub_x(Bw, epoch) + (size_t)i * RSZ;
    // Border without a second pass (was k_bcr_border): every block's helper B publishes the Gram of its
    // forward-solved x = [b_a | B]; the root sums them with its own, solves the 4x4 border system before its
    // back-substitution and publishes y_k with y_root, so each block applies its camera step right after its
    // own back-substitution (no wait for every block).
    // This block's slots of the next epoch's buffers start empty (y, published rows).
    if (roleB) reinterpret_cast<unsigned long long*>(ybuf(Bw, epoch + 1))[(size_t)i * RSZ + tid] = BCR_Y_EMPTY;
    {
        unsigned long long* nl = reinterpret_cast<unsigned long long*>(pub_xl(Bw, epoch + 1) + (size_t)i * BSZ);
        unsigned long long* nr = reinterpret_cast<unsigned long long*>(pub_xr(Bw, epoch + 1) + (size_t)i * BSZ);
        if (pubL)
#pragma unroll
            for (int q = 0; q < NQ; ++q) nl[tid + TPB_E * q] = BCR_Y_EMPTY;
        if (pubR)
#pragma unroll
            for (int q = 0; q < NQ; ++q) nr[tid + TPB_E * q] = BCR_Y_EMPTY;
        if (pubX) reinterpret_cast<unsigned long long*>(pub_x(Bw, epoch + 1) + (size_t)i * RSZ)[tid] = BCR_Y_EMPTY;
    }
    // level-0 inputs (loaded in the prologue, before the LM-state check)
    const double bkv = pre_bk;
    {
        const bool has_r0 = i + 1 < nblk;
        const double* xv = pre;
        const int r = tid >> 3, c = tid & 7;
        const double rv = pre_r;
        if (mi == 0) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int e = tid + TPB_E * q, rq = e >> 6, cq = e & 63;
                if (NH == 1 || roleA) {
                    const bool okl = i >= 1 && rq < G_DOF && b0 + rq < nd && cq < G_DOF;
                    L.X[rq * XW + cq] = okl ? xv[q] : 0.0;
                }
                if (NH == 1 || roleB) {
                    const int b1 = b0 + G_DOF;
                    const bool okr = has_r0 && rq < G_DOF && b1 + rq < nd && cq < G_DOF;
                    L.X[cq * XW + BB + rq] = okr ? xv[NQX - NQ + q] : 0.0;
                }
            }
        }
        L.X[r * XW + 2 * BB + c] = rv;
    }
    if (root && tid < 14) L.bk[tid] = bkv;
    // Survived levels: the Schur terms of the level's eliminated neighbours a = i - s, b = i + s, pulled row
    // block by row block (Pull; staging in L / rdiag / W, which hold nothing before the first panel):
    //   x -= XR_a^T x_a + XL_b^T x_b              (x waves: row block wu - xw0; one chain over the row blocks)
    //   last level: XL = -XR_a^T XL_a (helper A / H waves 0-3: column tile wu)
    //               XR = -XL_b^T XR_b (helper B waves 0-3 / H waves 4-7: column tile wu & 3)
    {
        static_assert(4 * SG_W + 2 * RSZ / 4 <= (int)((offsetof(HLds, Bl) - offsetof(HLds, L)) / sizeof(double)),
                      "pulled row blocks fit L / rdiag / W");
        double* const sg = L.L;
        const double* const sx = sg + 4 * SG_W;
        constexpr int xw0 = NH == 2 ? 4 : 0;
        const bool xwave = wu >= xw0 && wu < xw0 + 4;
        const int xr = wu - xw0;
        const bool sideA = NH == 1 ? wu < 4 : roleA;                    // fill side of this wave
        const bool fwave = NH == 1 ? true : wu < 4;                      // waves holding a fill column tile
        for (int m = 0; m < mi; ++m) {
            const int s = 1 << m, a = i - s, b = i + s;
            const bool ha = a >= 0, hb = b < nblk;
            const bool last = m == mi - 1 && !root;
            const bool fa = last && has_l && (NH == 1 || roleA), fb = last && has_r && roleB;
            PullSrc<4, 2> ps;
            ps.w[0] = ha ? pub_xr(Bw, epoch) + (size_t)a * BSZ : nullptr;
            ps.w[1] = hb ? pub_xl(Bw, epoch) + (size_t)b * BSZ : nullptr;
            ps.w[2] = fa ? pub_xl(Bw, epoch) + (size_t)a * BSZ : nullptr;
            ps.w[3] = fb ? pub_xr(Bw, epoch) + (size_t)b * BSZ : nullptr;
            ps.x[0] = ha ? pub_x(Bw, epoch) + (size_t)a * RSZ : nullptr;
            ps.x[1] = hb ? pub_x(Bw, epoch) + (size_t)b * RSZ : nullptr;
            const bool fon = fwave && (sideA ? fa : fb);
            d4b xacc = {0.0, 0.0, 0.0, 0.0};
            d4b facc[4];
#pragma unroll
            for (int ii = 0; ii < 4; ++ii) facc[ii] = d4b{0.0, 0.0, 0.0, 0.0};
            Pull<4, 2> pl;
            pl.issue(ps, 0);
            for (int kb = 0; kb < 4; ++kb) {
                if (!pl.commit(ps, kb, sg, &L.ok, spin_lim, true)) {
                    if (tid == 0) raise_flag(flag, FLAG_TIMEOUT);
                    return;
                }
                if (kb < 3) pl.issue(ps, kb + 1);
                if (xwave) {
#pragma unroll
                    for (int src = 0; src < 2; ++src) {
                        if (!(src ? hb : ha)) continue;
                        double av[4], bv[4];
#pragma unroll
                        for (int s4 = 0; s4 < 4; ++s4) {
                            av[s4] = sg[src * SG_W + (4 * s4 + kk) * SG_LD + 16 * xr + rr];
                            const double xb_ = sx[src * RSZ / 4 + (4 * s4 + kk) * RC + (rr & 7)];
                            bv[s4] = rr < RC ? xb_ : 0.0;
                        }
#pragma unroll
                        for (int s4 = 0; s4 < 4; ++s4) xacc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], xacc, 0, 0, 0);
                    }
                }
                if (fon) {
                    const double* sa = sg + (sideA ? 0 : 1) * SG_W;  // XR_a (A) / XL_b (B): row tiles of the fill
                    const double* sb = sg + (sideA ? 2 : 3) * SG_W;  // XL_a (A) / XR_b (B): its column tile
                    double av[4][4], bv[4];
#pragma unroll
                    for (int s4 = 0; s4 < 4; ++s4) {
                        bv[s4] = sb[(4 * s4 + kk) * SG_LD + 16 * (wu & 3) + rr];
#pragma unroll
                        for (int ii = 0; ii < 4; ++ii) av[ii][s4] = sa[(4 * s4 + kk) * SG_LD + 16 * ii + rr];
                    }
#pragma unroll
                    for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
                        for (int ii = 0; ii < 4; ++ii)
                            facc[ii] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[ii][s4], bv[s4], facc[ii], 0, 0, 0);
                }
            }
            if (xwave && rr < RC)
#pragma unroll
                for (int g = 0; g < 4; ++g) L.X[(16 * xr + kk + 4 * g) * XW + 2 * BB + rr] -= xacc[g];
            if (last && fwave) {
                // this side's coupling of level mi (zero without the neighbour)
                const int col = sideA ? 16 * (wu & 3) : BB + 16 * (wu & 3);
                const bool f = sideA ? fa : fb;
#pragma unroll
                for (int ii = 0; ii < 4; ++ii)
#pragma unroll
                    for (int g = 0; g < 4; ++g) L.X[(16 * ii + kk + 4 * g) * XW + col + rr] = f ? -facc[ii][g] : 0.0;
            }
        }
    }
    if (root) {
        // the other blocks' Grams (published by their helpers B after their forward substitution), summed in
        // block order; overlaps F's first panel
        if (!wait_all_eq(gram_f, nblk, epoch, &L.ok, i)) {
            if (tid == 0) raise_flag(flag, FLAG_TIMEOUT);
            return;
        }
        double gsum = 0.0;
        for (int j0 = 0; j0 < nblk; j0 += BP_CHUNK) {
            const int nb = nblk - j0 < BP_CHUNK ? nblk - j0 : BP_CHUNK;
            for (int e = tid; e < 25 * nb; e += TPB_E) L.bpl[e] = j0 + e / 25 == i ? 0.0 : ld_pub(Bw.Bp + (size_t)(j0 + e / 25) * 32 + e % 25);
            __syncthreads();
            if (tid < 25)
                for (int b = 0; b < nb; ++b) gsum += L.bpl[25 * b + tid];
            __syncthreads();
        }
        if (tid < 25) L.bred[tid] = gsum;
    }
    TLS(1);
    double* X = root ? L.X + 2 * BB : L.X;
    const int ncol = root ? RC : XC;
    // Column-tile ownership (helper_cb): each wave keeps its column tiles of X in registers
    // (MFMA accumulator layout x[g] = X[16 ii + kk + 4 g][16 cb + rr], which is also the B-operand
    // layout of a 16x16x4 step), so the forward substitution of its columns (X_kb <- W_kb X_kb,
    // X_ii -= L(ii,kb) X_kb) needs no barrier and no LDS round trip; the finished row block kb is stored
    // to LDS (the back-substitution's copy, the Gram) and published for the next level (pull hand-off).
    constexpr int MAXOWN = NH == 1 ? 2 : 1;
    int own_cb[MAXOWN];
    own_cb[0] = helper_cb<NH>(roleB, wu, root);
    if constexpr (MAXOWN > 1) own_cb[1] = (!root && wu == 0) ? 8 : -1;
    d4b xt[MAXOWN][4];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MAXOWN; ++j) {
        const int cb = own_cb[j];
        const bool colok = cb >= 0 && 16 * cb + rr < ncol;
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
            for (int g = 0; g < 4; ++g) xt[j][ii][g] = colok ? X[(16 * ii + kk + 4 * g) * XW + 16 * cb + rr] : 0.0;
    }
    // the Gram x^T x (5 x 5 of the 8 x columns, row block by row block) on one wave of helper B / H
    const bool gram_on = !root && roleB && wu == (NH == 2 ? 6 : 3);
    d4b gacc = {0.0, 0.0, 0.0, 0.0};
    // Panel data of panel kb -> registers, then LDS. The loads of panel kb + 1 are issued right after
    // the X update of panel kb, so their latency hides under the contributions; values that were still
    // empty (the factor workgroup had not stored them yet) are polled again at the panel's commit.
    unsigned long long pv[4];
    auto paddr = [&](int k, int u) -> const double* {  // this thread's value u of panel k (nullptr: none)
        if (u < 2) {  // L tiles (ii, k), ii >= k, column-major: thread -> (row, column) = (16 k + e % nr, 16 k + e / nr)
            const int e = tid + TPB_E * u, nr = 64 - 16 * k;
            return e < (4 - k) * 256 ? pg + (16 * k + e / nr) * BB + 16 * k + e % nr : nullptr;
        }
        if (u == 2) return tid < 256 ? pg + BB * BB + k * 256 + tid : nullptr;
        return tid < 16 ? pg + BB * BB + 4 * 256 + 16 * k + tid : nullptr;
    };
    auto issue = [&](int k) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double* a = paddr(k, u);
            pv[u] = a ? ld_u64(a) : 0ull;
        }
    };
    auto commit = [&](int k) -> int {  // polls the values still empty, then stores them to LDS
        int ok = 1;
        for (unsigned n = 0;; ++n) {
            bool pend = false;
#pragma unroll
            for (int u = 0; u < 4; ++u) pend = pend || pv[u] == BCR_Y_EMPTY;
            if (!pend) break;
            if (n > SPIN_LIMIT) { ok = 0; break; }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (pv[u] == BCR_Y_EMPTY) pv[u] = ld_u64(paddr(k, u));
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = tid + TPB_E * u, nr = 64 - 16 * k;
            if (e < (4 - k) * 256) L.L[(16 * k + e % nr) * BLD + 16 * k + e / nr] = __longlong_as_double((long long)pv[u]);
        }
        if (tid < 256) L.W[k][tid] = __longlong_as_double((long long)pv[2]);
        if (tid < 16) L.rdiag[16 * k + tid] = __longlong_as_double((long long)pv[3]);
        return ok;
    };
    issue(0);
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
        TLS(2 + 2 * kb);
        if (!__syncthreads_and(commit(kb))) {
            if (tid == 0) raise_flag(flag, FLAG_TIMEOUT);
            return;
        }
        TLS(16 + 4 * kb);
        if (NH == 2 && wu == 4 + kb) {  // x_kb <- W_kb x_kb (LDS row block, 8 valid columns)
            double aw[4], bx[4];
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                aw[s4] = L.W[kb][rr * 16 + 4 * s4 + kk];
                bx[s4] = rr < RC ? L.X[(16 * kb + 4 * s4 + kk) * XW + 2 * BB + rr] : 0.0;
            }
            d4b w = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) w = __builtin_amdgcn_mfma_f64_16x16x4f64(aw[s4], bx[s4], w, 0, 0, 0);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (rr < RC)
#pragma unroll
                for (int g = 0; g < 4; ++g) L.X[(16 * kb + kk + 4 * g) * XW + 2 * BB + rr] = w[g];
            if (pubX && rr < RC)  // helper A: x row block kb for the next level
#pragma unroll
                for (int g = 0; g < 4; ++g) st_pub(x_pub + (16 * kb + kk + 4 * g) * RC + rr, w[g]);
        }
#pragma unroll
        for (int j = 0; j < MAXOWN; ++j) {
            const int cb = own_cb[j];
            if (cb < 0) continue;
            // operands first, then the three update chains interleaved (independent accumulators)
            double aw[4], al[3][4];
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) aw[s4] = L.W[kb][rr * 16 + 4 * s4 + kk];
#pragma unroll
            for (int ii = kb + 1; ii < 4; ++ii)
#pragma unroll
                for (int s4 = 0; s4 < 4; ++s4) al[ii - kb - 1][s4] = -L.L[(16 * ii + rr) * BLD + 16 * kb + 4 * s4 + kk];
            d4b w = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) w = __builtin_amdgcn_mfma_f64_16x16x4f64(aw[s4], xt[j][kb][s4], w, 0, 0, 0);
            xt[j][kb] = w;
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
                for (int ii = kb + 1; ii < 4; ++ii)
                    xt[j][ii] = __builtin_amdgcn_mfma_f64_16x16x4f64(al[ii - kb - 1][s4], w[s4], xt[j][ii], 0, 0, 0);
            if (16 * cb + rr < ncol)
#pragma unroll
                for (int g = 0; g < 4; ++g) X[(16 * kb + kk + 4 * g) * XW + 16 * cb + rr] = w[g];
            // the finished row block for the next level's pulls (no drain: the consumers poll the values)
            if (cb < 4 ? pubL : (cb < 8 ? pubR : (pubX && rr < RC))) {
                double* dst = cb < 4 ? xl_pub + 16 * cb : (cb < 8 ? xr_pub + 16 * (cb - 4) : x_pub);
                const int ldd = cb < 8 ? BB : RC;
#pragma unroll
                for (int g = 0; g < 4; ++g) st_pub(dst + (16 * kb + kk + 4 * g) * ldd + rr, w[g]);
            }
        }
        __syncthreads();
        TLS(17 + 4 * kb);
        // next panel's loads in flight (values still empty are polled at its commit)
        if (kb < 3) issue(kb + 1);
        if (NH == 2 && wu > 4 + kb) {  // x_ii -= L(ii,kb) x_kb, ii = wave - 4
            const int ii = wu - 4;
            double al[4], bx[4];
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                al[s4] = -L.L[(16 * ii + rr) * BLD + 16 * kb + 4 * s4 + kk];
                bx[s4] = rr < RC ? L.X[(16 * kb + 4 * s4 + kk) * XW + 2 * BB + rr] : 0.0;
            }
            d4b acc;
#pragma unroll
            for (int g = 0; g < 4; ++g) acc[g] = rr < RC ? L.X[(16 * ii + kk + 4 * g) * XW + 2 * BB + rr] : 0.0;
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(al[s4], bx[s4], acc, 0, 0, 0);
            if (rr < RC)
#pragma unroll
                for (int g = 0; g < 4; ++g) L.X[(16 * ii + kk + 4 * g) * XW + 2 * BB + rr] = acc[g];
        }
        if (gram_on) {
            double xv[4];
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) {
                const double v = L.X[(16 * kb + 4 * s4 + kk) * XW + 2 * BB + (rr & 7)];
                xv[s4] = rr < RC ? v : 0.0;
            }
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4) gacc = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[s4], xv[s4], gacc, 0, 0, 0);
        }
        if constexpr (STAMP) __syncthreads();
        TLS(3 + 2 * kb);
    }
    __syncthreads();
    if (root) {
        double* Yl = L.yt;
        {
            const int r = tid >> 3, c = tid & 7;
            Yl[tid] = L.X[r * XW + 2 * BB + c];
        }
        __syncthreads();
        // the root's Gram z^T z: 25 entries x 4 row quarters (fixed-order sums)
        if (tid < 100) {
            const int q = tid >> 2, part4 = tid & 3, gr = q / 5, gc = q % 5;
            double acc = 0.0;
#pragma unroll
            for (int k = 16 * part4; k < 16 * part4 + 16; ++k) acc = __builtin_fma(Yl[k * RC + gr], Yl[k * RC + gc], acc);
            L.red[tid] = acc;
        }
        __syncthreads();
        // border system on one lane of wave 4 while waves 0-3 back-solve [u | V] = Cf^-T z
        if (tid == 256) {
            double g20[20];  // (B^T A^-1 [b_a | B])[m][c] = G[1 + m][c]
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int cc = 0; cc < 5; ++cc) {
                    const int q = (1 + m) * 5 + cc;
                    g20[m * 5 + cc] = L.bred[q] + (((L.red[4 * q] + L.red[4 * q + 1]) + L.red[4 * q + 2]) + L.red[4 * q + 3]);
                }
            bool bad = false;
            border_solve4(L.bk, g20, L.byk, bad);
            if (bad) raise_flag(flag, FLAG_NOT_PD);
        }
        trsm_t_lanes(L.L, L.rdiag, Yl);  // ends with a barrier
        st_pub(ybuf(Bw, epoch) + (size_t)i * RSZ + tid, ((tid & 7) == 5 && tid < 4 * RC) ? L.byk[tid >> 3] : Yl[tid]);
        // (the next call's epoch is advanced by k_final, after every workgroup of this launch has exited)
        TLS(14);
        block_step(st, P, rhs, c, scale, camdata, lin, delta, part, i, true, Yl, L.byk, L.bybl);
        return;
    }
    if (roleA) {  // helper A's rows are all published
        TLS(10);
        TLS(11);
        return;
    }
    // the Gram x^T x (5 x 5) -> Bp[i], published with its flag (the root sums every block's)
    if (gram_on)
#pragma unroll
        for (int g = 0; g < 4; ++g)
            if (kk + 4 * g < 5 && rr < 5) st_pub(Bw.Bp + (size_t)i * 32 + (kk + 4 * g) * 5 + rr, gacc[g]);
    publish_flag(gram_f + i, epoch);
    TLS(10);
    if (NH == 2) {
        // the back-substitution needs XL: helper A's published rows (out long ago; polled value by value)
        const double* xs = pub_xl(Bw, epoch) + (size_t)i * BSZ;
        unsigned long long xv[BSZ / TPB_E];
#pragma unroll
        for (int u = 0; u < BSZ / TPB_E; ++u) xv[u] = has_l ? ld_u64(xs + tid + TPB_E * u) : 0ull;
        int okp = 1;
        for (unsigned n = 0;; ++n) {
            bool pend = false;
#pragma unroll
            for (int u = 0; u < BSZ / TPB_E; ++u) pend = pend || xv[u] == BCR_Y_EMPTY;
            if (!pend) break;
            if (n > SPIN_LIMIT) { okp = 0; break; }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int u = 0; u < BSZ / TPB_E; ++u)
                if (xv[u] == BCR_Y_EMPTY) xv[u] = ld_u64(xs + tid + TPB_E * u);
        }
#pragma unroll
        for (int u = 0; u < BSZ / TPB_E; ++u) {
            const int e = tid + TPB_E * u;
            L.X[(e >> 6) * XW + (e & 63)] = __longlong_as_double((long long)xv[u]);
        }
        if (!__syncthreads_and(okp)) {
            if (tid == 0) raise_flag(flag, FLAG_TIMEOUT);
            return;
        }
        TLS(11);
    }
    // ---- off the critical path: [P | Q | u] = Cf^-T [XL | XR | x]; then y_i = u - P y_{i-s} - Q y_{i+s}
    trsm_lower64_t(L.L, L.rdiag, L.X, XW, XC);
    {
        // the neighbours' y rows and y_k, polled value by value (bounded)
        const double* Yb = ybuf(Bw, epoch);
        const double* pl = Yb + (size_t)(i - s_i) * RSZ + tid;
        const double* pr = Yb + (size_t)(i + s_i) * RSZ + tid;
        const double* pk = Yb + (size_t)Bw.vroot * RSZ + tid * RC + 5;
        unsigned long long ul = has_l ? ld_u64(pl) : 0ull, ur = has_r ? ld_u64(pr) : 0ull, uk = tid < 4 ? ld_u64(pk) : 0ull;
        int okp = 1;
        unsigned n = 0;
        while (ul == BCR_Y_EMPTY || ur == BCR_Y_EMPTY || uk == BCR_Y_EMPTY) {
            __builtin_amdgcn_s_sleep(1);
            if (ul == BCR_Y_EMPTY) ul = ld_u64(pl);
            if (ur == BCR_Y_EMPTY) ur = ld_u64(pr);
            if (uk == BCR_Y_EMPTY) uk = ld_u64(pk);
            if (++n > SPIN_LIMIT) { okp = 0; break; }
        }
        L.yl[tid] = __longlong_as_double((long long)ul);
        L.yr[tid] = __longlong_as_double((long long)ur);
        if (tid < 4) L.byk[tid] = __longlong_as_double((long long)uk);
        L.yt[tid] = L.X[(tid >> 3) * XW + 2 * BB + (tid & 7)];
        if (!__syncthreads_and(okp)) {
            if (tid == 0) raise_flag(flag, FLAG_TIMEOUT);
            return;
        }
    }
    TLS(12);
    {
        // y_i = u - P y_l - Q y_r on all 8 waves: wave w owns row block w & 3 and half (w >> 2) of the
        // 64-deep contraction (two 8-deep MFMA chains, operands loaded up front); the second half's
        // partials meet the first's in LDS, and the first-half waves store the finished rows straight
        // from registers (the next hop's consumers poll them)
        const int rb = wave & 3, kh = wave >> 2;
        double al[8], ar[8], bl[8], br[8];
#pragma unroll
        for (int s4 = 0; s4 < 8; ++s4) {
            const int k = 8 * kh + s4;
            const double* row = L.X + (16 * rb + rr) * XW + 4 * k + kk;
            al[s4] = has_l ? row[0] : 0.0;
            ar[s4] = has_r ? row[BB] : 0.0;
            bl[s4] = has_l && rr < RC ? L.yl[(4 * k + kk) * RC + rr] : 0.0;
            br[s4] = has_r && rr < RC ? L.yr[(4 * k + kk) * RC + rr] : 0.0;
        }
        d4b acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s4 = 0; s4 < 8; ++s4) {
            if (has_l) acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(al[s4], bl[s4], acc0, 0, 0, 0);
            if (has_r) acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[s4], br[s4], acc1, 0, 0, 0);
        }
        double* part2 = L.bpl;  // 64 x RC partials of the second half
        if (kh == 1 && rr < RC)
#pragma unroll
            for (int g = 0; g < 4; ++g) part2[(16 * rb + kk + 4 * g) * RC + rr] = acc0[g] + acc1[g];
        __syncthreads();
        if (kh == 0 && rr < RC) {
            double* yout = ybuf(Bw, epoch) + (size_t)i * RSZ;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int e = (16 * rb + kk + 4 * g) * RC + rr;
                const double v = L.yt[e] - ((acc0[g] + acc1[g]) + part2[e]);
                st_pub(yout + e, v);
                L.yt[e] = v;
            }
        }
    }
    __syncthreads();
    TLS(14);
    block_step(st, P, rhs, c, scale, camdata, lin, delta, part, i, false, L.yt, L.byk, L.bybl);
}

#undef TLS

// ---- one-block windows (<= 10 active cameras: the reference's TUM windows) -------------------------------------
// The whole reduced system — the 6 nac camera dofs and the 4 intrinsics rows that follow them in S, n = 6 nac + 4
// <= 64 — is one dense SPD block. One workgroup loads it into LDS (identity pad), factors it with the split
// kernel's pivot chain on wave 0 and the trailing tiles on the other waves' f64 MFMA, solves L z = b and
// L^T y = z on wave 0 (lane = row, v_readlane broadcasts, the next column prefetched) and applies the camera /
// intrinsics step (block_step with y in the u column): no border system, no cross-workgroup hand-off — the split
// kernel's factor / helper pair spends ~5 us of a ~21 us one-block launch on those (C1 stamps).
static constexpr int TPB_D1 = 512;
// Wave roles after the load (k_bcr_split's factor workgroup, plus the solve):
//   wave 0     the pivot chain of column block kb once its critical update is in (LDS flags, no barriers)
//   waves 1-3  the critical update of column block kb + 1 by panel kb (one tile each)
//   waves 6-7  the other trailing tiles (panel 0 on column blocks 2, 3; panel 1 on 3)
//   wave 5     W_kb = L_kk^-1 and the forward substitution's block kb as each panel lands (lane = row), then the
//              backward substitution by blocks and the camera / intrinsics step from its prefetched operands
//   wave 4     idle (it shares wave 0's SIMD)
// STAMP: s_memrealtime after each phase into tl[0..8] (loaded, 4 panels, forward, backward, step)
template <bool STAMP>
__global__ __launch_bounds__(TPB_D1) void k_bcr_dense1(const LmState* __restrict__ st, DevProblem P,
                                                      const double* __restrict__ S, double* __restrict__ rhs,
                                                      int* __restrict__ flag, BaConsts c,
                                                      const double* __restrict__ scale,
                                                      const double* __restrict__ camdata,
                                                      const double* __restrict__ lin, double* __restrict__ delta,
                                                      double* __restrict__ part, unsigned long long* __restrict__ tl) {
#define D1S(k)                                                                      \
    do {                                                                            \
        if constexpr (STAMP) if ((threadIdx.x & 63) == 0) tl[(k)] = realtime_now(); \
    } while (0)
    if constexpr (STAMP) if (threadIdx.x == 0) tl[9] = realtime_now();
    __shared__ __attribute__((aligned(16))) double T[BB * BLD];
    __shared__ double rdg[BB];
    __shared__ double Wm[4][256];          // W_kb = L_kk^-1, row-major
    __shared__ double vr[BB], vz[BB];      // wave 5's broadcast rows of the blocked triangular solves
    __shared__ int sync[12];               // [0] panels factored, [1..3] critical updates, [5..8] trailing per column
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, rr = lane & 15, kk = lane >> 4;
    const int n = P.kb + 4;  // camera dofs, then the intrinsics rows (P.kb = 6 nac)
    const size_t ld = P.npad;
    // the lower triangle (every load in flight together: clamped addresses, selects after)
    {
        constexpr int NL = BB * BB / TPB_D1;
        double v[NL];
#pragma unroll
        for (int q = 0; q < NL; ++q) {
            const int e = tid + TPB_D1 * q, r = e >> 6, cc = e & 63;
            const bool ok = cc <= r && r < n;
            v[q] = S[ok ? (size_t)r * ld + cc : 0];
        }
        if (skip_step(st)) return;
#pragma unroll
        for (int q = 0; q < NL; ++q) {
            const int e = tid + TPB_D1 * q, r = e >> 6, cc = e & 63;
            T[r * BLD + cc] = (cc <= r && r < n) ? v[q] : (r == cc ? 1.0 : 0.0);
        }
    }
    if (tid < 12) sync[tid] = 0;
    // wave 5: rhs and the step's operands (cameras on lanes < nac, the intrinsics on lane BCR_CAMS), in flight
    // through the factorization
    const int cur = st->cur;
    const double radius = st->radius;
    CamStepOps cops;
    IntrStepOps iops;
    double b = 0.0;
    if (wave == 5) {
        if (lane < P.nac) load_cam_step_ops(P, cur, scale, camdata, lane, cops);
        if (lane == BCR_CAMS) load_intr_step_ops(P, cur, scale, lin, iops);
        b = lane < n ? rhs[lane] : 0.0;
    }
    __syncthreads();
    D1S(0);
    const unsigned spin_lim = g_spin_limit;
    auto lds_ld = [&](int k) { return __hip_atomic_load(sync + k, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); };
    auto spin_ge = [&](int k, int v) {
        unsigned cnt = 0;
        while (lds_ld(k) < v) {
            __builtin_amdgcn_s_sleep(1);
            if (++cnt > spin_lim) return false;
        }
        return true;
    };
    auto tile_sub = [&](int ii, int jj, int pn) {  // T(ii,jj) -= L(ii,pn) L(jj,pn)^T
        const d4b acc = mfma16_abt(T + (16 * ii) * BLD + 16 * pn, BLD, T + (16 * jj) * BLD + 16 * pn, BLD, rr, kk);
#pragma unroll
        for (int g = 0; g < 4; ++g) T[(16 * ii + kk + 4 * g) * BLD + 16 * jj + rr] -= acc[g];
    };
    auto signal = [&](int k) {
        if (lane == 0) __hip_atomic_fetch_add(sync + k, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    bool ok = true;
    if (wave == 0) {
        bool bad = false;
        for (int kb = 0; kb < 4; ++kb) {
            if (kb > 0 && !spin_ge(1 + kb - 1, 4 - kb)) { ok = false; break; }  // column block kb updated
            const int r = lane, row = 16 * kb + r;
            const bool live = row < BB;
            double a[16];
#pragma unroll
            for (int cc = 0; cc < 16; ++cc) a[cc] = live ? T[row * BLD + 16 * kb + cc] : 0.0;
            double my_inv = 0.0;
            double dn = bcast_b(a[0], 0);
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const double d = dn;
                bad = bad || !(d > 0.0 && d < INFINITY);
                const double y = __builtin_amdgcn_rsq(d);
                const double e = __builtin_fma(-d * y, y, 1.0);
                const double l = __builtin_fma(0.5 * a[j] * y, e, a[j] * y);
                my_inv = (r == j) ? __builtin_fma(0.5 * y, e, y) : my_inv;
                a[j] = l;
                if (j < 15) {
                    dn = bcast_b(__builtin_fma(-l, l, a[j + 1]), j + 1);
#pragma unroll
                    for (int k = j + 1; k < 16; ++k) a[k] = __builtin_fma(-l, bcast_b(l, k), a[k]);
                }
            }
            if (live)
#pragma unroll
                for (int cc = 0; cc < 16; ++cc) T[row * BLD + 16 * kb + cc] = (r >= 16 || cc <= r) ? a[cc] : 0.0;
            if (r < 16) rdg[16 * kb + r] = my_inv;
            if (lane == 0) __hip_atomic_store(sync, kb + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            D1S(1 + kb);
        }
        if (bad && lane == 0) raise_flag(flag, FLAG_NOT_PD);
    } else if (wave <= 3) {
        for (int kb = 0; kb + wave <= 3 && kb < 3; ++kb) {
            if (!spin_ge(0, kb + 1)) { ok = false; break; }
            if (kb + 1 >= 2 && !spin_ge(5 + kb + 1, 2)) { ok = false; break; }  // earlier panels' trailing updates
            tile_sub(kb + wave, kb + 1, kb);
            signal(1 + kb);
        }
    } else if (wave == 6) {  // tile (3,3): panel 0, then panel 1
        for (int pn = 0; pn < 2 && ok; ++pn) {
            if (!spin_ge(0, pn + 1)) { ok = false; break; }
            tile_sub(3, 3, pn);
            signal(5 + 3);
        }
    } else if (wave == 7) {  // tiles (2,2), (3,2): panel 0
        if (!spin_ge(0, 1)) ok = false;
        else {
            tile_sub(2, 2, 0);
            tile_sub(3, 2, 0);
            __hip_atomic_fetch_add(sync + 5 + 2, lane == 0 ? 2 : 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    } else if (wave == 5) {
        auto wsync = [] {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
        // panel by panel: W_kb (lanes 0-15, column `lane` by forward substitution), then L z = b's block kb:
        // z_kb = W_kb r_kb, r -= L(:, kb) z_kb below (lane = row)
        for (int kb = 0; kb < 4; ++kb) {
            if (!spin_ge(0, kb + 1)) { ok = false; break; }
            if (lane < 16) {
                double w[16];
#pragma unroll
                for (int m = 0; m < 16; ++m) w[m] = (m == lane) ? 1.0 : 0.0;
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    w[m] *= rdg[16 * kb + m];
#pragma unroll
                    for (int j = m + 1; j < 16; ++j)
                        w[j] = __builtin_fma(-T[(16 * kb + j) * BLD + 16 * kb + m], w[m], w[j]);
                }
#pragma unroll
                for (int m = 0; m < 16; ++m) Wm[kb][m * 16 + lane] = w[m];
            }
            const bool in = (lane >> 4) == kb;
            if (in) vr[lane] = b;
            wsync();
            if (in) {
                double z = 0.0;
#pragma unroll
                for (int m = 0; m < 16; ++m) z = __builtin_fma(Wm[kb][(lane & 15) * 16 + m], vr[16 * kb + m], z);
                b = z;
                vz[lane] = z;
            }
            wsync();
            if ((lane >> 4) > kb)
#pragma unroll
                for (int j = 0; j < 16; ++j) b = __builtin_fma(-T[lane * BLD + 16 * kb + j], vz[16 * kb + j], b);
            wsync();
        }
        if (ok) {
            D1S(5);
            // L^T y = z by blocks, last first: y_kb = W_kb^T r_kb, then r -= L(kb, :)^T y_kb above
            for (int kb = 3; kb >= 0; --kb) {
                const bool in = (lane >> 4) == kb;
                if (in) vr[lane] = b;
                wsync();
                if (in) {
                    double y = 0.0;
#pragma unroll
                    for (int m = 0; m < 16; ++m) y = __builtin_fma(Wm[kb][m * 16 + (lane & 15)], vr[16 * kb + m], y);
                    b = y;
                    vz[lane] = y;
                }
                wsync();
                if ((lane >> 4) < kb)
#pragma unroll
                    for (int j = 0; j < 16; ++j) b = __builtin_fma(-T[(16 * kb + j) * BLD + lane], vz[16 * kb + j], b);
                wsync();
            }
            D1S(6);
            // the step (block_step's arithmetic): y into rhs for the back-substitution, the camera / intrinsics
            // updates from the prefetched operands, the step scalars reduced over the wave in block_step's order
            if (lane < n) {
                rhs[lane] = b;
                vz[lane] = b;
            }
            wsync();
            double acc[4] = {0.0, 0.0, 0.0, 0.0};  // sn2, mcc, cand cost, |x_cand|^2
            if (lane < P.nac) cam_step(P, c, cur, radius, cops, lane, vz + 6 * lane, delta, acc);
            else if (lane == BCR_CAMS) intr_step(P, c, cur, radius, iops, vz + P.kb, delta, acc);
            // (only lanes <= BCR_CAMS hold a term: the row-0 sum by DPP is the total)
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[k] = dpp_row_sum(acc[k]);
            if (lane == 0) {
                part[PART_UPD_SN2 * P.part_stride] = acc[0];
                part[PART_UPD_MCC * P.part_stride] = acc[1];
                part[PART_UPD_COST * P.part_stride] = acc[2];
                part[PART_UPD_XN2 * P.part_stride] = acc[3];
            }
            D1S(7);
        }
    }
    if (!ok && lane == 0) raise_flag(flag, FLAG_TIMEOUT);
#undef D1S
}

static_assert(PANEL_DOUBLES <= BCR_BLOCK_DOUBLES, "published panels fit the block's workspace");
static_assert(2 * PANEL_DOUBLES <= BB * BB + BB * XW, "two epochs' panels fit the Cf | X slots");

#define CKB(x)                            \
    do {                                  \
        hipError_t e_ = (x);              \
        if (e_ != hipSuccess) return e_;  \
    } while (0)

static constexpr int NSTAMP = 32 * 256;
static inline int n_elim(int nblk, int m) {
    const int s = 1 << m;
    return (nblk - s + 2 * s - 1) / (2 * s);
}

#define BPL(kid, ...)                     \
    do {                                  \
        if (pf) pf->begin(kid, s);        \
        hipLaunchKernelGGL(__VA_ARGS__);  \
        if (pf) pf->end(s);               \
        CKB(hipGetLastError());           \
    } while (0)

// k_bcr_split's workgroups wait on each other, so the grid must be co-resident. MIBA_BCR_COOP=1 launches it
// cooperatively: the runtime then refuses a grid that cannot be (hipErrorCooperativeLaunchTooLarge -> the
// per-level launches) instead of letting it run into the hand-off timeouts. Off by default: on MI355X
// (ROCm 7.2) the cooperative launch of the C4 grid costs ~20 us more per launch (k_bcr_split 108.5 -> 129 us,
// C4 3719 -> 3359 LM it/s, same-box A/B, profiles/r03_ab_coop_c4.txt); the default relies on the bounded
// hand-off waits, whose timeout re-runs the iteration with the per-level launches inside the same solve.
static bool bcr_coop() {
    const char* e = getenv("MIBA_BCR_COOP");  // read per launch (tests switch it inside one process)
    return e && e[0] == '1';
}
template <bool STAMP, int NH>
static hipError_t launch_split(const DevProblem& P, const BaConsts& c, DevWork& W, const BcrWork& Bw, hipStream_t s,
                               unsigned long long* stamps, Prof* pf) {
    const int nwg = (NH + 1) * Bw.nblk;
    const dim3 grid(Bw.xmap ? 8 * ((nwg + 3) / 4) : nwg), block(TPB_E);
    if (!bcr_coop()) {
        BPL(K_BCR_PERSIST, (k_bcr_split<STAMP, NH>), grid, block, sizeof(HLds), s, W.st, P, W.S, W.rhs, Bw, W.chol_flag,
            stamps, c, W.scale, W.camdata, W.lin, W.delta, W.part);
        return hipSuccess;
    }
    const LmState* a_st = W.st;
    DevProblem a_P = P;
    const double* a_S = W.S;
    double* a_rhs = W.rhs;
    BcrWork a_Bw = Bw;
    int* a_flag = W.chol_flag;
    unsigned long long* a_tl = stamps;
    BaConsts a_c = c;
    const double* a_scale = W.scale;
    const double* a_camdata = W.camdata;
    const double* a_lin = W.lin;
    double* a_delta = W.delta;
    double* a_part = W.part;
    void* args[] = {&a_st, &a_P, &a_S, &a_rhs, &a_Bw, &a_flag, &a_tl, &a_c, &a_scale, &a_camdata, &a_lin, &a_delta, &a_part};
    if (pf) pf->begin(K_BCR_PERSIST, s);
    const hipError_t e = hipLaunchCooperativeKernel((const void*)k_bcr_split<STAMP, NH>, grid, block, args, sizeof(HLds), s);
    if (pf) pf->end(s);
    return e;
}

template <bool STAMP>
static hipError_t launch_per_level(const DevProblem& P, const BaConsts& c, DevWork& W, const BcrWork& Bw, hipStream_t s,
                                   unsigned long long* stamps, Prof* pf);

template <bool STAMP>
static hipError_t launch_bcr_t(const DevProblem& P, const BaConsts& c, DevWork& W, BcrWork& Bw, hipStream_t s,
                               unsigned long long* stamps, Prof* pf) {
    const int nblk = Bw.nblk;
    if (Bw.persist >= 2) {
        // the border solve and the camera step run inside the split kernel (no k_bcr_border launch)
        const hipError_t e = Bw.persist == 3 ? launch_split<STAMP, 2>(P, c, W, Bw, s, stamps, pf)
                                             : launch_split<STAMP, 1>(P, c, W, Bw, s, stamps, pf);
        if (e == hipSuccess) return hipSuccess;
        (void)hipGetLastError();  // the refused launch's error is not sticky: clear it
        if (e != hipErrorCooperativeLaunchTooLarge) return e;
        // the grid cannot be co-resident on this device: this context uses the per-level launches
        // (the k_final of this iteration sees persist == 0 and advances no epoch)
        Bw.persist = 0;
        CKB(bcr_reset_pull_slots(Bw, false, s));
        return launch_per_level<STAMP>(P, c, W, Bw, s, stamps, pf);
    }
    if (Bw.persist) {
        BPL(K_BCR_PERSIST, k_bcr_persist<STAMP>, dim3(nblk), dim3(TPB_E), sizeof(PersistLds), s, W.st, P, W.S, W.rhs,
            Bw, W.chol_flag, stamps);
        BPL(K_BCR_BORDER, k_bcr_border, dim3(nblk), dim3(TPB_BD), 0, s, W.st, P, W.rhs, Bw, W.chol_flag, c, W.scale,
            W.camdata, W.lin, W.delta, W.part);
        return hipSuccess;
    }
    return launch_per_level<STAMP>(P, c, W, Bw, s, stamps, pf);
}

// the reference arithmetic: one launch per level (no inter-workgroup waits)
template <bool STAMP>
static hipError_t launch_per_level(const DevProblem& P, const BaConsts& c, DevWork& W, const BcrWork& Bw, hipStream_t s,
                                   unsigned long long* stamps, Prof* pf) {
    const int nblk = Bw.nblk;
    for (int m = 0; m < Bw.levels; ++m) {
        const int nel = n_elim(nblk, m);
        const int nacc = m >= 1 ? (nblk + (2 << m) - 1) / (2 << m) : 0;
        BPL(K_BCR_ELIM, k_bcr_elim<STAMP>, dim3(nel + nacc), dim3(TPB_E), sizeof(ElimLds), s, W.st, P, W.S, W.rhs, Bw, m,
            nel, W.chol_flag, stamps);
        BPL(K_BCR_CONTRIB, k_bcr_contrib, dim3(nel * NCONTRIB_WG), dim3(TPB_C), 0, s, W.st, Bw, m);
    }
    BPL(K_BCR_ELIM, k_bcr_elim<STAMP>, dim3(1), dim3(TPB_E), sizeof(ElimLds), s, W.st, P, W.S, W.rhs, Bw, Bw.levels, 1,
        W.chol_flag, stamps);
    for (int m = Bw.levels - 1; m >= 0; --m)
        BPL(K_BCR_BACK, k_bcr_back<STAMP>, dim3(n_elim(nblk, m)), dim3(TPB_C), sizeof(BackLds), s, W.st, P, W.S, Bw, m,
            stamps);
    BPL(K_BCR_BORDER, k_bcr_border, dim3(nblk), dim3(TPB_BD), 0, s, W.st, P, W.rhs, Bw, W.chol_flag, c, W.scale,
            W.camdata, W.lin, W.delta, W.part);
    return hipSuccess;
}

static hipError_t bcr_persist_attr() {
    static DeviceOnce once;
    return once([]() -> hipError_t {
        CKB(hipFuncSetAttribute((const void*)k_bcr_persist<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)sizeof(PersistLds)));
        CKB(hipFuncSetAttribute((const void*)k_bcr_persist<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)sizeof(PersistLds)));
        const void* fns[] = {(const void*)k_bcr_split<false, 1>, (const void*)k_bcr_split<true, 1>,
                             (const void*)k_bcr_split<false, 2>, (const void*)k_bcr_split<true, 2>};
        for (const void* f : fns) CKB(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)sizeof(HLds)));
        return hipSuccess;
    });
}

// k_bcr_split's pull slots (published XL / XR / x rows, two epochs: UL | UR | F, rL | rR, F2) start empty;
// the per-level and persistent paths use the same buffers for their contributions and need zeros there
// (the upper tiles of UL / UR are read, never written)
hipError_t bcr_reset_pull_slots(const BcrWork& Bw, bool split, hipStream_t s) {
    const size_t b64 = (size_t)BSZ * Bw.nblk, b8 = (size_t)RSZ * Bw.nblk;
    const unsigned pat = split ? BCR_Y_EMPTY_D32 : 0u;
    CKB(hipMemsetD32Async((hipDeviceptr_t)Bw.UL, pat, 2 * 3 * b64, s));  // UL | UR | F
    CKB(hipMemsetD32Async((hipDeviceptr_t)Bw.rL, pat, 2 * 2 * b8, s));   // rL | rR
    CKB(hipMemsetD32Async((hipDeviceptr_t)Bw.F2, pat, 2 * b64, s));
    return hipSuccess;
}

hipError_t bcr_set_spin_limit(unsigned limit) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_spin_limit), &limit, sizeof(limit));
}

// One-block windows take k_bcr_dense1 (MIBA_BCR_DENSE1=0, or any MIBA_BCR path override, keeps the split kernel).
int bcr_dense1_ok(int nblk, int kb) {
    if (nblk != 1 || kb + 4 > BB || std::getenv("MIBA_BCR")) return 0;
    const char* e = std::getenv("MIBA_BCR_DENSE1");
    return (e && e[0] == '0') ? 0 : 1;
}

int bcr_persist_ok(int nblk) {
    if (bcr_persist_attr() != hipSuccess) return 0;
    int dev = 0, ncu = 0, per_cu = 0, per_cu2 = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu2, k_bcr_split<false, 2>, TPB_E, sizeof(HLds)) == hipSuccess &&
        per_cu2 >= 1 && 3 * nblk <= per_cu2 * ncu)
        return 3;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu2, k_bcr_split<false, 1>, TPB_E, sizeof(HLds)) == hipSuccess &&
        per_cu2 >= 1 && 2 * nblk <= per_cu2 * ncu)
        return 2;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_bcr_persist<false>, TPB_E, sizeof(PersistLds)) !=
        hipSuccess)
        return 0;
    return per_cu >= 1 && nblk <= per_cu * ncu ? 1 : 0;
}

// MIBA_BCR_XMAP=1 (opt-in): k_bcr_split's workgroups on XCDs 0-3 only, when they all fit there at once (every
// workgroup of the split kernel waits on others: a launch that does not fit would time out)
int bcr_xmap_ok(int nblk, int persist) {
    const char* e = std::getenv("MIBA_BCR_XMAP");
    if (!(e && e[0] == '1') || persist < 2) return 0;
    int dev = 0, ncu = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    const hipError_t r = persist == 3
        ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_bcr_split<false, 2>, TPB_E, sizeof(HLds))
        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_bcr_split<false, 1>, TPB_E, sizeof(HLds));
    return r == hipSuccess && persist * nblk <= per_cu * (ncu / 2) ? 1 : 0;
}

hipError_t launch_bcr(const DevProblem& P, const BaConsts& c, DevWork& W, BcrWork& Bw, hipStream_t s, Prof* pf) {
    if (Bw.band) return launch_bcr_band(P, c, W, Bw.band, s, pf);  // narrow band: one workgroup (ba_band.hip)
    if (Bw.dense1) {  // one-block window: the dense single-workgroup solve (bcr_dense1_ok)
        static DeviceScratch stamp_buf;
        static const int dmode = env_on("MIBA_BCR_STAMPS");
        if (dmode) {
            unsigned long long* dst = stamp_buf.get<unsigned long long>(16 * sizeof(unsigned long long));
            if (!dst) return hipErrorOutOfMemory;
            CKB(hipMemsetAsync(dst, 0, 16 * sizeof(unsigned long long), s));
            BPL(K_BCR_PERSIST, k_bcr_dense1<true>, dim3(1), dim3(TPB_D1), 0, s, W.st, P, W.S, W.rhs, W.chol_flag, c,
                W.scale, W.camdata, W.lin, W.delta, W.part, dst);
            unsigned long long h[16];
            CKB(hipMemcpyAsync(h, dst, sizeof(h), hipMemcpyDeviceToHost, s));
            CKB(hipStreamSynchronize(s));
            if (h[9] && h[7]) {
                auto us = [&](int k) { return (double)(h[k] - h[9]) * 0.01; };
                fprintf(stderr, "bcr_dense1 us: loaded %.2f panels %.2f %.2f %.2f %.2f forward %.2f backward %.2f step %.2f\n",
                        us(0), us(1), us(2), us(3), us(4), us(5), us(6), us(7));
            }
            return hipSuccess;
        }
        BPL(K_BCR_PERSIST, k_bcr_dense1<false>, dim3(1), dim3(TPB_D1), 0, s, W.st, P, W.S, W.rhs, W.chol_flag, c,
            W.scale, W.camdata, W.lin, W.delta, W.part, (unsigned long long*)nullptr);
        return hipSuccess;
    }
    static DeviceOnce attr;
    static DeviceScratch stamp_buf;
    static const int smode = env_on("MIBA_BCR_STAMPS");
    CKB(attr([]() -> hipError_t {
        const int le = (int)sizeof(ElimLds), lb = (int)sizeof(BackLds);
        CKB(hipFuncSetAttribute((const void*)k_bcr_elim<false>, hipFuncAttributeMaxDynamicSharedMemorySize, le));
        CKB(hipFuncSetAttribute((const void*)k_bcr_elim<true>, hipFuncAttributeMaxDynamicSharedMemorySize, le));
        CKB(hipFuncSetAttribute((const void*)k_bcr_back<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lb));
        CKB(hipFuncSetAttribute((const void*)k_bcr_back<true>, hipFuncAttributeMaxDynamicSharedMemorySize, lb));
        return hipSuccess;
    }));
    if (smode) {
        unsigned long long* stamps = stamp_buf.get<unsigned long long>(sizeof(unsigned long long) * NSTAMP);
        if (!stamps) return hipErrorOutOfMemory;
        CKB(hipMemsetAsync(stamps, 0, sizeof(unsigned long long) * NSTAMP, s));
        CKB(launch_bcr_t<true>(P, c, W, Bw, s, stamps, nullptr));
        std::vector<unsigned long long> hv(NSTAMP);
        unsigned long long* h = hv.data();
        CKB(hipMemcpyAsync(h, stamps, sizeof(unsigned long long) * NSTAMP, hipMemcpyDeviceToHost, s));
        CKB(hipStreamSynchronize(s));
        if (Bw.persist >= 2) {
            const int nr = Bw.persist;  // workgroups per block
            unsigned long long t0 = ~0ull;
            for (int g = 0; g < nr * Bw.nblk && g < 256; ++g) if (h[32 * g]) t0 = std::min(t0, h[32 * g]);
            auto us = [&](unsigned long long t) { return t ? (double)(t - t0) * 0.01 : -1.0; };
            for (int g = 0; g < nr * Bw.nblk && g < 256; ++g) {
                const unsigned long long* q = h + 32 * g;
                if (g % nr == 0) {
                    fprintf(stderr, "bcr F%3d start %7.2f loaded %7.2f panels %7.2f %7.2f %7.2f %7.2f\n", g / nr, us(q[0]),
                            us(q[1]), us(q[2]), us(q[3]), us(q[4]), us(q[5]));
                    fprintf(stderr, "        chain start | chain end | published:");
                    for (int kb = 0; kb < 4; ++kb)
                        fprintf(stderr, "  %7.2f %7.2f %7.2f", us(q[17 + 3 * kb]), us(q[16 + 3 * kb]), us(q[2 + kb]));
                    // shader clocks per pivot (LDS loads .. chain .. LDS stores) and the clock rate they imply
                    const double c0 = (double)(q[29] - q[28]) / 16.0, c3 = (double)(q[31] - q[30]) / 16.0;
                    fprintf(stderr, "  | chain clk/pivot %.0f %.0f", c0, c3);
                    fprintf(stderr, "\n");
                } else
                {
                    fprintf(stderr, "bcr H%c%3d start %7.2f loaded %7.2f panel got/done %7.2f %7.2f %7.2f %7.2f %7.2f %7.2f %7.2f %7.2f contrib %7.2f fill/xl %7.2f back-wait %7.2f done %7.2f\n",
                            nr == 2 ? ' ' : (g % nr == 1 ? 'A' : 'B'), g / nr, us(q[0]), us(q[1]), us(q[2]), us(q[3]), us(q[4]), us(q[5]), us(q[6]), us(q[7]), us(q[8]),
                            us(q[9]), us(q[10]), us(q[11]), us(q[12]), us(q[14]));
                    fprintf(stderr, "        panel got | loaded | x-updated | contrib:");
                    for (int kb = 0; kb < 4; ++kb)
                        fprintf(stderr, "  %7.2f %7.2f %7.2f %7.2f", us(q[2 + 2 * kb]), us(q[16 + 4 * kb]), us(q[17 + 4 * kb]),
                                us(q[3 + 2 * kb]));
                    fprintf(stderr, "\n");
                }
            }
            return hipSuccess;
        }
        if (Bw.persist) {
            // per block: level-0 loaded, survivor waits done, factor start/end, contributions published,
            // back wait done, y published — us after the earliest start
            unsigned long long t0 = ~0ull;
            for (int i = 0; i < Bw.nblk && i < 256; ++i) if (h[32 * i]) t0 = std::min(t0, h[32 * i]);
            auto us = [&](unsigned long long t) { return t ? (double)(t - t0) * 0.01 : -1.0; };
            for (int i = 0; i < Bw.nblk && i < 256; ++i) {
                const unsigned long long* q = h + 32 * i;
                fprintf(stderr, "bcr blk %3d start %7.2f loaded %7.2f waits", i, us(q[0]), us(q[1]));
                for (int m = 0; m < 7; ++m) if (q[2 + m]) fprintf(stderr, " %7.2f", us(q[2 + m]));
                fprintf(stderr, " | factor %7.2f-%7.2f contrib %7.2f pre %7.2f back-wait %7.2f done %7.2f\n", us(q[9]),
                        us(q[10]), us(q[11]), us(q[13]), us(q[12]), us(q[14]));
                if (i <= 2) {
                    fprintf(stderr, "    factor phases (end of phase 1 / phase 2 per panel):");
                    for (int k = 0; k < 8; ++k) fprintf(stderr, " %7.2f", us(q[16 + k]));
                    fprintf(stderr, "\n");
                }
            }
            return hipSuccess;
        }
        for (int m = 0; m <= Bw.levels; ++m) {
            const unsigned long long* q = h + (size_t)m * 8;
            const unsigned long long* b = h + (size_t)(16 + m) * 8;
            const unsigned long long* f = h + 8 * 24 + 4 * m;
            fprintf(stderr, "bcr level %d blk0 cycles: elim load %llu factor+fwd %llu [potrf16 %llu fwd16 %llu trailing %llu] store %llu | back load %llu gemv %llu trsm+store %llu\n",
                    m, q[1] - q[0], q[2] - q[1], f[0], f[1], f[2], q[3] - q[2], b[0] ? b[1] - b[0] : 0ull,
                    b[0] ? b[2] - b[1] : 0ull, b[0] ? b[3] - b[2] : 0ull);
        }
    } else {
        CKB(launch_bcr_t<false>(P, c, W, Bw, s, nullptr, pf));
    }
    return hipSuccess;
}

}  // namespace miba
