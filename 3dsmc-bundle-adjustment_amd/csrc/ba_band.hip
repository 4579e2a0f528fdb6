// ba_band.hip — the reduced camera system of a narrow-band window in ONE workgroup: cyclic reduction at the
// granularity of the camera band, everything in LDS.
//
// The reference's windows are sequential keyframes that share landmarks only along short tracks
// (Map3D.cpp:7-27, 62-74: a keyframe links to its predecessor's landmarks), so the camera part of the
// reduced system S (ceres SPARSE_SCHUR's reduced camera matrix, OptimizationUtils.cpp:300) is block-banded: an
// active camera couples only to the cameras within `cam_band` of it. With blocks of BC = max(cam_band, 1)
// consecutive cameras (G = 6 BC dofs) the camera part is exactly block-tridiagonal; the 4 intrinsics rows that
// follow the camera dofs in S form a dense border:
//     S = [A  B; B^T C],   A block-tridiagonal (nb blocks of G x G), B (6 nac x 4), C (4 x 4).
// k_bcr_split solves such systems as 64-dof blocks spread over three workgroups per block with cross-CU
// hand-offs (C3, 50 keyframes / camera_band 1: five 64-dof blocks that are mostly zeros, 58 us). Here the
// whole system of a window of up to ~100 cameras (G = 6: 158 doubles of LDS per block) is loaded into one
// workgroup's LDS and eliminated by odd-even cyclic reduction — a Cholesky factorisation of A in
// nested-dissection order, so it is as stable as Cholesky for the SPD A — with the border carried as four more
// right-hand sides:
//   level m eliminates the blocks i with (i + 1) = odd * 2^m, one per half-wave (32 lanes):
//     lane = row:     L_i = chol(D_i)           (pivot chain: v_rsq_f64 + one Newton step, v_readlane broadcasts)
//     lane = column:  [XL | XR | x | XB] = L_i^-1 [A(i, i - 2^m) | A(i, i + 2^m) | b_i | B_i]
//   then, every thread one output element (fixed summation order, no atomics), each survivor j pulls the Schur
//   terms of its eliminated neighbours i1 = j - 2^m, i2 = j + 2^m:
//     D_j -= XR_i1^T XR_i1 + XL_i2^T XL_i2,   b_j -= XR_i1^T x_i1 + XL_i2^T x_i2,   B_j -= (same with XB),
//     A(j, j - 2^(m+1)) = -XR_i1^T XL_i1       (the fill between the two survivors i1 separated)
//   and each eliminated block its border Gram [XB | x]^T XB (14 values), summed over all blocks in block order
//   into the 4x4 border system (C - B^T A^-1 B) y_k = b_k - B^T A^-1 b (border_solve4, as k_bcr_split).
//   The root is block 2^K - 1 (K = floor(log2 nb)); depth K + 1 block factorisations of G pivots each
//   (C3: 6 of 6 pivots, against 5 of 64 on the split kernel's critical path).
// Back-substitution, top level first, one half-wave per block: y_i = L_i^-T (x_i - XL_i y_(i-2^m) -
// XR_i y_(i+2^m) - XB_i y_k). Then y goes to rhs (the points' back-substitution reads it) and the camera /
// intrinsics step runs as in k_bcr_split's block_step: wave w applies cameras [10 w, 10 w + 10) (w = 0 also the
// intrinsics) and writes the step scalars to part slot w, the slots k_final sums for the BCR path.
// No inter-workgroup wait anywhere: the kernel cannot time out.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "ba_device.h"
#include "ba_kernels.h"
#include "ba_solve_util.h"

namespace miba {

// workgroup size: 16 waves (32 half-wave block units) for blocks of one camera; 8 waves for blocks of 2-3 cameras
// (half as many blocks, and the wider blocks' pivot rows / triangular solves need the 256-VGPR budget of 2 waves
// per SIMD: at 4 waves per SIMD they spill 420 / 1280 B per lane)
template <int BC>
struct BandTpb {
    static constexpr int TPB = BC == 1 ? 1024 : 512;
    static constexpr int NW = TPB / 64;
};
static constexpr int BAND_OPS = 25;    // staged camera-step operands per active camera: sc 6 | ud 6 | g 6 | x 7
static constexpr int BAND_IOPS = 20;   // intrinsics: K 4 | sk 4 | uk 4 | gk 4 | prior 4
static constexpr int BAND_GR = 16;     // per-block border Gram slot (14 used)
static constexpr int BAND_NL = 8;      // loads in flight per thread in the load phase
static constexpr int BAND_STAMPS = 24;

// LDS layout (doubles) of one window: per block j (nb blocks of G dofs, block-major = dof order)
//   D  G x G   diagonal block, then L_j (lower; upper zero) once j is eliminated
//   CL G x G   coupling to the current left neighbour A(j, j - 2^m), then XL_j
//   XR G x G   XR_j
//   BB G x 4   border rows B_j, then XB_j
//   BV G       rhs b_j, then x_j;   RI G   1 / diag(L_j);   YV G   y_j
//   GR 16      border Gram of block j
// then bk = [b_k | S_kk lower packed] (14) | red (20) | y_k (4), the intrinsics' and cameras' step operands and
// the active cameras' indices (ints, two per double).
struct BandLayout {
    int D, CL, XR, BB, BV, RI, YV, GR, BK, RED, YK, IOPS, OPS, AC, total;
};
__host__ __device__ inline BandLayout band_layout(int G, int nb, int nac) {
    BandLayout L;
    int o = 0;
    L.D = o;    o += nb * G * G;
    L.CL = o;   o += nb * G * G;
    L.XR = o;   o += nb * G * G;
    L.BB = o;   o += nb * G * 4;
    L.BV = o;   o += nb * G;
    L.RI = o;   o += nb * G;
    L.YV = o;   o += nb * G;
    L.GR = o;   o += nb * BAND_GR;
    L.BK = o;   o += 16;
    L.RED = o;  o += 24;
    L.YK = o;   o += 8;
    L.IOPS = o; o += BAND_IOPS;
    L.OPS = o;  o += nac * BAND_OPS;
    L.AC = o;   o += (nac + 1) / 2 + 1;
    L.total = o;
    return L;
}

// lane j of this lane's half-wave to every lane of the half (two v_readlane pairs and a select)
__device__ __forceinline__ double bcast_half(double v, int j, bool hi) {
    const double lo = bcast_b(v, j), up = bcast_b(v, 32 + j);
    return hi ? up : lo;
}
// wide blocks (G = 18): a compiler barrier between the steps of an unrolled triangular solve keeps the compiler
// from hoisting every LDS operand of the solve into registers at once (752 B per lane of spills without it)
template <int G>
__device__ __forceinline__ void narrow_live_range() {
    if constexpr (G > 12) asm volatile("" ::: "memory");
}
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int BC, bool STAMP>
__global__ __launch_bounds__(BandTpb<BC>::TPB) void k_bcr_band(const LmState* __restrict__ st, DevProblem P,
                                                       const double* __restrict__ S, double* __restrict__ rhs,
                                                       int* __restrict__ flag, BaConsts c,
                                                       const double* __restrict__ scale,
                                                       const double* __restrict__ camdata,
                                                       const double* __restrict__ lin, double* __restrict__ delta,
                                                       double* __restrict__ part, int nb,
                                                       unsigned long long* __restrict__ tl) {
    constexpr int G = 6 * BC;
    constexpr int GG = G * G;
    constexpr int TPB_BAND = BandTpb<BC>::TPB, NW_BAND = BandTpb<BC>::NW;
    constexpr int NCOL = 2 * G + 5;  // [XL | XR | x | XB] columns of the forward solve
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, hl = lane & 31;
    const bool hi = lane >= 32;
    const int nac = P.nac, ncd = P.kb;  // active cameras, camera dofs (= 6 nac = first intrinsics row)
    const size_t ld = P.npad;
    const BandLayout Ly = band_layout(G, nb, nac);
    double* const Dm = lds + Ly.D;
    double* const CL = lds + Ly.CL;
    double* const XR = lds + Ly.XR;
    double* const BBm = lds + Ly.BB;
    double* const BV = lds + Ly.BV;
    double* const RI = lds + Ly.RI;
    double* const YV = lds + Ly.YV;
    double* const GR = lds + Ly.GR;
    int* const AC = reinterpret_cast<int*>(lds + Ly.AC);
    int ts = 0;
    auto stamp = [&]() {
        if constexpr (STAMP) {
            __syncthreads();
            if (tid == 0) tl[ts] = realtime_now();
            ++ts;
        }
    };
    if constexpr (STAMP) if (tid == 0) tl[BAND_STAMPS - 1] = realtime_now();
    // ---- load: S blocks, border, rhs, corner and the step operands, NL loads in flight per thread (clamped
    // addresses, selects after), the LM-state check behind them
    const bool skip = skip_step(st);
    const int cur = st->cur;
    const int nD = nb * GG, nBB = nb * G * 4, nBV = nb * G;
    const int e_cl = nD, e_bb = 2 * nD, e_bv = e_bb + nBB, e_bk = e_bv + nBV, e_io = e_bk + 14, e_op = e_io + BAND_IOPS;
    const int E = e_op + 18 * nac;
    const int acv = tid < nac ? P.ac_cam[tid] : 0;
    for (int e0 = 0; e0 < E; e0 += TPB_BAND * BAND_NL) {
        double v[BAND_NL];
        int dst[BAND_NL];
#pragma unroll
        for (int q = 0; q < BAND_NL; ++q) {
            const int e = e0 + TPB_BAND * q + tid;
            const double* p = S;
            size_t idx = 0;
            bool ok = false;
            double cst = 0.0;
            int d = -1;
            if (e < e_cl) {  // diagonal blocks, both halves (identity past the last camera dof)
                const int j = e / GG, r = (e / G) % G, cc = e % G;
                const int dr = j * G + r, dc = j * G + cc;
                ok = dr < ncd && dc < ncd;
                idx = dr >= dc ? (size_t)dr * ld + dc : (size_t)dc * ld + dr;
                cst = r == cc ? 1.0 : 0.0;
                d = Ly.D + e;
            } else if (e < e_bb) {  // couplings A(j, j - 1)
                const int f = e - e_cl, j = f / GG, r = (f / G) % G, cc = f % G;
                const int dr = j * G + r, dc = (j - 1) * G + cc;
                ok = j >= 1 && dr < ncd;
                idx = (size_t)dr * ld + dc;
                d = Ly.CL + f;
            } else if (e < e_bv) {  // border rows B_j (S rows kb .. kb + 3 at the block's columns)
                const int f = e - e_bb, dr = f >> 2, k = f & 3;
                ok = dr < ncd;
                idx = (size_t)(ncd + k) * ld + dr;
                d = Ly.BB + f;
            } else if (e < e_bk) {  // rhs
                const int dr = e - e_bv;
                ok = dr < ncd;
                p = rhs;
                idx = dr;
                d = Ly.BV + dr;
            } else if (e < e_io) {  // bk: b_k, then S_kk lower packed
                const int f = e - e_bk;
                ok = true;
                if (f < 4) {
                    p = rhs;
                    idx = ncd + f;
                } else {
                    int q2 = f - 4, mm = 0;
                    while (q2 > mm) { q2 -= mm + 1; ++mm; }
                    idx = (size_t)(ncd + mm) * ld + ncd + q2;
                }
                d = Ly.BK + f;
            } else if (e < e_op) {  // the intrinsics' step operands (load_intr_step_ops)
                const int f = e - e_io, kind = f >> 2, m = f & 3;
                ok = true;
                p = kind == 0 ? P.K[cur] : kind == 1 ? scale : kind == 4 ? P.prior : lin;
                idx = kind == 0 ? m : kind == 1 ? P.off_k + m : kind == 2 ? 2 + 4 * m - (m * (m - 1)) / 2
                                                              : kind == 3 ? 12 + m : m;
                d = Ly.IOPS + f;
            } else if (e < E) {  // the cameras' step operands (load_cam_step_ops, but the pose: below)
                const int f = e - e_op, t = f / 18, k = f % 18;
                ok = true;
                p = k < 6 ? scale : camdata;
                idx = k < 6 ? 6 * (size_t)t + k
                            : (size_t)t * CAMDATA + (k < 12 ? (k - 6) * 6 - ((k - 6) * (k - 7)) / 2 : 45 + k - 12);
                d = Ly.OPS + t * BAND_OPS + k;
            }
            v[q] = p[ok ? idx : 0];
            v[q] = ok ? v[q] : cst;
            dst[q] = d;
        }
#pragma unroll
        for (int q = 0; q < BAND_NL; ++q)
            if (dst[q] >= 0) lds[dst[q]] = v[q];
    }
    if (skip) return;
    if (tid < nac) AC[tid] = acv;
    const double radius = st->radius;
    __syncthreads();
    // the poses of the step (a dependent load: the camera index first), held in a register until the step
    const int nx = 7 * nac;
    double xv = 0.0;
    if (tid < nx) xv = P.cams[cur][7 * (size_t)AC[tid / 7] + tid % 7];
    stamp();  // 0: loaded
    // K = floor(log2 nb): the root is block 2^K - 1, eliminated at level K with no neighbour
    int K = 0;
    while ((2 << K) <= nb) ++K;
    bool bad = false;
    for (int m = 0; m <= K; ++m) {
        const int s = 1 << m;
        const int ne = ((nb >> m) + 1) >> 1;  // blocks i with i + 1 = odd * 2^m, i < nb
        // ---- factor + forward solve, one half-wave per eliminated block
        for (int s0 = 0; s0 < ne; s0 += 2 * NW_BAND) {
            const int slot = s0 + 2 * wave + (hi ? 1 : 0);
            const bool act = slot < ne;
            const int i = act ? ((2 * slot + 1) << m) - 1 : 0;
            const int r = hl < G ? hl : G - 1;
            double a[G];
#pragma unroll
            for (int k = 0; k < G; ++k) a[k] = Dm[i * GG + r * G + k];
            double my_inv = 0.0;
            double dn = bcast_half(a[0], 0, hi);
#pragma unroll
            for (int j = 0; j < G; ++j) {
                const double dd = dn;
                bad = bad || (act && !(dd > 0.0 && dd < INFINITY));
                const double y = __builtin_amdgcn_rsq(dd);
                const double ee = __builtin_fma(-dd * y, y, 1.0);
                const double l = __builtin_fma(0.5 * a[j] * y, ee, a[j] * y);
                my_inv = (hl == j) ? __builtin_fma(0.5 * y, ee, y) : my_inv;
                a[j] = l;
                if (j + 1 < G) {
                    dn = bcast_half(__builtin_fma(-l, l, a[j + 1]), j + 1, hi);
#pragma unroll
                    for (int k = j + 1; k < G; ++k) a[k] = __builtin_fma(-l, bcast_half(l, k, hi), a[k]);
                }
            }
            if (act && hl < G) {
#pragma unroll
                for (int k = 0; k < G; ++k) Dm[i * GG + hl * G + k] = k <= hl ? a[k] : 0.0;
                RI[i * G + hl] = my_inv;
            }
            wave_sync();
            // lane = column of [A(i, i - s) | A(i, i + s) = A(i + s, i)^T | b_i | B_i]
            const int rb = i + s;
            const bool has_r = rb < nb;
            const double* Li = Dm + i * GG;
            const double* ri = RI + i * G;
            for (int col = hl; act && col < NCOL; col += 32) {
                // the column as (base, stride): A(i, i - s) column col in place (-> XL); A(i + s, i) row col - G
                // (-> XR, stored to XR_i); b_i (-> x); B_i column k (-> XB)
                double* src;
                double* out;
                int stride;
                if (col < G) {
                    src = out = CL + i * GG + col;
                    stride = G;
                } else if (col < 2 * G) {
                    src = CL + (has_r ? rb : i) * GG + (col - G) * G;
                    out = XR + i * GG + col - G;
                    stride = has_r ? 1 : 0;  // (no right neighbour: a zero column, read below as 0)
                } else if (col == 2 * G) {
                    src = out = BV + i * G;
                    stride = 1;
                } else {
                    src = out = BBm + i * G * 4 + col - 2 * G - 1;
                    stride = 4;
                }
                const bool zero = col >= G && col < 2 * G && !has_r;
                const int ostride = (col >= G && col < 2 * G) ? G : stride;
                double x[G];
#pragma unroll
                for (int q = 0; q < G; ++q) x[q] = zero ? 0.0 : src[q * stride];
#pragma unroll
                for (int j = 0; j < G; ++j) {
                    x[j] *= ri[j];
#pragma unroll
                    for (int q = j + 1; q < G; ++q) x[q] = __builtin_fma(-Li[q * G + j], x[j], x[q]);
                    narrow_live_range<G>();
                }
#pragma unroll
                for (int q = 0; q < G; ++q) out[q * ostride] = x[q];
            }
        }
        __syncthreads();
        // ---- survivors pull their eliminated neighbours' Schur terms; eliminated blocks form their border Gram
        constexpr int ND = G * (G + 1) / 2, NSI = ND + G + 4 * G + GG;
        const int ns = m < K ? nb >> (m + 1) : 0;  // survivors j with j + 1 = multiple of 2^(m+1)
        const int total = ns * NSI + ne * 14;
        for (int e = tid; e < total; e += TPB_BAND) {
            if (e < ns * NSI) {
                const int t = e / NSI, q = e % NSI;
                const int j = ((t + 1) << (m + 1)) - 1, i1 = j - s, i2 = j + s;
                const bool h2 = i2 < nb;
                const double* xr1 = XR + i1 * GG;  // XR_i1 (rows: i1's dofs, columns: j's)
                const double* xl2 = CL + (h2 ? i2 : i1) * GG;  // XL_i2 (columns: j's dofs)
                if (q < ND) {  // D_j (r, cc), cc <= r, written to both halves
                    int r = 0, cc = q;
                    while (cc > r) { cc -= r + 1; ++r; }
                    double a1 = 0.0, a2 = 0.0;
#pragma unroll
                    for (int u = 0; u < G; ++u) a1 = __builtin_fma(xr1[u * G + r], xr1[u * G + cc], a1);
                    if (h2)
#pragma unroll
                        for (int u = 0; u < G; ++u) a2 = __builtin_fma(xl2[u * G + r], xl2[u * G + cc], a2);
                    const double nv = (Dm[j * GG + r * G + cc] - a1) - a2;
                    Dm[j * GG + r * G + cc] = nv;
                    Dm[j * GG + cc * G + r] = nv;
                } else if (q < ND + G) {  // b_j
                    const int r = q - ND;
                    double a1 = 0.0, a2 = 0.0;
#pragma unroll
                    for (int u = 0; u < G; ++u) a1 = __builtin_fma(xr1[u * G + r], BV[i1 * G + u], a1);
                    if (h2)
#pragma unroll
                        for (int u = 0; u < G; ++u) a2 = __builtin_fma(xl2[u * G + r], BV[i2 * G + u], a2);
                    BV[j * G + r] = (BV[j * G + r] - a1) - a2;
                } else if (q < ND + 5 * G) {  // B_j (r, k)
                    const int f = q - ND - G, r = f >> 2, k = f & 3;
                    double a1 = 0.0, a2 = 0.0;
#pragma unroll
                    for (int u = 0; u < G; ++u) a1 = __builtin_fma(xr1[u * G + r], BBm[(i1 * G + u) * 4 + k], a1);
                    if (h2)
#pragma unroll
                        for (int u = 0; u < G; ++u) a2 = __builtin_fma(xl2[u * G + r], BBm[(i2 * G + u) * 4 + k], a2);
                    BBm[(j * G + r) * 4 + k] = (BBm[(j * G + r) * 4 + k] - a1) - a2;
                } else {  // the fill A(j, j - 2s) = -XR_i1^T XL_i1
                    const int f = q - ND - 5 * G, r = f / G, cc = f % G;
                    const double* xl1 = CL + i1 * GG;
                    double a1 = 0.0;
#pragma unroll
                    for (int u = 0; u < G; ++u) a1 = __builtin_fma(xr1[u * G + r], xl1[u * G + cc], a1);
                    CL[j * GG + r * G + cc] = -a1;
                }
            } else {  // border Gram of eliminated block i: XB^T XB (10, lower packed) | XB^T x (4)
                const int f = e - ns * NSI, g = f / 14, q = f % 14;
                const int i = ((2 * g + 1) << m) - 1;
                const double* xb = BBm + i * G * 4;
                int k = 0, l = 0;
                if (q < 10) {
                    l = q;
                    while (l > k) { l -= k + 1; ++k; }
                } else {
                    k = q - 10;
                }
                double acc = 0.0;
#pragma unroll
                for (int u = 0; u < G; ++u)
                    acc = __builtin_fma(xb[u * 4 + k], q < 10 ? xb[u * 4 + l] : BV[i * G + u], acc);
                GR[i * BAND_GR + q] = acc;
            }
        }
        __syncthreads();
        stamp();  // 1 + m: level m done
    }
    // ---- border system: the blocks' Grams summed in block order (four interleaved partial chains combined in a
    // fixed order), then (C - B^T V) y_k = b_k - B^T u on one lane
    double* const red = lds + Ly.RED;
    double* const yk = lds + Ly.YK;
    if (wave == 0) {
        const int q = lane >> 2, p = lane & 3;
        double acc = 0.0;
        if (q < 14)
            for (int i = p; i < nb; i += 4) acc += GR[i * BAND_GR + q];
        acc += __shfl_xor(acc, 1);  // (p0 + p1), (p2 + p3)
        acc += __shfl_xor(acc, 2);  // (p0 + p1) + (p2 + p3)
        if (q < 14 && p == 0) {
            int k = 0, l = q;
            if (q < 10) {
                while (l > k) { l -= k + 1; ++k; }
                red[k * 5 + 1 + l] = acc;
                red[l * 5 + 1 + k] = acc;
            } else {
                red[(q - 10) * 5] = acc;
            }
        }
        wave_sync();
        if (lane == 0) {
            bool bb = false;
            border_solve4(lds + Ly.BK, red, yk, bb);
            bad = bad || bb;
        }
    }
    if (bad && hl == 0) raise_flag(flag, FLAG_NOT_PD);
    __syncthreads();
    stamp();  // K + 2: border
    // ---- back-substitution, top level first: y_i = L_i^-T (x_i - XL_i y_l - XR_i y_r - XB_i y_k)
    for (int m = K; m >= 0; --m) {
        const int s = 1 << m;
        const int ne = ((nb >> m) + 1) >> 1;
        for (int s0 = 0; s0 < ne; s0 += 2 * NW_BAND) {
            const int slot = s0 + 2 * wave + (hi ? 1 : 0);
            const bool act = slot < ne;
            const int i = act ? ((2 * slot + 1) << m) - 1 : 0;
            const int r = hl < G ? hl : G - 1;
            const int lb = i - s, rb = i + s;
            const bool hl_ = lb >= 0, hr = rb < nb;
            double w0 = BV[i * G + r], w1 = 0.0, w2 = 0.0;
#pragma unroll
            for (int u = 0; u < G; ++u) {
                w1 = __builtin_fma(CL[i * GG + r * G + u], hl_ ? YV[(hl_ ? lb : 0) * G + u] : 0.0, w1);
                w2 = __builtin_fma(XR[i * GG + r * G + u], hr ? YV[(hr ? rb : 0) * G + u] : 0.0, w2);
                if (u % 6 == 5) narrow_live_range<G>();
            }
            double w3 = 0.0;
#pragma unroll
            for (int k = 0; k < 4; ++k) w3 = __builtin_fma(BBm[(i * G + r) * 4 + k], yk[k], w3);
            double w = ((w0 - w1) - w2) - w3;
            const double* Li = Dm + i * GG;
            double yv = 0.0;
#pragma unroll
            for (int R = G - 1; R >= 0; --R) {
                const double yR = bcast_half(w, R, hi) * RI[i * G + R];
                yv = hl == R ? yR : yv;
                if (hl < R) w = __builtin_fma(-Li[R * G + r], yR, w);
                if (R % 6 == 0) narrow_live_range<G>();
            }
            if (act && hl < G) YV[i * G + hl] = yv;
        }
        __syncthreads();
    }
    stamp();  // K + 3: back-substitution
    // ---- y to rhs (the points' back-substitution reads it), the poses into the staged operands
    for (int d = tid; d < ncd + 4; d += TPB_BAND) rhs[d] = d < ncd ? YV[d] : yk[d - ncd];
    if (tid < nx) lds[Ly.OPS + (tid / 7) * BAND_OPS + 18 + tid % 7] = xv;
    __syncthreads();
    // ---- the step (block_step's arithmetic and grouping: wave w = cameras [10 w, 10 w + 10), w = 0 also the
    // intrinsics; part slot w)
    const int nupd = (nac + BCR_CAMS - 1) / BCR_CAMS;
    for (int w = wave; w < nupd; w += NW_BAND) {
        double acc[4] = {0.0, 0.0, 0.0, 0.0};  // sn2, mcc, cand cost, |x_cand|^2
        const int t = w * BCR_CAMS + lane;
        if (lane < BCR_CAMS && t < nac) {
            CamStepOps o;
            const double* op = lds + Ly.OPS + t * BAND_OPS;
            o.cam = AC[t];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                o.sc[k] = op[k];
                o.ud[k] = op[6 + k];
                o.g[k] = op[12 + k];
            }
#pragma unroll
            for (int k = 0; k < 7; ++k) o.x[k] = op[18 + k];
            cam_step(P, c, cur, radius, o, t, YV + 6 * t, delta, acc);
        } else if (w == 0 && lane == BCR_CAMS) {
            IntrStepOps o;
            const double* op = lds + Ly.IOPS;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                o.K[k] = op[k];
                o.sk[k] = op[4 + k];
                o.uk[k] = op[8 + k];
                o.gk[k] = op[12 + k];
                o.prior[k] = op[16 + k];
            }
            intr_step(P, c, cur, radius, o, yk, delta, acc);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1)
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[k] += __shfl_xor(acc[k], off);
        if (lane == 0) {
            part[PART_UPD_SN2 * P.part_stride + w] = acc[0];
            part[PART_UPD_MCC * P.part_stride + w] = acc[1];
            part[PART_UPD_COST * P.part_stride + w] = acc[2];
            part[PART_UPD_XN2 * P.part_stride + w] = acc[3];
        }
    }
    stamp();  // K + 4: step
}

static size_t band_lds_bytes(int bc, int nb, int nac) { return sizeof(double) * (size_t)band_layout(6 * bc, nb, nac).total; }

// The band path for this window: cameras per block (1..3), 0 when it does not apply. mode: MIBA_BCR_BAND
// (0 off, 2 also for one-block windows, else the default: windows of more than one 64-dof BCR block).
int bcr_band_ok(int nac, int cam_band, int kb) {
    if (nac < 2 || cam_band > 3 || std::getenv("MIBA_BCR")) return 0;
    const char* e = std::getenv("MIBA_BCR_BAND");
    const int mode = e ? std::atoi(e) : 1;
    if (mode == 0) return 0;
    if (mode != 2 && nac <= BCR_CAMS && kb + 4 <= 64) return 0;  // one BCR block: k_bcr_dense1
    const int bc = cam_band < 1 ? 1 : cam_band;
    const int nb = (nac + bc - 1) / bc;
    int dev = 0, lmax = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&lmax, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess)
        return 0;
    if (lmax < 160 * 1024) lmax = 160 * 1024;  // gfx950: 160 KB per workgroup (the attribute may report 64 KB)
    return band_lds_bytes(bc, nb, nac) <= (size_t)lmax ? bc : 0;
}

#define CKD(x)                            \
    do {                                  \
        hipError_t e_ = (x);              \
        if (e_ != hipSuccess) return e_;  \
    } while (0)

template <int BC>
static hipError_t launch_band_t(const DevProblem& P, const BaConsts& c, DevWork& W, int nb, hipStream_t s, Prof* pf) {
    static bool attr = false;
    static int smode = -1;
    static unsigned long long* dst = nullptr;
    if (!attr) {
        CKD(hipFuncSetAttribute((const void*)k_bcr_band<BC, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024));
        CKD(hipFuncSetAttribute((const void*)k_bcr_band<BC, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024));
        const char* e = std::getenv("MIBA_BCR_STAMPS");
        smode = (e && e[0] == '1') ? 1 : 0;
        attr = true;
    }
    const size_t lds = band_lds_bytes(BC, nb, P.nac);
    if (smode) {
        if (!dst) CKD(hipMalloc(&dst, BAND_STAMPS * sizeof(unsigned long long)));
        CKD(hipMemsetAsync(dst, 0, BAND_STAMPS * sizeof(unsigned long long), s));
        if (pf) pf->begin(K_BCR_PERSIST, s);
        hipLaunchKernelGGL((k_bcr_band<BC, true>), dim3(1), dim3(BandTpb<BC>::TPB), lds, s, W.st, P, W.S, W.rhs, W.chol_flag, c,
                           W.scale, W.camdata, W.lin, W.delta, W.part, nb, dst);
        if (pf) pf->end(s);
        CKD(hipGetLastError());
        unsigned long long h[BAND_STAMPS];
        CKD(hipMemcpyAsync(h, dst, sizeof(h), hipMemcpyDeviceToHost, s));
        CKD(hipStreamSynchronize(s));
        if (h[0]) {  // (0: the launch exited at once, skip_step)
            int K = 0;
            while ((2 << K) <= nb) ++K;
            std::fprintf(stderr, "bcr_band<%d> nb=%d us:", BC, nb);
            const unsigned long long t0 = h[BAND_STAMPS - 1];
            for (int k = 0; k <= K + 4; ++k) std::fprintf(stderr, " %.2f", (double)(h[k] - t0) / 100.0);
            std::fprintf(stderr, "  (loaded, levels 0..%d, border, back, step)\n", K);
        }
        return hipSuccess;
    }
    if (pf) pf->begin(K_BCR_PERSIST, s);
    hipLaunchKernelGGL((k_bcr_band<BC, false>), dim3(1), dim3(BandTpb<BC>::TPB), lds, s, W.st, P, W.S, W.rhs, W.chol_flag, c,
                       W.scale, W.camdata, W.lin, W.delta, W.part, nb, (unsigned long long*)nullptr);
    if (pf) pf->end(s);
    return hipGetLastError();
}

hipError_t launch_bcr_band(const DevProblem& P, const BaConsts& c, DevWork& W, int bc, hipStream_t s, Prof* pf) {
    const int nb = (P.nac + bc - 1) / bc;
    switch (bc) {
        case 1: return launch_band_t<1>(P, c, W, nb, s, pf);
        case 2: return launch_band_t<2>(P, c, W, nb, s, pf);
        case 3: return launch_band_t<3>(P, c, W, nb, s, pf);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace miba
