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

#include <vector>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "ba_device.h"
#include "ba_kernels.h"
#include "ba_solve_util.h"
#include "ba_tail.h"

namespace miba {

// one workgroup of 8 waves (2 per SIMD: the 256-VGPR budget; at 16 waves the kernel spilled, and the element-parallel
// phases are issue-bound, so more waves per SIMD add nothing)
static constexpr int BAND_TPB = 512;
static constexpr int BAND_OPS = 25;    // staged camera-step operands per active camera: sc 6 | ud 6 | g 6 | x 7
static constexpr int BAND_IOPS = 20;   // intrinsics: K 4 | sk 4 | uk 4 | gk 4 | prior 4
static constexpr int BAND_STAMPS = 24;
static constexpr int BAND_FSTAMPS = 8 * 8;  // STAMP: inside each level's factor phase, unit 0 of wave 0

// LDS layout (doubles) of one window: per block j (nb blocks of G dofs, block-major = dof order)
//   D  G x G   diagonal block, then L_j (lower; upper zero) once j is eliminated
//   CL G x G   coupling to the current left neighbour A(j, j - 2^m), then XL_j
//   XR G x G   XR_j
//   BB G x 4   border rows B_j, then XB_j
//   BV G       rhs b_j, then x_j;   RI G   1 / diag(L_j);   YV G   y_j
// then bk = [b_k | S_kk lower packed] (14) | red (20) | y_k (4), the intrinsics' and cameras' step operands and
// the active cameras' indices (ints, two per double).
struct BandLayout {
    int D, CL, XR, BB, BV, RI, YV, BK, RED, YK, IOPS, OPS, AC, ST, total;
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
    L.BK = o;   o += 16;
    L.RED = o;  o += 24;
    L.YK = o;   o += 8;
    L.IOPS = o; o += BAND_IOPS;
    L.OPS = o;  o += nac * BAND_OPS;
    L.AC = o;   o += (nac + 1) / 2 + 1;
    L.ST = o;   o += BAND_STAMPS + BAND_FSTAMPS;
    L.total = o;
    return L;
}

// lane j of this lane's half-wave to every lane of the half (two v_readlane pairs and a select)
__device__ __forceinline__ double bcast_half(double v, int j, bool hi) {
    const double lo = bcast_b(v, j), up = bcast_b(v, 32 + j);
    return hi ? up : lo;
}
// A block's rows live on one unit of U lanes: a 16-lane DPP row when the block has <= 16 dofs (four blocks per wave;
// the broadcast of lane J to its row is one v_mov_b32_dpp row_newbcast per dword, gfx90a+), else a half-wave
// (v_readlane pairs and a select — on the chain that costs ~2x the DPP move, measured)
template <int G>
struct BandUnit {
    static constexpr int U = G <= 16 ? 16 : 32;
    static constexpr int PER_WAVE = 64 / U;
};
template <int U, int J>
__device__ __forceinline__ double ubc(double v, bool hi) {
    if constexpr (U == 16) {
        const unsigned long long u = __double_as_longlong(v);
        const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, 0x150 + J, 0xF, 0xF, false);
        const int up = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), 0x150 + J, 0xF, 0xF, false);
        return __longlong_as_double((long long)(((unsigned long long)(unsigned)up << 32) | (unsigned)lo));
    } else {
        return bcast_half(v, J, hi);
    }
}
// 4x4 border system as border_solve4 (bk = [b_k | S_kk lower packed], red[m * 5 + c] = (B^T [u | V])[m][c]), the
// Cholesky pivots by v_rsq_f64 + one Newton step and the solves by products: no square root or division on the path
// (border_solve4's IEEE square roots and divisions took ~1.5 us here). bad: a non-positive pivot.
__device__ __forceinline__ void border_solve4_rsq(const double* bk, const double* red, double* yk, bool& bad) {
    double Cm[16], bp[4];
    int q = 0;
    for (int mm = 0; mm < 4; ++mm)
        for (int l = 0; l <= mm; ++l, ++q) {
            const double v = bk[4 + q];
            Cm[mm * 4 + l] = v - red[mm * 5 + 1 + l];
        }
    for (int mm = 0; mm < 4; ++mm) bp[mm] = bk[mm] - red[mm * 5];
    double Lm[16] = {0}, ri[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        double d = Cm[j * 4 + j];
#pragma unroll
        for (int k = 0; k < j; ++k) d = __builtin_fma(-Lm[j * 4 + k], Lm[j * 4 + k], d);
        if (!(d > 0.0 && d < INFINITY)) { bad = true; d = 1.0; }
        const double y = __builtin_amdgcn_rsq(d);
        const double ee = __builtin_fma(-d * y, y, 1.0);
        const double yi = __builtin_fma(0.5 * y, ee, y);  // 1 / L_jj
        ri[j] = yi;
        Lm[j * 4 + j] = d * yi;
#pragma unroll
        for (int r = j + 1; r < 4; ++r) {
            double v = Cm[r * 4 + j];
#pragma unroll
            for (int k = 0; k < j; ++k) v = __builtin_fma(-Lm[r * 4 + k], Lm[j * 4 + k], v);
            Lm[r * 4 + j] = v * yi;
        }
    }
    double z[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        double v = bp[r];
#pragma unroll
        for (int k = 0; k < r; ++k) v = __builtin_fma(-Lm[r * 4 + k], z[k], v);
        z[r] = v * ri[r];
    }
#pragma unroll
    for (int r = 3; r >= 0; --r) {
        double v = z[r];
#pragma unroll
        for (int k = r + 1; k < 4; ++k) v = __builtin_fma(-Lm[k * 4 + r], z[k], v);
        z[r] = v * ri[r];
    }
    for (int mm = 0; mm < 4; ++mm) yk[mm] = z[mm];
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

// Operands of one output element of a survivor update (decoded once per thread, before the level loop): the element
// is dest = (keep ? dest : 0) - sum_u a1[u G] b1[u bs] - [second source] sum_u a2[u G] b2[u bs], a1 / a2 the column r
// of XR_i1 / XL_i2; b1 / b2 a column of one of the block arrays at the blocks i1 / i2 (stride bblk per block); dest
// in the survivor's block, mirrored for the diagonal block's upper half.
struct BandItem {
    int ok, r, b1_arr, b2_arr, boff, bs, dst_arr, doff, mirror, two, keep;
};

template <int BC, bool STAMP, bool PUB = false>
__device__ __forceinline__ void band_body(const LmState* __restrict__ st, const DevProblem& P,
                                          const double* __restrict__ S, double* __restrict__ rhs,
                                          int* __restrict__ flag, const BaConsts& c, const double* __restrict__ scale,
                                          const double* __restrict__ camdata, const double* __restrict__ lin,
                                          double* __restrict__ delta, double* __restrict__ part, int nb,
                                          unsigned long long* __restrict__ tl, double* __restrict__ lds,
                                          unsigned* __restrict__ yflag = nullptr, unsigned yseq = 0,
                                          double* __restrict__ ybuf = nullptr) {
    constexpr int G = 6 * BC;
    constexpr int GG = G * G;
    constexpr int TPB = BAND_TPB, NW = BAND_TPB / 64;
    constexpr int NCOL = 2 * G + 5;  // [XL | XR | x | XB] columns of the forward solve
    constexpr int U = BandUnit<G>::U, UPW = BandUnit<G>::PER_WAVE;
    constexpr bool FUSE = G == 6;  // the forward solve inside the factor unit (blocks of one camera)
    constexpr int ND = G * (G + 1) / 2;
    constexpr int NSI = ND + G + 4 * G + GG;      // output elements per survivor: D lower | b | B | fill
    constexpr int NQ = (NSI + TPB - 1) / TPB;     // elements per thread and survivor
    constexpr int GRP = NSI <= TPB ? TPB / NSI : 1;  // survivors per pass
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool hi = lane >= 32;
    const int ul = lane & (U - 1);
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
    int* const AC = reinterpret_cast<int*>(lds + Ly.AC);
    // STAMP: s_memrealtime after each phase, kept in LDS until the end (a global store before a barrier would make
    // the barrier's workgroup fence wait for its acknowledgement)
    unsigned long long* const stl = reinterpret_cast<unsigned long long*>(lds + Ly.ST);
    int ts = 0;
    auto stamp = [&]() {
        if constexpr (STAMP) {
            __syncthreads();
            if (tid == 0) stl[ts] = realtime_now();
            ++ts;
        }
    };
    if constexpr (STAMP) if (tid == 0) stl[BAND_STAMPS - 1] = realtime_now();
    // STAMP: wave 0 lane 0 inside the factor phase of level m (no barrier): slot BAND_STAMPS + 8 m + k
    auto fst = [&](int m, int k) {
        if constexpr (STAMP) if (tid == 0 && m < 8) stl[BAND_STAMPS + 8 * m + k] = realtime_now();
    };
    const bool skip = skip_step(st);
    const int cur = st->cur;
    // ---- load. Camera dof rows: one thread per row dr of block j, its 2G contiguous doubles of S row dr at columns
    // (j - 1) G .. j G + G - 1 (the coupling A(j, j - 1) and the diagonal block's lower part; the upper part stays
    // zero, the pivot chain reads only the lower), its border entries S[kb + k][dr] and rhs[dr]; identity past the
    // last camera dof. Cameras: their step operands (the pose after the camera index), on the threads from the top.
    const int nrow = nb * G;
    {
        // The 2G doubles of S row dr at columns (j - 1) G .. j G + G - 1, element e = 2G dr + cc: consecutive threads
        // read consecutive columns (a thread per row read 2G lines per wave and instruction: 4.2 us at C3). The first
        // pass of these, this thread's border row and rhs entry, its camera's step operands and its bk / intrinsics
        // operand are ALL loaded before any is stored to LDS: one memory round trip for the load phase instead of one
        // per loop (each loop waited for its own loads); larger windows' further passes / rows / cameras follow.
        constexpr int NL = 8;
        const int ne2 = nrow * 2 * G;
        auto s_load = [&](int e) {
            const int dr = e / (2 * G), cc = e - dr * (2 * G), j = dr / G, r = dr - j * G;
            const int col = (j - 1) * G + cc;
            const bool okc = e < ne2 && dr < ncd && col >= 0 && (cc < G || cc - G <= r);
            const double v = S[okc ? (size_t)dr * ld + col : 0];
            return okc ? v : ((e < ne2 && dr >= ncd && cc - G == r) ? 1.0 : 0.0);  // identity past the dofs
        };
        auto s_store = [&](int e, double v) {
            if (e < ne2) {
                const int dr = e / (2 * G), cc = e - dr * (2 * G), j = dr / G, r = dr - j * G;
                lds[(cc < G ? Ly.CL : Ly.D) + j * GG + r * G + (cc < G ? cc : cc - G)] = v;
            }
        };
        // border entries S[kb + k][dr] and rhs[dr] (coalesced over dr)
        auto b_load = [&](int dr, double (&bb)[5]) {
            const bool ok = dr < ncd;
#pragma unroll
            for (int k = 0; k < 4; ++k) bb[k] = S[(size_t)(ncd + k) * ld + (ok ? dr : 0)];
            bb[4] = rhs[ok ? dr : 0];
#pragma unroll
            for (int k = 0; k < 5; ++k) bb[k] = ok ? bb[k] : 0.0;
        };
        auto b_store = [&](int dr, const double (&bb)[5]) {
#pragma unroll
            for (int k = 0; k < 4; ++k) BBm[dr * 4 + k] = bb[k];
            BV[dr] = bb[4];
        };
        // the cameras' step operands (load_cam_step_ops), on the threads from the top
        auto c_load = [&](int t, double (&o)[18]) {
            const double* cd = camdata + (size_t)t * CAMDATA;
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                o[k] = scale[6 * (size_t)t + k];
                o[6 + k] = cd[k * 6 - (k * (k - 1)) / 2];
                o[12 + k] = cd[45 + k];
            }
            return P.ac_cam[t];
        };
        auto c_store = [&](int t, const double (&o)[18], int cam) {
#pragma unroll
            for (int k = 0; k < 18; ++k) lds[Ly.OPS + t * BAND_OPS + k] = o[k];
            AC[t] = cam;
        };
        double v[NL];
#pragma unroll
        for (int q = 0; q < NL; ++q) v[q] = s_load(q * TPB + tid);
        const bool hb = tid < nrow;
        double bb0[5];
        b_load(hb ? tid : 0, bb0);
        const int t0 = TPB - 1 - tid;
        const bool hc = t0 < nac;
        double o0[18];
        const int cam0 = c_load(hc ? t0 : 0, o0);
        // bk = [b_k | S_kk lower packed] (14) | intrinsics' step operands (20)
        const bool hk = tid >= TPB / 2 && tid < TPB / 2 + 34;
        double kv = 0.0;
        int kdst = 0;
        if (hk) {
            const int f = tid - TPB / 2;
            const double* p;
            size_t idx;
            if (f < 4) {
                p = rhs; idx = ncd + f; kdst = Ly.BK + f;
            } else if (f < 14) {
                const int q2 = f - 4, mm = q2 < 1 ? 0 : q2 < 3 ? 1 : q2 < 6 ? 2 : 3, l = q2 - mm * (mm + 1) / 2;
                p = S; idx = (size_t)(ncd + mm) * ld + ncd + l; kdst = Ly.BK + f;
            } else {
                const int g = f - 14, kind = g >> 2, m = g & 3;
                p = kind == 0 ? P.K[cur] : kind == 1 ? scale : kind == 4 ? P.prior : lin;
                idx = kind == 0 ? m : kind == 1 ? P.off_k + m : kind == 2 ? 2 + 4 * m - (m * (m - 1)) / 2 : kind == 3 ? 12 + m : m;
                kdst = Ly.IOPS + g;
            }
            kv = p[idx];
        }
#pragma unroll
        for (int q = 0; q < NL; ++q) s_store(q * TPB + tid, v[q]);
        if (hb) b_store(tid, bb0);
        if (hc) c_store(t0, o0, cam0);
        if (hk) lds[kdst] = kv;
        for (int e0 = NL * TPB; e0 < ne2; e0 += NL * TPB) {
#pragma unroll
            for (int q = 0; q < NL; ++q) v[q] = s_load(e0 + q * TPB + tid);
#pragma unroll
            for (int q = 0; q < NL; ++q) s_store(e0 + q * TPB + tid, v[q]);
        }
        for (int dr = tid + TPB; dr < nrow; dr += TPB) {
            double bb[5];
            b_load(dr, bb);
            b_store(dr, bb);
        }
        for (int t = t0 + TPB; t < nac; t += TPB) {
            double o[18];
            const int cam = c_load(t, o);
            c_store(t, o, cam);
        }
    }
    if (skip) return;
    const double radius = st->radius;
    // ---- this thread's survivor-update elements: decoded once (blocks of <= 12 dofs; the wider blocks' two elements
    // per thread would hold 22 registers through the level loop, and the kernel spilled: decoded per use there)
    auto decode = [&](int k) {
        const int q = NQ == 1 ? tid % NSI : tid + k * TPB;
        BandItem I;
        I.ok = (NQ == 1 ? tid / NSI < GRP : q < NSI) ? 1 : 0;
        I.two = 1;
        I.keep = 1;
        I.mirror = -1;
        if (q < ND) {  // D_j (r, cc), cc <= r: XR_i1^T XR_i1 + XL_i2^T XL_i2
            int r = 0;
            while ((r + 1) * (r + 2) / 2 <= q) ++r;
            const int cc = q - r * (r + 1) / 2;
            I.r = r; I.b1_arr = Ly.XR; I.b2_arr = Ly.CL; I.boff = cc; I.bs = G;
            I.dst_arr = Ly.D; I.doff = r * G + cc; I.mirror = cc * G + r;
        } else if (q < ND + G) {  // b_j: x
            I.r = q - ND; I.b1_arr = I.b2_arr = Ly.BV; I.boff = 0; I.bs = 1;
            I.dst_arr = Ly.BV; I.doff = I.r;
        } else if (q < ND + 5 * G) {  // B_j (r, k)
            const int f = q - ND - G;
            I.r = f >> 2; I.b1_arr = I.b2_arr = Ly.BB; I.boff = f & 3; I.bs = 4;
            I.dst_arr = Ly.BB; I.doff = f;
        } else {  // the fill A(j, j - 2s) = -XR_i1^T XL_i1
            const int f = q < NSI ? q - ND - 5 * G : 0, r = f / G, cc = f - r * G;
            I.r = r; I.b1_arr = I.b2_arr = Ly.CL; I.boff = cc; I.bs = G; I.two = 0; I.keep = 0;
            I.dst_arr = Ly.CL; I.doff = f;
        }
        return I;
    };
    constexpr bool PRE = G <= 12;
    BandItem it[PRE ? NQ : 1];
    if constexpr (PRE)
#pragma unroll
        for (int k = 0; k < NQ; ++k) it[k] = decode(k);
    const int grp = NQ == 1 ? tid / NSI : 0;
    // per-block strides of the arrays (doubles): D / CL / XR GG, BB 4G, BV G
    auto bstride = [&](int arr) { return arr == Ly.BB ? 4 * G : arr == Ly.BV ? G : GG; };
    __syncthreads();
    // the poses of the step (a dependent load: the camera index first), in flight through the elimination
    const int nx = 7 * nac;
    double xv[2] = {0.0, 0.0};
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int e = tid + q * TPB;
        if (e < nx) xv[q] = P.cams[cur][7 * (size_t)AC[e / 7] + e % 7];
    }
    stamp();  // 0: loaded
    // K = floor(log2 nb): the root is block 2^K - 1, eliminated at level K with no neighbour
    int K = 0;
    while ((2 << K) <= nb) ++K;
    bool bad = false;
    for (int m = 0; m <= K; ++m) {
        const int s = 1 << m;
        const int ne = ((nb >> m) + 1) >> 1;  // blocks i with i + 1 = odd * 2^m, i < nb
        // ---- factor, one unit (U lanes, lane = row) per eliminated block
        for (int s0 = 0; s0 < ne; s0 += UPW * NW) {
            const int slot = s0 + wave * UPW + lane / U;
            const bool act = slot < ne;
            const int i = act ? ((2 * slot + 1) << m) - 1 : 0;
            const int r = ul < G ? ul : G - 1;
            if (s0 == 0) fst(m, 0);
            double a[G];
#pragma unroll
            for (int k = 0; k < G; ++k) a[k] = Dm[i * GG + r * G + k];
            double my_inv = 0.0;
            double dn = ubc<U, 0>(a[0], hi);
            if (s0 == 0) fst(m, 1);
            sfor<0, G>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                const double dd = dn;
                bad = bad || (act && !(dd > 0.0 && dd < INFINITY));
                const double y = __builtin_amdgcn_rsq(dd);
                const double ee = __builtin_fma(-dd * y, y, 1.0);
                const double l = __builtin_fma(0.5 * a[j] * y, ee, a[j] * y);
                my_inv = (ul == j) ? __builtin_fma(0.5 * y, ee, y) : my_inv;
                a[j] = l;
                if constexpr (j + 1 < G) {
                    dn = ubc<U, j + 1>(__builtin_fma(-l, l, a[j + 1]), hi);
                    sfor<j + 1, G>([&](auto kc) {
                        constexpr int k = decltype(kc)::value;
                        // a 16-lane unit: one v_fmac_f64_dpp per column (row_newbcast hands lane k's l to the FMA)
                        if constexpr (U == 16) fnma_row_bcast<k, k == j + 1>(a[k], l, l);
                        else a[k] = __builtin_fma(-l, ubc<U, k>(l, hi), a[k]);
                    });
                }
            });
            if (s0 == 0) fst(m, 2);
            if (act && ul < G) {
#pragma unroll
                for (int k = 0; k < G; ++k) Dm[i * GG + ul * G + k] = k <= ul ? a[k] : 0.0;
                RI[i * G + ul] = my_inv;
            }
            wave_sync();
            if (s0 == 0) fst(m, 3);
            // forward solve by the same unit (lane = column; lanes < NCOL - U take a second column, interleaved), no
            // workgroup barrier between a block's factorisation and its solve:
            // [XL | XR | x | XB] = L_i^-1 [A(i, i - s) | A(i, i + s) = A(i + s, i)^T | b_i | B_i]
            // (blocks of one camera; the wider blocks' two columns per lane spill: they take the separate phase below)
            if (FUSE && act) {
                const int rb = i + s;
                const bool has_r = rb < nb;
                const double* Li = Dm + i * GG;
                const double* ri = RI + i * G;
                constexpr int NCP = (NCOL + U - 1) / U;  // columns per lane
                double x[NCP][G];
                double* out[NCP];
                int ostride[NCP];
                bool live[NCP];
#pragma unroll
                for (int p = 0; p < NCP; ++p) {
                    const int col = ul + p * U;
                    live[p] = col < NCOL;
                    // the column as (base, stride): A(i, i - s) column col in place (-> XL); A(i + s, i) row col - G
                    // (-> XR_i); b_i (-> x); B_i column k (-> XB)
                    const double* src;
                    int stride;
                    if (col < G) {
                        out[p] = CL + i * GG + col; src = out[p]; stride = G; ostride[p] = G;
                    } else if (col < 2 * G) {
                        src = CL + (has_r ? rb : i) * GG + (col - G) * G; out[p] = XR + i * GG + col - G; stride = 1;
                        ostride[p] = G;
                    } else if (col == 2 * G) {
                        out[p] = BV + i * G; src = out[p]; stride = 1; ostride[p] = 1;
                    } else {
                        const int k = live[p] ? col - 2 * G - 1 : 0;
                        out[p] = BBm + i * G * 4 + k; src = out[p]; stride = 4; ostride[p] = 4;
                    }
                    const bool zero = !live[p] || (col >= G && col < 2 * G && !has_r);
#pragma unroll
                    for (int q = 0; q < G; ++q) x[p][q] = zero ? 0.0 : src[q * stride];
                }
                if (s0 == 0) fst(m, 4);
#pragma unroll
                for (int j = 0; j < G; ++j) {
                    const double rj = ri[j];
#pragma unroll
                    for (int p = 0; p < NCP; ++p) x[p][j] *= rj;
#pragma unroll
                    for (int q = j + 1; q < G; ++q) {
                        const double lq = Li[q * G + j];
#pragma unroll
                        for (int p = 0; p < NCP; ++p) x[p][q] = __builtin_fma(-lq, x[p][j], x[p][q]);
                    }
                    narrow_live_range<G>();
                }
                if (s0 == 0) fst(m, 5);
#pragma unroll
                for (int p = 0; p < NCP; ++p)
                    if (live[p])
#pragma unroll
                        for (int q = 0; q < G; ++q) out[p][q * ostride[p]] = x[p][q];
            }
            if (s0 == 0) fst(m, 6);
        }
        __syncthreads();
        if constexpr (!FUSE) {
            // ---- forward solve (blocks of 2-3 cameras): thread (fgrp, fcol) takes column fcol of the blocks fgrp,
            // fgrp + FGRP, ...
            const int fcol = tid % NCOL, fgrp = tid / NCOL;
            constexpr int FGRP = TPB / NCOL;
            for (int g = fgrp; g < ne && fgrp < FGRP; g += FGRP) {
                const int i = ((2 * g + 1) << m) - 1;
                const int rb = i + s;
                const bool has_r = rb < nb;
                const double* Li = Dm + i * GG;
                const double* ri = RI + i * G;
                const double* src;
                double* out;
                int stride, ostride;
                if (fcol < G) {
                    out = CL + i * GG + fcol; src = out; stride = G; ostride = G;
                } else if (fcol < 2 * G) {
                    src = CL + (has_r ? rb : i) * GG + (fcol - G) * G; out = XR + i * GG + fcol - G; stride = 1;
                    ostride = G;
                } else if (fcol == 2 * G) {
                    out = BV + i * G; src = out; stride = 1; ostride = 1;
                } else {
                    out = BBm + i * G * 4 + fcol - 2 * G - 1; src = out; stride = 4; ostride = 4;
                }
                const bool zero = fcol >= G && fcol < 2 * G && !has_r;
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
            __syncthreads();
        }
        stamp();  // 1 + 2m: level m factored
        // ---- survivors pull their eliminated neighbours' Schur terms (every thread the same code: its elements'
        // operands were decoded before the loop); eliminated blocks form their border Gram
        const int ns = m < K ? nb >> (m + 1) : 0;  // survivors j with j + 1 = multiple of 2^(m+1)
        for (int t = grp; t < ns; t += GRP) {
            const int j = ((t + 1) << (m + 1)) - 1, i1 = j - s, i2 = j + s;
            const bool h2 = i2 < nb;
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                BandItem I;
                if constexpr (PRE) I = it[k];
                else I = decode(k);
                if (!I.ok) continue;
                const double* a1 = XR + i1 * GG + I.r;                 // column r of XR_i1
                const double* a2 = CL + (h2 ? i2 : i1) * GG + I.r;     // column r of XL_i2
                const double* b1 = lds + I.b1_arr + i1 * bstride(I.b1_arr) + I.boff;
                const double* b2 = lds + I.b2_arr + (h2 ? i2 : i1) * bstride(I.b2_arr) + I.boff;
                double acc1 = 0.0, acc2 = 0.0;
#pragma unroll
                for (int u = 0; u < G; ++u) {
                    acc1 = __builtin_fma(a1[u * G], b1[u * I.bs], acc1);
                    acc2 = __builtin_fma(a2[u * G], b2[u * I.bs], acc2);
                    if (u % 6 == 5) narrow_live_range<G>();
                }
                double* d = lds + I.dst_arr + j * bstride(I.dst_arr);
                const double v = ((I.keep ? d[I.doff] : 0.0) - acc1) - ((I.two && h2) ? acc2 : 0.0);
                d[I.doff] = v;
                if (I.mirror >= 0) d[I.mirror] = v;
            }
        }
        if (ns > 0) {
            __syncthreads();
            stamp();  // 2 + 2m: level m's survivors updated
        }
    }
    // ---- border system. Every block's XB and x are final once it is eliminated, and the blocks are stored in dof
    // order, so sum_i XB_i^T [XB_i | x_i] is one dot product over the camera dof rows: 14 sums, each split over 32
    // lanes (rows r = lane, lane + 32, ...) and reduced in a fixed order; then (C - B^T V) y_k = b_k - B^T u on one lane
    double* const red = lds + Ly.RED;
    double* const yk = lds + Ly.YK;
    {
        constexpr int SPL = 32;
        for (int o = tid / SPL; o < 14; o += TPB / SPL) {
            const int p = tid % SPL;
            const int k = o < 1 ? 0 : o < 3 ? 1 : o < 6 ? 2 : o < 10 ? 3 : o - 10;
            const int l = o < 10 ? o - k * (k + 1) / 2 : 0;
            double acc = 0.0;
            for (int rr = p; rr < nrow; rr += SPL)
                acc = __builtin_fma(BBm[rr * 4 + k], o < 10 ? BBm[rr * 4 + l] : BV[rr], acc);
#pragma unroll
            for (int off = 1; off < SPL; off <<= 1) acc += __shfl_xor(acc, off);  // fixed butterfly order
            if (p == 0) {
                if (o < 10) {
                    red[k * 5 + 1 + l] = acc;
                    red[l * 5 + 1 + k] = acc;
                } else {
                    red[k * 5] = acc;
                }
            }
        }
        __syncthreads();
        if (tid == 0) {
            bool bb = false;
            border_solve4_rsq(lds + Ly.BK, red, yk, bb);
            bad = bad || bb;
        }
    }
    if (bad && ul == 0) raise_flag(flag, FLAG_NOT_PD);
    __syncthreads();
    stamp();  // 2K + 3: border
    // ---- back-substitution, top level first, one unit (lane = row) per block:
    // y_i = L_i^-T (x_i - XL_i y_l - XR_i y_r - XB_i y_k)
    for (int m = K; m >= 0; --m) {
        const int s = 1 << m;
        const int ne = ((nb >> m) + 1) >> 1;
        for (int s0 = 0; s0 < ne; s0 += UPW * NW) {
            const int slot = s0 + wave * UPW + lane / U;
            const bool act = slot < ne;
            const int i = act ? ((2 * slot + 1) << m) - 1 : 0;
            const int r = ul < G ? ul : G - 1;
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
            if constexpr (U == 16) {
                // a 16-lane unit: y_R = w_R / L_RR on lane R, and w_r += w_R (-L_Rr / L_RR) on every lane in ONE
                // v_fmac_f64_dpp (row_newbcast:R hands lane R's w to the row; the coefficients are loaded and formed
                // first, off the chain) — one dependent instruction per step instead of the broadcast, the product and
                // the FMA. (Lanes >= R take updates they never read again.)
                double rv[G], cf[G];
                sfor<0, G>([&](auto Rc) {
                    constexpr int R = decltype(Rc)::value;
                    rv[R] = RI[i * G + R];
                    cf[R] = -Li[R * G + r] * rv[R];
                });
                sfor<0, G>([&](auto Rc) {
                    constexpr int R = G - 1 - decltype(Rc)::value;
                    yv = ul == R ? w * rv[R] : yv;
                    if constexpr (R > 0) fmac_self_row_bcast<R>(w, cf[R]);
                });
            } else {
                sfor<0, G>([&](auto Rc) {
                    constexpr int R = G - 1 - decltype(Rc)::value;
                    const double yR = ubc<U, R>(w, hi) * RI[i * G + R];
                    yv = ul == R ? yR : yv;
                    if (ul < R) w = __builtin_fma(-Li[R * G + r], yR, w);
                });
            }
            if (act && ul < G) YV[i * G + ul] = yv;
        }
        __syncthreads();
    }
    stamp();  // 2K + 4: back-substitution
    // ---- y to rhs (the points' back-substitution reads it); the step (block_step's arithmetic and grouping: wave w =
    // cameras [10 w, 10 w + 10), w = 0 also the intrinsics; part slot w)
    // (the band tail: y to its flag-free hand-off buffer, which the chunks poll; else to rhs)
    for (int d = tid; d < ncd + 4; d += TPB) st_opt<PUB>((ybuf ? ybuf : rhs) + d, d < ncd ? YV[d] : yk[d - ncd]);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int e = tid + q * TPB;
        if (e < nx) lds[Ly.OPS + (e / 7) * BAND_OPS + 18 + e % 7] = xv[q];
    }
    // the band tail: y drained by every thread, then published before the step (the chunks compute their candidate
    // poses from y themselves, so the step runs beside them instead of ahead of them)
    if (yflag) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (yflag && tid == 0) __hip_atomic_store(yflag, yseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int nupd = (nac + BCR_CAMS - 1) / BCR_CAMS;
    for (int w = wave; w < nupd; w += NW) {
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
            cam_step<PUB>(P, c, cur, radius, o, t, YV + 6 * t, delta, acc);
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
            intr_step<PUB>(P, c, cur, radius, o, yk, delta, acc);
        }
        // (lanes >= 16 hold no term: a 16-lane butterfly in a fixed order)
        static_assert(BCR_CAMS + 1 <= 16, "the step's terms sit on lanes < 16");
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] = dpp_row_sum(acc[k]);
        if (lane == 0) {
            st_opt<PUB>(part + PART_UPD_SN2 * P.part_stride + w, acc[0]);
            st_opt<PUB>(part + PART_UPD_MCC * P.part_stride + w, acc[1]);
            st_opt<PUB>(part + PART_UPD_COST * P.part_stride + w, acc[2]);
            st_opt<PUB>(part + PART_UPD_XN2 * P.part_stride + w, acc[3]);
        }
    }
    stamp();  // 2K + 5: step
    if constexpr (STAMP)
        for (int k = tid; k < BAND_STAMPS + BAND_FSTAMPS; k += TPB)
            tl[k] = k < ts || k >= BAND_STAMPS - 1 ? stl[k] : 0ull;
}

template <int BC, bool STAMP>
__global__ __launch_bounds__(BAND_TPB) void k_bcr_band(const LmState* __restrict__ st, DevProblem P,
                                                       const double* __restrict__ S, double* __restrict__ rhs,
                                                       int* __restrict__ flag, BaConsts c,
                                                       const double* __restrict__ scale,
                                                       const double* __restrict__ camdata,
                                                       const double* __restrict__ lin, double* __restrict__ delta,
                                                       double* __restrict__ part, int nb,
                                                       unsigned long long* __restrict__ tl) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    band_body<BC, STAMP>(st, P, S, rhs, flag, c, scale, camdata, lin, delta, part, nb, tl, lds);
}

// ---- the band solve's tail in the same launch (DevWork::tail) -------------------------------------------------
// Workgroup 0 runs the band solve; workgroups 1..nb_bs the point back-substitution chunks (backsub_body), each
// waiting for the solve's launch number in tail_flags[0]; the last one the final reduction and LM decision
// (final_body), waiting until tail_flags[1] counts every chunk of this launch. The chunks zero S's envelope tiles
// only after the solve has read them. Two launches and their dependent-launch latency less per LM iteration, and
// the chunks' prologue overlaps the solve. Every workgroup is resident at once (band_tail_blocks bounds the grid),
// waits are bounded (a timeout raises FLAG_TIMEOUT: the decision then asks the host to re-run the iteration with
// the separate launches). Roles past the solve use waves 0-3 (the bodies are written for 256 threads).
__device__ unsigned g_tail_spin_limit = 1u << 20;

__device__ __forceinline__ bool tail_wait(const unsigned* w, unsigned target, unsigned lim) {
    for (unsigned n = 0;; ++n) {  // relaxed: the payload is read past the L2 (PUB bodies), no invalidate needed
        if (__hip_atomic_load(const_cast<unsigned*>(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target)
            return true;
        if (n >= lim) return false;
        __builtin_amdgcn_s_sleep(2);
    }
}

// Three hand-off words per launch (numbered by seq): tflags[0] = y published (the solve, before its camera step),
// tflags[1] = back-substitution chunks done (counted), tflags[2] = the camera step's candidates and partials
// published (the decision reads the partials).
// STAMP (MIBA_BCR_STAMPS=1): the band solve's phase stamps in tl[0..BAND_STAMPS + BAND_FSTAMPS), then per workgroup b
// s_memrealtime marks at tl[TAIL_ST0 + 16 b + k]: 0 start, 1 prologue done (chunks: backsub_pre; solve: step done),
// 2 wait done, 3 body done (before the count / the flag), 4 exit
static constexpr int TAIL_ST0 = 128;
template <int BC, bool O32, bool STAMP = false>
__global__ __launch_bounds__(BAND_TPB) void k_band_tail(const LmState* __restrict__ st_c, DevProblem P, BaConsts c,
                                                        LmParams prm, double* __restrict__ S, double* __restrict__ rhs,
                                                        int* __restrict__ flag, const double* __restrict__ scale,
                                                        const double* __restrict__ camdata,
                                                        const double* __restrict__ lin, double* __restrict__ delta,
                                                        double* __restrict__ part, int nb, const double* __restrict__ pdata,
                                                        const int2* __restrict__ ztiles, int n_ztiles, int nb_bs,
                                                        int nb_pt, int nb_upd, double* __restrict__ scal,
                                                        double* __restrict__ log, unsigned* __restrict__ tflags,
                                                        unsigned seq, unsigned long long* __restrict__ tl,
                                                        double* __restrict__ tail_y) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    __shared__ int ok_s;
    LmState* const st = const_cast<LmState*>(st_c);
    const int b = blockIdx.x, tid = threadIdx.x;
    unsigned long long tst[5] = {0, 0, 0, 0, 0};
    auto mark = [&](int k) {
        if constexpr (STAMP) if (tid == 0) tst[k] = realtime_now();
    };
    auto flush_marks = [&]() {
        if constexpr (STAMP) if (tid == 0) for (int k = 0; k < 5; ++k) tl[TAIL_ST0 + 16 * b + k] = tst[k];
    };
    mark(0);
    // y of this launch in buffer (seq & 1) of tail_y; the other one (this launch's successor's) is emptied by the solve
    double* const ybuf = tail_y + (size_t)(seq & 1u) * P.npad;
    if (b == 0) {
        {  // the next launch's y buffer: read by the previous launch's chunks, which have all finished
            double* const ynext = tail_y + (size_t)((seq + 1u) & 1u) * P.npad;
            for (int d = tid; d < P.npad; d += BAND_TPB) tail_st(ynext + d, __longlong_as_double((long long)BCR_Y_EMPTY));
        }
        // y, the candidate cameras and intrinsics, the step and the partials are stored past the L2 (PUB) and
        // drained by every thread before the count: no L2 write-back fence on the critical path (the consumers
        // read them with agent-scope loads)
        band_body<BC, STAMP, true>(st, P, S, rhs, flag, c, scale, camdata, lin, delta, part, nb, tl, lds, tflags, seq,
                                   ybuf);
        mark(1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        mark(3);
        if (tid == 0) __hip_atomic_store(tflags + 2, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        mark(4);
        flush_marks();
        return;
    }
    if (tid >= 256) return;  // (the back-substitution and final bodies are written for 256 threads)
    const bool skip = skip_step(st);
    // a back-substitution chunk loads its records and point data and evaluates its y-free products before it waits
    BsPre<O32> pre;
    BsPreLds* const pl = reinterpret_cast<BsPreLds*>(reinterpret_cast<char*>(lds) + sizeof(BsLds));
    double* const CL = reinterpret_cast<double*>(reinterpret_cast<char*>(lds) + sizeof(BsLds) + sizeof(BsPreLds));
    if (b <= nb_bs) {
        backsub_pre<O32>(P, c, st, scale, pdata, b - 1, *pl, pre);
        cand_prefetch<O32>(P, st, scale, CL);
    }
    mark(1);
    // A wait past the spin bound marks the iteration for a re-run (FLAG_TIMEOUT) and then still waits for its
    // producer (which waits on nothing and runs ahead of its consumers in dispatch order) before this workgroup
    // touches S or rhs, which the re-run assembles onto
    constexpr unsigned BOUND = 1u << 26;
    if (b <= nb_bs) {
        // y polled straight from its hand-off buffer into this chunk's LDS (flag-free: every value is the solve's f64
        // arithmetic, an unwritten one BCR_Y_EMPTY) — one store-to-load hop instead of the flag's and then y's
        double* const yl = CL + cand_lds_doubles(P.n_cams, P.nac);
        bool yok = true;
        if (!skip)
            for (int d = tid; d < P.kb + 4; d += 256) {
                const unsigned long long* q = reinterpret_cast<const unsigned long long*>(ybuf + d);
                unsigned long long u = 0;
                for (unsigned n = 0;; ++n) {
                    u = __hip_atomic_load(const_cast<unsigned long long*>(q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (u != BCR_Y_EMPTY) break;
                    if (n >= g_tail_spin_limit) { yok = false; break; }
                    __builtin_amdgcn_s_sleep(1);
                }
                if (!yok) break;
                yl[d] = __longlong_as_double((long long)u);
            }
        if (tid == 0) ok_s = 1;
        __syncthreads();
        if (!yok) ok_s = 0;
        __syncthreads();
        if (!ok_s && tid == 0) {
            raise_flag(flag, FLAG_TIMEOUT);
            (void)tail_wait(tflags, seq, BOUND);  // (the solve's y flag: it has run before S or rhs is touched)
        }
        mark(2);
        if (ok_s) {
            backsub_body<O32, true, true, true>(P, c, st, scale, pdata, yl, delta, part, ztiles, n_ztiles, S, b - 1,
                                                nb_bs, *reinterpret_cast<BsLds*>(lds), pre, pl, CL,
                                                STAMP ? tl + TAIL_ST0 + 16 * b + 8 : nullptr);
        } else if (tid == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the flag) drained before the count
        }
        mark(3);
        // thread 0 stored and drained this chunk's partials (PUB): count the chunk, no fence
        if (tid == 0) __hip_atomic_fetch_add(tflags + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // then this chunk's share of S's envelope tiles for the next iteration's assembly (the solve has read S;
        // the next launch sees the stores)
        if (!skip)
            for (int t = (b - 1) * n_ztiles / nb_bs; t < b * n_ztiles / nb_bs; ++t) {
                const int2 ij = ztiles[t];
                S[(size_t)(16 * ij.x + (tid >> 4)) * P.npad + 16 * ij.y + (tid & 15)] = 0.0;
            }
        mark(4);
        flush_marks();
        return;
    }
    // the final workgroup: the solve's camera step is published; the chunks' partials are polled in final_body
    // (POLL: flag-free slots, no count on this path)
    if (tid == 0) {
        ok_s = (skip || tail_wait(tflags + 2, seq, g_tail_spin_limit)) ? 1 : 0;
        if (!ok_s) {
            raise_flag(flag, FLAG_TIMEOUT);
            (void)tail_wait(tflags + 1, seq * (unsigned)nb_bs, BOUND);  // every chunk done before rhs is zeroed
            (void)tail_wait(tflags + 2, seq, BOUND);
        }
    }
    __syncthreads();
    mark(2);
    final_body<2, true, true>(P, st, nb_pt, nb_upd, nb_bs, part, flag, scal, prm, lin, log, rhs, nullptr,
                              *reinterpret_cast<FinLds*>(lds), STAMP ? tl + TAIL_ST0 + 16 * b + 5 : nullptr,
                              TailPoll{ok_s ? g_tail_spin_limit : 0u, tflags + 1, seq * (unsigned)nb_bs});
    mark(3);
    flush_marks();
}

// ---- the back-substitution and the decision in one launch (C4-size windows: DevWork::bsfin) ----------------------
// k_backsub_chunk's chunks as workgroups 0..nb_bs-1 and k_final's reduction + LM decision as workgroup nb_bs, which is
// dispatched last and waits until tail_flags[1] counts every chunk of this launch (the chunks wait on nothing, so the
// wait always ends). The chunks read y and the candidates from the previous launch with plain loads and store only
// their partials past the L2, drained before the count (backsub_body<O32, false, true>); the decision workgroup
// reads them with agent-scope loads (final_body<2, true>). One launch less per LM iteration, and the reduction starts
// the moment the last chunk has counted. A wait past the spin bound raises FLAG_TIMEOUT (the iteration is re-run
// with the separate launches) after waiting for the chunks, as the band tail does.
template <bool O32>
__global__ __launch_bounds__(TPB) void k_backsub_final(DevProblem P, BaConsts c, LmState* __restrict__ st,
                                                       const double* __restrict__ scale,
                                                       const double* __restrict__ pdata, double* __restrict__ rhs,
                                                       double* __restrict__ part, const int2* __restrict__ ztiles,
                                                       int n_ztiles, double* __restrict__ S, int nb_bs, int nb_pt,
                                                       int nb_upd, int* __restrict__ flag, double* __restrict__ scal,
                                                       LmParams prm, const double* __restrict__ lin,
                                                       double* __restrict__ log, unsigned* __restrict__ bcr_epoch,
                                                       unsigned* __restrict__ tflags, unsigned seq) {
    __shared__ union {
        BsLds bs;
        FinLds fin;
    } L;
    __shared__ int ok_s;
    const int b = blockIdx.x, tid = threadIdx.x;
    // (the decision role tested first, on b == nb_bs: written the other way round the compiler gave the kernel 134
    // VGPRs instead of the chunks' 126, 3 waves per SIMD instead of 4)
    if (b == nb_bs) {
        constexpr unsigned BOUND = 1u << 26;
        if (tid == 0) {
            const bool skip = skip_step(st);
            ok_s = (skip || tail_wait(tflags + 1, seq * (unsigned)nb_bs, g_tail_spin_limit)) ? 1 : 0;
            if (!ok_s) {
                raise_flag(flag, FLAG_TIMEOUT);
                (void)tail_wait(tflags + 1, seq * (unsigned)nb_bs, BOUND);  // every chunk done before rhs is zeroed
            }
        }
        __syncthreads();
        final_body<2, true>(P, st, nb_pt, nb_upd, nb_bs, part, flag, scal, prm, lin, log, rhs, bcr_epoch, L.fin);
        return;
    }
    backsub_body<O32, false, true>(P, c, st, scale, pdata, rhs, nullptr, part, ztiles, n_ztiles, S, b, nb_bs, L.bs);
    // thread 0 stored and drained this chunk's partials (or the chunk skipped: nothing to publish)
    if (tid == 0) __hip_atomic_fetch_add(tflags + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

hipError_t launch_backsub_final(const DevProblem& P, const BaConsts& c, const LmParams& prm, DevWork& W, int nb_pt,
                                int nb_upd, unsigned* bcr_epoch, hipStream_t s, Prof* pf) {
    const int nb_bs = P.n_bs_chunks;
    ++W.tail_seq;
    if (pf) pf->begin(K_BACKSUB_EVAL, s);
    if (P.obs32)
        hipLaunchKernelGGL(k_backsub_final<true>, dim3(nb_bs + 1), dim3(TPB), 0, s, P, c, W.st, W.scale, W.pdata, W.rhs,
                           W.part, W.env_tile, W.n_env, W.S, nb_bs, nb_pt, nb_upd, W.chol_flag, W.scal, prm, W.lin, W.log,
                           bcr_epoch, W.tail_flags, W.tail_seq);
    else
        hipLaunchKernelGGL(k_backsub_final<false>, dim3(nb_bs + 1), dim3(TPB), 0, s, P, c, W.st, W.scale, W.pdata, W.rhs,
                           W.part, W.env_tile, W.n_env, W.S, nb_bs, nb_pt, nb_upd, W.chol_flag, W.scal, prm, W.lin, W.log,
                           bcr_epoch, W.tail_flags, W.tail_seq);
    if (pf) pf->end(s);
    return hipGetLastError();
}

static size_t band_lds_bytes(int bc, int nb, int nac) { return sizeof(double) * (size_t)band_layout(6 * bc, nb, nac).total; }

// The band path for this window: cameras per block (1..3), 0 when it does not apply. mode: MIBA_BCR_BAND
// (0 off, 2 also for one-block windows, else the default: windows of more than one 64-dof BCR block).
int bcr_band_ok(int nac, int cam_band, int kb, bool one_block) {
    if (nac < 2 || cam_band > 3 || std::getenv("MIBA_BCR")) return 0;
    const char* e = std::getenv("MIBA_BCR_BAND");
    const int mode = e ? std::atoi(e) : 1;
    if (mode == 0) return 0;
    // one BCR block: k_bcr_dense1, unless the band solve's tail launch will run (C1: 46.8-47.8 us per LM iteration
    // against 48.0-48.9 with k_bcr_dense1, same box) or MIBA_BCR_BAND=2
    if (mode != 2 && !one_block && nac <= BCR_CAMS && kb + 4 <= 64) return 0;
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
    static DeviceOnce attr;
    static DeviceScratch stamp_buf;
    static const int smode = env_on("MIBA_BCR_STAMPS");
    CKD(attr([] {
        CKD(hipFuncSetAttribute((const void*)k_bcr_band<BC, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024));
        return hipFuncSetAttribute((const void*)k_bcr_band<BC, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024);
    }));
    const size_t lds = band_lds_bytes(BC, nb, P.nac);
    if (smode) {
        unsigned long long* dst = stamp_buf.get<unsigned long long>((BAND_STAMPS + BAND_FSTAMPS) * sizeof(unsigned long long));
        if (!dst) return hipErrorOutOfMemory;
        CKD(hipMemsetAsync(dst, 0, (BAND_STAMPS + BAND_FSTAMPS) * sizeof(unsigned long long), s));
        if (pf) pf->begin(K_BCR_PERSIST, s);
        hipLaunchKernelGGL((k_bcr_band<BC, true>), dim3(1), dim3(BAND_TPB), lds, s, W.st, P, W.S, W.rhs, W.chol_flag, c,
                           W.scale, W.camdata, W.lin, W.delta, W.part, nb, dst);
        if (pf) pf->end(s);
        CKD(hipGetLastError());
        unsigned long long h[BAND_STAMPS + BAND_FSTAMPS];
        CKD(hipMemcpyAsync(h, dst, sizeof(h), hipMemcpyDeviceToHost, s));
        CKD(hipStreamSynchronize(s));
        if (h[0]) {  // (0: the launch exited at once, skip_step)
            int K = 0;
            while ((2 << K) <= nb) ++K;
            std::fprintf(stderr, "bcr_band<%d> nb=%d us:", BC, nb);
            const unsigned long long t0 = h[BAND_STAMPS - 1];
            double prev = 0.0;
            for (int k = 0; k < BAND_STAMPS - 1 && h[k]; ++k) {
                const double t = (double)(h[k] - t0) / 100.0;
                std::fprintf(stderr, " %.2f", t - prev);
                prev = t;
            }
            std::fprintf(stderr, "  = %.2f us (phase durations: load, [factor, update] x levels 0..%d (the root: factor "
                                 "only), border, back, step)\n", prev, K);
            for (int m = 0; m <= K && m < 8; ++m) {  // inside the factor phase: wave 0's first unit
                const unsigned long long* f = h + BAND_STAMPS + 8 * m;
                std::fprintf(stderr, "  level %d factor unit: D rows %.2f chain %.2f L stored %.2f cols loaded %.2f solve %.2f "
                                     "stored %.2f us\n", m, (f[1] - f[0]) / 100.0, (f[2] - f[1]) / 100.0, (f[3] - f[2]) / 100.0,
                             (f[4] - f[3]) / 100.0, (f[5] - f[4]) / 100.0, (f[6] - f[5]) / 100.0);
            }
        }
        return hipSuccess;
    }
    if (pf) pf->begin(K_BCR_PERSIST, s);
    hipLaunchKernelGGL((k_bcr_band<BC, false>), dim3(1), dim3(BAND_TPB), lds, s, W.st, P, W.S, W.rhs, W.chol_flag, c,
                       W.scale, W.camdata, W.lin, W.delta, W.part, nb, (unsigned long long*)nullptr);
    if (pf) pf->end(s);
    return hipGetLastError();
}

// the chunks' and the decision's dynamic LDS: BsLds | BsPreLds | the candidate table (cand_lds_doubles) | y; FinLds
static size_t tail_role_lds(const DevProblem& P) {
    return std::max(sizeof(BsLds) + sizeof(BsPreLds) + sizeof(double) * (cand_lds_doubles(P.n_cams, P.nac) + P.kb + 4),
                    sizeof(FinLds));
}

int band_tail_blocks(const DevProblem& P, int bc) {
    if (bc < 1 || bc > 3) return 0;
    const int n = P.n_bs_chunks + 2;
    const size_t lds = std::max(band_lds_bytes(bc, (P.nac + bc - 1) / bc, P.nac), tail_role_lds(P));
    // one resident round with room to spare (>= 256 CUs), the dynamic LDS beside the launch's static word
    return (P.n_ap > 0 && n <= 128 && lds <= 160 * 1024 - 256) ? n : 0;
}

hipError_t tail_set_spin_limit(unsigned limit) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_tail_spin_limit), &limit, sizeof(limit));
}

template <int BC, bool O32>
static hipError_t launch_tail_t(const DevProblem& P, const BaConsts& c, const LmParams& prm, DevWork& W, int nb,
                                int nb_pt, int nb_upd, hipStream_t s, Prof* pf) {
    static DeviceOnce attr;
    static DeviceScratch stamp_buf;
    static const int smode = env_on("MIBA_BCR_STAMPS");
    CKD(attr([] {
        CKD(hipFuncSetAttribute((const void*)k_band_tail<BC, O32, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                160 * 1024 - 256));
        return hipFuncSetAttribute((const void*)k_band_tail<BC, O32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024 - 256);
    }));
    const size_t lds = std::max(band_lds_bytes(BC, nb, P.nac), tail_role_lds(P));
    const int nb_bs = P.n_bs_chunks;
    ++W.tail_seq;
    if (smode) {  // diagnostic: the band solve's phases and every tail workgroup's marks (MIBA_BCR_STAMPS=1)
        const size_t nst = TAIL_ST0 + 16 * (size_t)(nb_bs + 2);
        unsigned long long* dst = stamp_buf.get<unsigned long long>(nst * sizeof(unsigned long long));
        if (!dst) return hipErrorOutOfMemory;
        CKD(hipMemsetAsync(dst, 0, nst * sizeof(unsigned long long), s));
        hipLaunchKernelGGL((k_band_tail<BC, O32, true>), dim3(nb_bs + 2), dim3(BAND_TPB), lds, s, W.st, P, c, prm, W.S,
                           W.rhs, W.chol_flag, W.scale, W.camdata, W.lin, W.delta, W.part, nb, W.pdata, W.env_tile,
                           W.fused ? W.n_env : 0, nb_bs, nb_pt, nb_upd, W.scal, W.log, W.tail_flags, W.tail_seq, dst, W.tail_y);
        CKD(hipGetLastError());
        std::vector<unsigned long long> h(nst);
        CKD(hipMemcpyAsync(h.data(), dst, nst * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        CKD(hipStreamSynchronize(s));
        const unsigned long long* tw = h.data() + TAIL_ST0;
        if (tw[0] && h[0]) {
            const unsigned long long t0 = tw[0];  // the solve workgroup's start
            auto us = [&](unsigned long long t) { return t ? (double)((long long)(t - t0)) / 100.0 : -1.0; };
            std::fprintf(stderr, "band_tail<%d> nb=%d chunks=%d | solve wg: start 0 solved %.2f flag %.2f | solve phases:",
                         BC, nb, nb_bs, us(tw[1]), us(tw[4]));
            const unsigned long long bt0 = h[BAND_STAMPS - 1];
            double prev = (double)((long long)(bt0 - t0)) / 100.0;
            for (int k = 0; k < BAND_STAMPS - 1 && h[k]; ++k) {
                const double t = (double)((long long)(h[k] - t0)) / 100.0;
                std::fprintf(stderr, " %.2f", t - prev);
                prev = t;
            }
            std::fprintf(stderr, "\n");
            double mx[5] = {0, 0, 0, 0, 0}, mn[5] = {1e30, 1e30, 1e30, 1e30, 1e30};
            for (int b = 1; b <= nb_bs; ++b)
                for (int k = 0; k < 5; ++k) {
                    const double v = us(tw[16 * b + k]);
                    mx[k] = std::max(mx[k], v);
                    mn[k] = std::min(mn[k], v);
                }
            std::fprintf(stderr, "  chunks (min..max us): start %.2f..%.2f pre %.2f..%.2f waited %.2f..%.2f body %.2f..%.2f "
                                 "exit %.2f..%.2f\n", mn[0], mx[0], mn[1], mx[1], mn[2], mx[2], mn[3], mx[3], mn[4], mx[4]);
            {  // inside the body of the chunk that finished last: phase 1 (+ candidates), 2, 3, reduced, drained
                int bl = 1;
                for (int b = 1; b <= nb_bs; ++b) if (tw[16 * b + 3] > tw[16 * bl + 3]) bl = b;
                const unsigned long long* q = tw + 16 * bl + 8;
                std::fprintf(stderr, "  last chunk %d: waited %.2f phase1 %.2f phase2 %.2f phase3 %.2f reduced %.2f drained %.2f\n",
                             bl - 1, us(tw[16 * bl + 2]), us(q[0]), us(q[1]), us(q[2]), us(q[3]), us(q[4]));
            }
            const unsigned long long* f = tw + 16 * (nb_bs + 1);
            std::fprintf(stderr, "  final: start %.2f waited %.2f | loads in %.2f reduced %.2f decided %.2f | exit %.2f\n",
                         us(f[0]), us(f[2]), us(f[5]), us(f[6]), us(f[7]), us(f[3]));
        }
        return hipSuccess;
    }
    if (pf) pf->begin(K_BCR_PERSIST, s);
    hipLaunchKernelGGL((k_band_tail<BC, O32>), dim3(nb_bs + 2), dim3(BAND_TPB), lds, s, W.st, P, c, prm, W.S, W.rhs,
                       W.chol_flag, W.scale, W.camdata, W.lin, W.delta, W.part, nb, W.pdata, W.env_tile,
                       W.fused ? W.n_env : 0, nb_bs, nb_pt, nb_upd, W.scal, W.log, W.tail_flags, W.tail_seq,
                       (unsigned long long*)nullptr, W.tail_y);
    if (pf) pf->end(s);
    return hipGetLastError();
}

hipError_t launch_band_tail(const DevProblem& P, const BaConsts& c, const LmParams& prm, DevWork& W, int bc, int nb_pt,
                            int nb_upd, hipStream_t s, Prof* pf) {
    const int nb = (P.nac + bc - 1) / bc;
    switch (bc * 2 + (P.obs32 ? 1 : 0)) {
        case 2: return launch_tail_t<1, false>(P, c, prm, W, nb, nb_pt, nb_upd, s, pf);
        case 3: return launch_tail_t<1, true>(P, c, prm, W, nb, nb_pt, nb_upd, s, pf);
        case 4: return launch_tail_t<2, false>(P, c, prm, W, nb, nb_pt, nb_upd, s, pf);
        case 5: return launch_tail_t<2, true>(P, c, prm, W, nb, nb_pt, nb_upd, s, pf);
        case 6: return launch_tail_t<3, false>(P, c, prm, W, nb, nb_pt, nb_upd, s, pf);
        case 7: return launch_tail_t<3, true>(P, c, prm, W, nb, nb_pt, nb_upd, s, pf);
        default: return hipErrorInvalidValue;
    }
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
