// ba_kernels.hip — libmiba HIP kernels for gfx950 (MI355X / CDNA4), f64 throughout.
//
// One LM iteration of the reference's ceres::Solve (OptimizationUtils.cpp:300;
// LM + SPARSE_SCHUR, BundleAdjustmentConfig.h:61-67) is, on the device:
//
//   k_cam_side      camera-major pass: per sub-segment  U=Jc^T Jc, C=Jc^T Jk, g=Jc^T f
//                   (+ intrinsics JkJk, Jk^T f, cost)  [only after an accepted step]
//   k_point_prep    point-major pass: per point V, e, K (scaled, LM-damped), V^-1, intrinsics
//                   Schur partials; extra workgroups assemble the envelope of S (camera blocks
//                   U + D^2, border C, Ukk, rhs) and finish the camera-side sums  [every iteration]
//   k_schur_tile    S -= W V^-1 W^T, rhs -= W V^-1 e on f64 MFMA (+ one workgroup: S_kk terms)
//   k_obs_pairs     the same for overflow points (global f64 atomics)
//   k_bcr_split     reduced camera system (ba_bcr.hip) + border solve + camera step;
//                   k_chol_band / k_chol + k_update_cams for short or wide windows
//   k_backsub_chunk point back-substitution, point model-change terms 0.5(e~^T y + y^T D~ y),
//                   candidate cost at x + delta
//   k_final         deterministic reduction of the per-block partials + the LM decision
// (k_cam_finalize / k_lin_finalize: iteration 0 and landmark-sharded windows)
//
// The residual/Jacobian is never stored: it is recomputed from the 32-byte
// observation record + the resident pose/point (cheaper than 304 B/obs of
// stored Jacobian blocks; DESIGN.md "Roofline").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <cstdlib>

#include "ba_common.h"
#include "ba_device.h"
#include "ba_kernels.h"
#include "ba_tail.h"

namespace miba {

// ---------------------------------------------------------------- camera side
// XCD-aware sub-segment order: workgroup b of a launch runs on XCD b % 8 (dispatch round-robin; a placement
// assumption for speed only, never for correctness). The camera-side workgroups [first, first + n) take the
// sub-segments (camera-major order) so that each XCD gets one contiguous eighth of the cameras: the points a
// camera band gathers are then cached in ONE XCD's L2 (a point is gathered by its ~10 co-visible cameras),
// instead of every XCD fetching every point. A bijection on [0, n); each segment's partial keeps its own slot.
__device__ __forceinline__ int xcd_seg(int b, int first, int n) {
    const int x = b & 7, j = b - first;
    int pre = 0;
#pragma unroll
    for (int y = 0; y < 8; ++y) {
        const int j0 = (y - first) & 7;
        const int cnt = j0 < n ? (n - j0 + 7) >> 3 : 0;
        pre += y < x ? cnt : 0;
    }
    return pre + ((j - ((x - first) & 7)) >> 3);
}

// One workgroup per sub-segment (<= SUBSEG_OBS observations of one camera) of the
// camera-major observation list; k_cam_finalize sums a camera's sub-segments in order.
// camdata (per sub-segment partial here): U upper-packed (21), C (6x4 = 24), g (6)
// seg_intr[s*SEGINTR + ..]: Ukk upper-packed (10), gk (4), cost (1)
template <bool O32>
__device__ __forceinline__ void cam_side_block(const DevProblem& P, const BaConsts& c, const LmState* __restrict__ st,
                                               int gated, double* __restrict__ camdata, double* __restrict__ seg_intr,
                                               double* __restrict__ gmax_word, const int s, bool pub = false) {
    // lin[1] is max-accumulated by the envelope tiles / k_cam_finalize (read only after a linearisation):
    // clear it here, one kernel boundary ahead, whether or not this iteration linearises
    // (pub: the small-window launch's envelope tiles read the outputs in the same launch, past the L2; stores
    // likewise, drained by the caller)
    if (s == 0 && threadIdx.x == 0) {
        if (pub) tail_st(gmax_word, 0.0); else *gmax_word = 0.0;
    }
    if (st->done || (gated && !st->need_lin)) return;
    const int cur = st->cur;
    __shared__ double lds[4 * CAM_NZ];
    __shared__ double out[CAM_NZ];
    const int cam = P.seg_cam[s];
    const int ac = P.seg_ac[s];
    const double* pose = P.cams[cur] + 7 * cam;
    const double* pts = P.pts[cur];
    const double* K = P.K[cur];
    // packed sums without the structural zeros of the Jacobian (cam_accum, ba_device.h)
    double acc[CAM_NZ];
#pragma unroll
    for (int i = 0; i < CAM_NZ; ++i) acc[i] = 0.0;
    const int o0 = P.seg_ptr[s], o1 = P.seg_ptr[s + 1];
    // software pipeline: observation record (point index, pixel, depth) two observations ahead, point one ahead
    const int oa = o0 + threadIdx.x;
    ObsRaw<O32> r_n = oa < o1 ? co_obs<O32>(P, oa) : obs_zero<O32>();
    ObsRaw<O32> r_nn = oa + TPB < o1 ? co_obs<O32>(P, oa + TPB) : obs_zero<O32>();
    double X_n[3] = {0.0, 0.0, 0.0};
    if (oa < o1) {
#pragma unroll
        for (int k = 0; k < 3; ++k) X_n[k] = pts[3 * r_n.idx() + k];
    }
    for (int o = oa; o < o1; o += TPB) {
        const double X[3] = {X_n[0], X_n[1], X_n[2]};
        const ObsRaw<O32> r = r_n;
        const int on = o + TPB;
        if (on < o1) {
            r_n = r_nn;
#pragma unroll
            for (int k = 0; k < 3; ++k) X_n[k] = pts[3 * r_n.idx() + k];
            r_nn = on + TPB < o1 ? co_obs<O32>(P, on + TPB) : obs_zero<O32>();
        }
        ObsEval e;
        double jc[18], jp[9], jk[8];
        lin_obs(c, pose, X, K, r.u(), r.v(), r.d(), e, jc, jp, jk);
        (void)jp;
        cam_accum(acc, jc, jk, e.f, e.ok ? e.cost : __builtin_nan(""), ac >= 0);
    }
    block_sum_rs<CAM_NZ>(acc, lds, out);
    if (ac >= 0)
        for (int i = threadIdx.x; i < CAMDATA; i += TPB) {
            double* q = camdata + (size_t)s * CAMDATA + i;
            if (pub) tail_st(q, cam_unpack(out, i)); else *q = cam_unpack(out, i);
        }
    for (int i = threadIdx.x; i < SEGINTR; i += TPB) {
        double* q = seg_intr + (size_t)s * SEGINTR + i;
        if (pub) tail_st(q, cam_unpack(out, CAMDATA + i)); else *q = cam_unpack(out, CAMDATA + i);
    }
}
template <bool O32>
__global__ __launch_bounds__(TPB) void k_cam_side(DevProblem P, BaConsts c, const LmState* __restrict__ st, int gated,
                                                  double* __restrict__ camdata, double* __restrict__ seg_intr,
                                                  double* __restrict__ gmax_word) {
    cam_side_block<O32>(P, c, st, gated, camdata, seg_intr, gmax_word, P.xcd_map ? xcd_seg(blockIdx.x, 0, P.n_seg) : (int)blockIdx.x);
}

// One launch for what follows the camera-side pass (was k_cam_reduce + k_lin_finalize):
//   workgroup ac < nac: camdata[ac] = sum of the camera's sub-segment partials, in sub-segment order
//     (zero when this landmark shard has no observation of the camera); mode 0 also takes the camera's
//     share of the gradient max-norm ||x - Plus(x, -g)||_inf and max-accumulates it into lin[1]
//     (non-negative doubles order like their bit patterns; k_cam_side cleared the word);
//   workgroup nac: the intrinsics partials, in a fixed order. mode 0: k_lin_finalize's mode-0 body
//     without the camera loop (lin[0], lin[2..16), intrinsics gradient max into lin[1]); mode 1
//     (sharded, before the all-reduce): the sums go to linpart, k_lin_finalize mode 2 finishes.
__global__ __launch_bounds__(TPB) void k_cam_finalize(DevProblem P, BaConsts c, const LmState* __restrict__ st,
                                                      int gated, const double* __restrict__ cpart,
                                                      double* __restrict__ camdata, const double* __restrict__ seg_intr,
                                                      double* __restrict__ lin, int mode, double* __restrict__ linpart) {
    if (st->done || (gated && !st->need_lin)) return;
    __shared__ double lds[4 * SEGINTR];
    __shared__ double out[SEGINTR];
    __shared__ double g6[6];
    const int cur = st->cur;
    const int b = blockIdx.x, tid = threadIdx.x;
    if (b < P.nac) {
        if (tid < CAMDATA) {
            const int2 r = P.ac_seg[b];
            double v = 0.0;
            for (int sg = r.x; sg < r.y; ++sg) v += cpart[(size_t)sg * CAMDATA + tid];
            camdata[(size_t)b * CAMDATA + tid] = v;
            if (tid >= 45) g6[tid - 45] = v;
        }
        if (mode != 0) return;
        __syncthreads();
        if (tid == 0) {
            const double* x = P.cams[cur] + 7 * P.ac_cam[b];
            double ng[6], tp[7];
#pragma unroll
            for (int d = 0; d < 6; ++d) ng[d] = -g6[d];
            se3_plus(x, ng, tp);
            double gm = 0.0;
#pragma unroll
            for (int j = 0; j < 7; ++j) gm = fmax(gm, fabs(x[j] - tp[j]));
            atomicMax((unsigned long long*)(lin + 1), (unsigned long long)__double_as_longlong(gm));
        }
        return;
    }
    double acc[SEGINTR];
#pragma unroll
    for (int i = 0; i < SEGINTR; ++i) acc[i] = 0.0;
    for (int sg = tid; sg < P.n_seg; sg += TPB)
#pragma unroll
        for (int i = 0; i < SEGINTR; ++i) acc[i] += seg_intr[(size_t)sg * SEGINTR + i];
    block_sum<SEGINTR>(acc, lds, out);
    if (mode == 1) {
        if (tid < SEGINTR) linpart[tid] = out[tid];
        return;
    }
    if (tid == 0) {
        const double* K = P.K[cur];
        double pc = 0.0, gm = 0.0;
        double gk[4];
        for (int m = 0; m < 4; ++m) {
            const double fk = c.sw_k * (P.prior[m] - K[m]);
            pc += fk * fk;
            gk[m] = out[10 + m] + (-c.sw_k) * fk;
            gm = fmax(gm, fabs(K[m] - (K[m] + -gk[m])));
        }
        lin[0] = out[14] + 0.5 * pc;
        atomicMax((unsigned long long*)(lin + 1), (unsigned long long)__double_as_longlong(gm));
        for (int q = 0; q < 10; ++q) lin[2 + q] = out[q];
        int q = 0;
        for (int m = 0; m < 4; ++m)
            for (int l = m; l < 4; ++l, ++q)
                if (l == m) lin[2 + q] += c.sw_k * c.sw_k;
        for (int m = 0; m < 4; ++m) lin[12 + m] = gk[m];
    }
}

// Reduce intrinsics partials (fixed order), add the IntrinsicsPrior block
// (OptimizationUtils.cpp:117-125, squared loss), compute the gradient max-norm of
// cameras + intrinsics: ||x - Plus(x, -g)||_inf (Ceres 2.0 trust_region_minimizer).
// lin[0] = cost(x), lin[1] = gmax(cams, intr), lin[2..12) = Ukk packed, lin[12..16) = gk
// mode 0: unsharded. mode 1 (sharded, before the all-reduce): only the fixed-order sum of
// this rank's segment partials -> linpart[0..SEGINTR). mode 2 (after the all-reduce): the
// summed partials are read from linpart and the rest runs as in mode 0.
__global__ __launch_bounds__(TPB) void k_lin_finalize(DevProblem P, BaConsts c, const LmState* __restrict__ st, int gated,
                                                      const double* __restrict__ camdata,
                                                      const double* __restrict__ seg_intr, double* __restrict__ lin,
                                                      int mode, double* __restrict__ linpart) {
    if (st->done || (gated && !st->need_lin)) return;
    const int cur = st->cur;
    __shared__ double lds[4 * SEGINTR];
    __shared__ double out[SEGINTR];
    __shared__ double red[4];
    if (mode == 2) {
        if (threadIdx.x < SEGINTR) out[threadIdx.x] = linpart[threadIdx.x];
        __syncthreads();
    } else {
        double acc[SEGINTR];
#pragma unroll
        for (int i = 0; i < SEGINTR; ++i) acc[i] = 0.0;
        // fixed-order: each thread sums a strided subset; block_sum order is fixed too
        for (int s = threadIdx.x; s < P.n_seg; s += TPB)
#pragma unroll
            for (int i = 0; i < SEGINTR; ++i) acc[i] += seg_intr[(size_t)s * SEGINTR + i];
        block_sum<SEGINTR>(acc, lds, out);
        if (mode == 1) {
            if (threadIdx.x < SEGINTR) linpart[threadIdx.x] = out[threadIdx.x];
            return;
        }
    }
    const double* K = P.K[cur];
    double gm = 0.0;
    for (int ac = threadIdx.x; ac < P.nac; ac += TPB) {
        const int cam = P.ac_cam[ac];
        const double* x = P.cams[cur] + 7 * cam;
        double ng[6], tp[7];
#pragma unroll
        for (int d = 0; d < 6; ++d) ng[d] = -camdata[(size_t)ac * CAMDATA + 45 + d];
        se3_plus(x, ng, tp);
#pragma unroll
        for (int j = 0; j < 7; ++j) gm = fmax(gm, fabs(x[j] - tp[j]));
    }
    gm = block_max(gm, red);
    if (threadIdx.x == 0) {
        double pc = 0.0;
        double gk[4];
        for (int m = 0; m < 4; ++m) {
            const double fk = c.sw_k * (P.prior[m] - K[m]);
            pc += fk * fk;
            gk[m] = out[10 + m] + (-c.sw_k) * fk;
            gm = fmax(gm, fabs(K[m] - (K[m] + -gk[m])));
        }
        lin[0] = out[14] + 0.5 * pc;
        lin[1] = gm;
        for (int q = 0; q < 10; ++q) lin[2 + q] = out[q];
        // prior block: J = -sqrt(w) I adds w on the diagonal of Ukk
        int q = 0;
        for (int m = 0; m < 4; ++m)
            for (int l = m; l < 4; ++l, ++q)
                if (l == m) lin[2 + q] += c.sw_k * c.sw_k;
        for (int m = 0; m < 4; ++m) lin[12 + m] = gk[m];
    }
}

// mode 0: column norms only (iteration 0, before the Jacobi scale exists)
// mode 1: full Schur preparation.
// pdata[ap*PDATA]: G = chol(V~)^-1 packed (6), e~ (3), K~ (12, [m][i]), D~ (3)
// PP_LANES lanes per point: lane q of the group evaluates observations q, q + PP_LANES, ... of
// the point; the group's xor-shuffle sums leave identical totals in every lane, each lane then
// runs the (redundant) 3x3 factorisation and stores its share of the point's record.
template <int PP_LANES, int NV>
__device__ __forceinline__ void group_sum(double (&v)[NV]) {
#pragma unroll
    for (int off = 1; off < PP_LANES; off <<= 1)
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] += __shfl_xor(v[i], off);
}
// Camera ac's value v (of CAMDATA) summed over its sub-segment partials, in sub-segment order.
__device__ __forceinline__ double cam_sum(const DevProblem& P, const double* __restrict__ cpart, int ac, int v,
                                          bool pub = false) {
    const int2 r = P.ac_seg[ac];
    double acc = 0.0;
    for (int sg0 = r.x; sg0 < r.y; sg0 += 4) {  // 4 loads in flight, added in segment order
        double t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double* q = cpart + (size_t)(sg0 + k) * CAMDATA + v;
            t[k] = sg0 + k < r.y ? (pub ? tail_ld(q) : *q) : 0.0;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (sg0 + k < r.y) acc += t[k];
    }
    return acc;
}
// The intrinsics partials of all sub-segments in a fixed order (strided per thread, then block_sum).
__device__ void intr_sums(const DevProblem& P, const double* __restrict__ seg_intr, double* lds, double* out,
                          bool pub = false) {
    double acc[SEGINTR];
#pragma unroll
    for (int i = 0; i < SEGINTR; ++i) acc[i] = 0.0;
    for (int sg = threadIdx.x; sg < P.n_seg; sg += TPB)
#pragma unroll
        for (int i = 0; i < SEGINTR; ++i) {
            const double* q = seg_intr + (size_t)sg * SEGINTR + i;
            acc[i] += pub ? tail_ld(q) : *q;
        }
    block_sum<SEGINTR>(acc, lds, out);
}

// ---------------------------------------------------------------- envelope assembly
// One workgroup per envelope tile of S (16x16, one element per thread): every element is written once —
// the camera blocks s U s + D^2 (lower), the border s C s_k, the intrinsics block and the pad identity
// (rank 0; the landmark shards of other ranks contribute zeros), zero elsewhere — and the diagonal tiles
// write their 16 rows of rhs; resets the factorisation flag.
// fin (unsharded LM loop): the camera-side sums are finished here instead of in k_cam_finalize. Each
// tile sums the sub-segment partials of the (<= 4) cameras its elements need, in sub-segment order; the
// diagonal tile holding a camera's first dof stores camdata and max-accumulates the camera's gradient
// term into lin[1]; the intrinsics tiles sum the intrinsics partials and the diagonal one holding row kb
// stores lin. Same values every iteration until the next linearisation. With stop (the terminal
// stop_next iteration) only lin[0] / lin[1] are produced, for the decision.
__device__ void env_tile(const DevProblem& P, const BaConsts& c, const LmState* __restrict__ st, int t,
                         const int2* __restrict__ tiles, const double* __restrict__ camdata,
                         const double* __restrict__ lin, const double* __restrict__ scale, double* __restrict__ S,
                         double* __restrict__ rhs, int* __restrict__ chol_flag, int fin,
                         const double* __restrict__ cpart, const double* __restrict__ seg_intr, double* camdata_w,
                         double* lin_w, bool accumulate = false, bool pub = false) {
    __shared__ double cds[4 * CAMDATA];
    __shared__ double l16[LIN_N];
    __shared__ double ilds[4 * SEGINTR];
    __shared__ double io[SEGINTR];
    const int2 ij = tiles[t];
    const int tid = threadIdx.x;
    const int r = 16 * ij.x + (tid >> 4), col = 16 * ij.y + (tid & 15);
    const int nd = 6 * P.nac, kb = P.kb;
    const bool stop = st->stop_next;
    int ac0 = 0;
    const double* cd = camdata;  // camera values: row ac at cd + (ac - ac0) * CAMDATA
    const double* linr = lin;
    if (fin) {
        const int r0 = 16 * ij.x, c0 = 16 * ij.y;
        const bool diag = ij.x == ij.y;
        const bool brd = r0 + 15 >= kb && r0 < kb + 4;  // tile holds intrinsics rows
        // cameras this tile needs: of its rows (diagonal tiles: camera blocks + rhs), of its columns (border
        // rows), else of rows and columns both (a camera block straddling two tile rows)
        const int rlo = r0 / 6, rhi = r0 < nd ? min(r0 + 15, nd - 1) / 6 : -1;
        const int clo = c0 / 6, chi = c0 < nd ? min(c0 + 15, nd - 1) / 6 : -1;
        int lo = 0, hi = -1;
        if (diag) { lo = rlo; hi = rhi; }
        else if (brd) { lo = clo; hi = chi; }
        else { lo = max(rlo, clo); hi = min(rhi, chi); }
        if (hi < lo) { lo = 0; hi = -1; }
        const int ncam = hi - lo + 1;
        for (int e = tid; e < ncam * CAMDATA; e += TPB) cds[e] = cam_sum(P, cpart, lo + e / CAMDATA, e % CAMDATA, pub);
        const bool kk_any = brd && c0 + 15 >= kb && c0 < kb + 4;
        if (kk_any) intr_sums(P, seg_intr, ilds, io, pub);  // (barriers inside; uniform per tile)
        __syncthreads();
        const int cur = st->cur;
        if (diag) {  // cameras whose first dof lies in this tile's rows
            for (int e = tid; e < ncam * CAMDATA; e += TPB) {
                const int ac = lo + e / CAMDATA;
                if (6 * ac >= r0 && (fin == 2 || !stop)) camdata_w[(size_t)ac * CAMDATA + e % CAMDATA] = cds[e];
            }
            if (fin == 1 && tid < ncam && 6 * (lo + tid) >= r0)
                atomic_max_nonneg(lin_w + 1, cam_gmax(P, cur, lo + tid, cds + tid * CAMDATA + 45));
        }
        if (fin == 2 && kk_any) {  // shard: this rank's raw intrinsics sums go into the exchange
            if (diag && r0 <= kb && kb < r0 + 16 && tid < SEGINTR) lin_w[tid] = io[tid];
            linr = nullptr;
        } else if (kk_any) {
            if (tid == 0) {
                const double gm = intr_lin(P, c, P.K[cur], io, l16);
                if (diag && r0 <= kb && kb < r0 + 16) {
                    lin_w[0] = l16[0];
                    for (int q = 2; q < LIN_N; ++q) lin_w[q] = l16[q];
                    atomic_max_nonneg(lin_w + 1, gm);
                }
            }
            __syncthreads();
            linr = l16;
        }
        ac0 = lo;
        cd = cds;
    }
    if (stop) return;
    const double* sk = scale + P.off_k;
    double v = 0.0;
    if (fin == 2) {
        // landmark shard, folded exchange: this rank's camera-side terms without the LM diagonal and the
        // prior (k_env_unpack_fin adds them from the reduced sums); the pad identity on rank 0
        if (r < nd && col <= r && r / 6 == col / 6) {
            const int ac = r / 6, i = col - 6 * ac, j = r - 6 * ac;
            const int q = 6 * i - i * (i - 1) / 2 + (j - i);
            v = scale[6 * ac + i] * cd[(size_t)(ac - ac0) * CAMDATA + q] * scale[6 * ac + j];
        } else if (r >= kb && r < kb + 4 && col < nd) {
            const int m = r - kb, ac = col / 6, i = col - 6 * ac;
            v = scale[6 * ac + i] * cd[(size_t)(ac - ac0) * CAMDATA + 21 + i * 4 + m] * sk[m];
        } else if (r >= kb && r < kb + 4 && col >= kb && col <= r) {
            const int m = col - kb, l = r - kb;
            const int q = 4 * m - m * (m - 1) / 2 + (l - m);
            v = sk[m] * io[q] * sk[l];
        } else if (r == col && r >= P.n && P.rank == 0) {
            v = 1.0;
        }
    } else if (P.rank == 0) {
        const double radius = st->radius;
        if (r < nd && col <= r && r / 6 == col / 6) {
            const int ac = r / 6, i = col - 6 * ac, j = r - 6 * ac;
            const int q = 6 * i - i * (i - 1) / 2 + (j - i);
            const double* sc = scale + 6 * ac;
            v = sc[i] * cd[(size_t)(ac - ac0) * CAMDATA + q] * sc[j];
            if (i == j) v += fmin(fmax(v, c.min_diag), c.max_diag) / radius;
        } else if (r >= kb && r < kb + 4 && col < nd) {
            const int m = r - kb, ac = col / 6, i = col - 6 * ac;
            v = scale[6 * ac + i] * cd[(size_t)(ac - ac0) * CAMDATA + 21 + i * 4 + m] * sk[m];
        } else if (r >= kb && r < kb + 4 && col >= kb && col <= r) {
            const int m = col - kb, l = r - kb;
            const int q = 4 * m - m * (m - 1) / 2 + (l - m);
            v = sk[m] * linr[2 + q] * sk[l];
            if (l == m) v += fmin(fmax(v, c.min_diag), c.max_diag) / radius;
        } else if (r == col && r >= P.n) {
            v = 1.0;
        }
    }
    if (!accumulate) S[(size_t)r * P.npad + col] = v;
    else if (v != 0.0) atomicAdd(&S[(size_t)r * P.npad + col], v);  // S zeroed by the last back-substitution
    if (ij.x == ij.y && tid < 16) {
        const int rr = 16 * ij.x + tid;
        double b = 0.0;
        if (fin == 2) {
            if (rr < nd) b = scale[rr] * cd[(size_t)(rr / 6 - ac0) * CAMDATA + 45 + rr % 6];
            else if (rr < kb + 4) b = sk[rr - kb] * io[10 + rr - kb];
        } else if (P.rank == 0) {
            if (rr < nd) b = scale[rr] * cd[(size_t)(rr / 6 - ac0) * CAMDATA + 45 + rr % 6];
            else if (rr < kb + 4) b = sk[rr - kb] * linr[12 + rr - kb];
        }
        if (!accumulate) rhs[rr] = b;
        else if (b != 0.0) atomicAdd(&rhs[rr], b);
    }
    if (t == 0 && tid == 0) *chol_flag = 0;
}
// Standalone assembly (windows without active points; otherwise these tiles are extra workgroups of
// k_point_prep, and k_schur_tile's last workgroup adds the points' intrinsics Schur terms).
__global__ __launch_bounds__(TPB) void k_env_assemble(DevProblem P, BaConsts c, const LmState* __restrict__ st,
                                                      const int2* __restrict__ tiles, const double* __restrict__ camdata,
                                                      const double* __restrict__ lin, const double* __restrict__ scale,
                                                      double* __restrict__ S, double* __restrict__ rhs,
                                                      int* __restrict__ chol_flag, int fin,
                                                      const double* __restrict__ cpart,
                                                      const double* __restrict__ seg_intr, double* camdata_w,
                                                      double* lin_w) {
    if (st->done || (!fin && st->stop_next)) return;
    env_tile(P, c, st, blockIdx.x, tiles, camdata, lin, scale, S, rhs, chol_flag, fin, cpart, seg_intr, camdata_w,
             lin_w);
}

template <int PP_LANES, bool O32>
__device__ __forceinline__ void point_prep_block(const DevProblem& P, const BaConsts& c, const LmState* __restrict__ st,
                                                 int mode, const double* __restrict__ scale, double* __restrict__ cnp,
                                                 double* __restrict__ pdata, double* __restrict__ part, const int b,
                                                 const int ap0 = 0, const int pb = -1, double* kkS = nullptr,
                                                 double* kkR = nullptr);
// Workgroups >= nb_pp assemble the envelope tiles of S (env_tile; independent of the point records),
// so the assembly needs no launch of its own.
template <int PP_LANES, bool O32>
__global__ __launch_bounds__(PP_TPB) void k_point_prep(DevProblem P, BaConsts c, const LmState* __restrict__ st, int mode,
                                                       const double* __restrict__ scale, double* __restrict__ cnp,
                                                       double* __restrict__ pdata, double* __restrict__ S,
                                                       double* __restrict__ rhs, double* __restrict__ part, int nb_pp,
                                                       const int2* __restrict__ tiles,
                                                       const double* __restrict__ camdata,
                                                       const double* __restrict__ lin, int* __restrict__ chol_flag,
                                                       int fin, const double* __restrict__ cpart,
                                                       const double* __restrict__ seg_intr, double* camdata_w,
                                                       double* lin_w) {
    if ((int)blockIdx.x >= nb_pp) {
        if (!st->done && (fin || !st->stop_next))
            env_tile(P, c, st, blockIdx.x - nb_pp, tiles, camdata, lin, scale, S, rhs, chol_flag, fin, cpart, seg_intr,
                     camdata_w, lin_w);
        return;
    }
    point_prep_block<PP_LANES, O32>(P, c, st, mode, scale, cnp, pdata, part, blockIdx.x);
}
// One observation's point-side sums: acc = V packed (6) | e (3) | Kt (12)
__device__ __forceinline__ void point_accum(double* acc, const double* jp, const double* jk, const ObsEval& ev) {
    acc[0] += jp[0] * jp[0] + jp[3] * jp[3] + jp[6] * jp[6];
    acc[1] += jp[0] * jp[1] + jp[3] * jp[4] + jp[6] * jp[7];
    acc[2] += jp[0] * jp[2] + jp[3] * jp[5] + jp[6] * jp[8];
    acc[3] += jp[1] * jp[1] + jp[4] * jp[4] + jp[7] * jp[7];
    acc[4] += jp[1] * jp[2] + jp[4] * jp[5] + jp[7] * jp[8];
    acc[5] += jp[2] * jp[2] + jp[5] * jp[5] + jp[8] * jp[8];
#pragma unroll
    for (int i = 0; i < 3; ++i) acc[6 + i] += jp[i] * ev.f[0] + jp[3 + i] * ev.f[1] + jp[6 + i] * ev.f[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {  // Kt = Jk^T Jp: jk row 0 is [k0, 0, su, 0], row 1 [0, k1, 0, su]
        acc[9 + 0 * 3 + i] += jk[0] * jp[i];
        acc[9 + 1 * 3 + i] += jk[5] * jp[3 + i];
        acc[9 + 2 * 3 + i] += jk[2] * jp[i];
        acc[9 + 3 * 3 + i] += jk[7] * jp[3 + i];
    }
}
// The point side of one active point on one thread (point_prep_block with one lane per point, the same sums in the
// same order): its record rec[PDATA], intrinsics terms kk[14], and its gradient max / bad flag max-accumulated.
template <bool O32>
__device__ __forceinline__ void point_rec(const DevProblem& P, const BaConsts& c, int cur, double radius,
                                          const double* __restrict__ scale, int ap, double* rec, double* kk,
                                          double& gmax, double& bad) {
    const double* X = P.pts[cur] + 3 * P.pt_idx[ap];
    const double* K = P.K[cur];
    const double* cams = P.cams[cur];
    double acc[21];
#pragma unroll
    for (int i = 0; i < 21; ++i) acc[i] = 0.0;
    const int o0 = P.pt_ptr[ap], o1 = P.pt_ptr[ap + 1];
    ObsRaw<O32> r_n = o0 < o1 ? po_obs<O32>(P, o0) : obs_zero<O32>();
    for (int o = o0; o < o1; ++o) {
        const ObsRaw<O32> r = r_n;
        double pose[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) pose[k] = cams[7 * r.idx() + k];
        if (o + 1 < o1) r_n = po_obs<O32>(P, o + 1);
        ObsEval ev;
        double jc[18], jp[9], jk[8];
        lin_obs(c, pose, X, K, r.u(), r.v(), r.d(), ev, jc, jp, jk);
        (void)jc;
        point_accum(acc, jp, jk, ev);
    }
    point_tail(P, c, radius, scale, ap, X, acc, true, rec, kk, gmax, bad);
}
// The points' intrinsics Schur terms of one workgroup (out[14]: -Zk Zk^T packed, -Zk ze) added to S_kk / rhs_k.
__device__ __forceinline__ void kk_add(const DevProblem& P, const double* out, double* S, double* rhs, bool atomic) {
    if (threadIdx.x < 10) {
        int m = 0, q = threadIdx.x;
        while (q >= 4 - m) { q -= 4 - m; ++m; }
        const int l = m + q;  // packed (m, l), l >= m
        if (atomic) atomicAdd(&S[(size_t)(P.kb + l) * P.npad + P.kb + m], out[threadIdx.x]);
        else S[(size_t)(P.kb + l) * P.npad + P.kb + m] += out[threadIdx.x];
    } else if (threadIdx.x < 14) {
        if (atomic) atomicAdd(&rhs[P.kb + threadIdx.x - 10], out[threadIdx.x]);
        else rhs[P.kb + threadIdx.x - 10] += out[threadIdx.x];
    }
}
// Point-side body of k_point_prep for point workgroup b (see k_point_prep). The small-window Schur launch
// (k_schur_tile<..., FP>) runs it for the non-tiled points: points ap0 + point block pb, partial slot b, and the
// intrinsics terms added to S / rhs (kkS / kkR, atomics) instead of a partial slot.
template <int PP_LANES, bool O32>
__device__ __forceinline__ void point_prep_block(const DevProblem& P, const BaConsts& c, const LmState* __restrict__ st,
                                                 int mode, const double* __restrict__ scale, double* __restrict__ cnp,
                                                 double* __restrict__ pdata, double* __restrict__ part, const int b,
                                                 const int ap0, const int pb, double* kkS, double* kkR) {
    __shared__ double lds[4 * 14];
    __shared__ double out[14];
    __shared__ double red[4];
    if (st->done) return;
    const int cur = st->cur;
    const double radius = st->radius;
    const int gt = (pb < 0 ? b : pb) * PP_TPB + threadIdx.x;
    const int ap = ap0 + gt / PP_LANES, q = gt % PP_LANES;
    double kk[14];
#pragma unroll
    for (int i = 0; i < 14; ++i) kk[i] = 0.0;
    double gmax = 0.0, bad = 0.0;
    if (ap < P.n_ap) {  // uniform over the lane group
        const int pi = P.pt_idx[ap];
        const double* X = P.pts[cur] + 3 * pi;
        const double* K = P.K[cur];
        // acc: V packed (6) | e (3) | Kt (12)
        double acc[21];
#pragma unroll
        for (int i = 0; i < 21; ++i) acc[i] = 0.0;
        const int o1 = P.pt_ptr[ap + 1];
        // software pipeline: observation record (camera index, pixel, depth) two observations ahead, pose one ahead
        const double* cams = P.cams[cur];
        const int o0 = P.pt_ptr[ap] + q;
        ObsRaw<O32> r_n = o0 < o1 ? po_obs<O32>(P, o0) : obs_zero<O32>();
        ObsRaw<O32> r_nn = o0 + PP_LANES < o1 ? po_obs<O32>(P, o0 + PP_LANES) : obs_zero<O32>();
        double pose_n[7];
        if (o0 < o1) {
#pragma unroll
            for (int k = 0; k < 7; ++k) pose_n[k] = cams[7 * r_n.idx() + k];
        }
        for (int o = o0; o < o1; o += PP_LANES) {
            double pose[7];
#pragma unroll
            for (int k = 0; k < 7; ++k) pose[k] = pose_n[k];
            const ObsRaw<O32> r = r_n;
            const int on = o + PP_LANES;
            if (on < o1) {
                r_n = r_nn;
#pragma unroll
                for (int k = 0; k < 7; ++k) pose_n[k] = cams[7 * r_n.idx() + k];
                r_nn = on + PP_LANES < o1 ? po_obs<O32>(P, on + PP_LANES) : obs_zero<O32>();
            }
            ObsEval ev;
            double jc[18], jp[9], jk[8];
            lin_obs(c, pose, X, K, r.u(), r.v(), r.d(), ev, jc, jp, jk);
            (void)jc;
            point_accum(acc, jp, jk, ev);
        }
        if (mode == 0) {
            double v3[3] = {acc[0], acc[3], acc[5]};
            group_sum<PP_LANES>(v3);
            #pragma unroll
            for (int i = 0; i < 3; ++i)
                if (i % PP_LANES == q) cnp[3 * ap + i] = v3[i];
        } else {
            group_sum<PP_LANES>(acc);
            double rec[PDATA];
            point_tail(P, c, radius, scale, ap, X, acc, q == 0, rec, kk, gmax, bad);
            double* pd_out = pdata + (size_t)ap * PDATA;
#pragma unroll
            for (int i = 0; i < PDATA; ++i)
                if (i % PP_LANES == q) pd_out[i] = rec[i];
        }
    }
    if (mode == 0) return;
    block_sum<14>(kk, lds, out);
    gmax = block_max(gmax, red);
    bad = block_max(bad, red);
    // intrinsics terms: one partial per workgroup, summed in a fixed order by k_schur_tile's last workgroup (a
    // same-address f64 atomic per workgroup serialises at ~45 ns each: 391 x 14 of them cost ~17 us)
    if (kkS) kk_add(P, out, kkS, kkR, true);
    else if (threadIdx.x < 14) part[(PART_PT_KK + threadIdx.x) * P.part_stride + b] = out[threadIdx.x];
    if (threadIdx.x == 0) {
        part[PART_PT_GMAX * P.part_stride + b] = gmax;
        part[PART_PT_BAD * P.part_stride + b] = bad;
    }
}

// Fused linearisation launch of the LM loop (default mode): point workgroups [0, nb_pp) run
// k_point_prep's point side, the rest k_cam_side's sub-segments (gated on an accepted step). mode 0
// (IterationZero): the points' column norms and the ungated camera side. The point
// side alone is one long dependent chain per thread at ~1.5 waves per SIMD; the camera sub-segments fill
// the CUs it leaves idle. The envelope tiles, which need the camera sums, ride in k_schur_tile.
template <int PP_LANES, bool O32>
__global__ __launch_bounds__(TPB) void k_lin_point(DevProblem P, BaConsts c, const LmState* __restrict__ st,
                                                   const double* __restrict__ scale, double* __restrict__ cnp,
                                                   double* __restrict__ pdata, double* __restrict__ part, int nb_pp,
                                                   double* __restrict__ cpart, double* __restrict__ seg_intr,
                                                   double* __restrict__ gmax_word, int mode, int ap0, int slot0) {
    // (ap0 / slot0: the fused-point-side Schur path runs only the non-tiled points here, into slots after the tiles')
    if ((int)blockIdx.x < nb_pp)
        point_prep_block<PP_LANES, O32>(P, c, st, mode, scale, cnp, pdata, part, slot0 + blockIdx.x, ap0, blockIdx.x);
    else cam_side_block<O32>(P, c, st, mode, cpart, seg_intr, gmax_word,
                        P.xcd_map ? xcd_seg(blockIdx.x, nb_pp, P.n_seg) : (int)blockIdx.x - nb_pp);
}

// Jacobi scale (Ceres: 1 / (1 + sqrt(squared column norm)), iteration 0 only)
__global__ void k_scale(DevProblem P, const double* __restrict__ camdata, const double* __restrict__ cnp,
                        const double* __restrict__ lin, int jacobi, double* __restrict__ scale) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int ncam = 6 * P.nac, npt = 3 * P.n_ap;
    double cn = -1.0;
    int dst = -1;
    if (t < ncam) {
        const int ac = t / 6, d = t % 6;
        // diag of the packed upper U: index of (d,d) = d*6 - d*(d-1)/2
        cn = camdata[(size_t)ac * CAMDATA + d * 6 - (d * (d - 1)) / 2];
        dst = t;
    } else if (t < ncam + npt) {
        cn = cnp[t - ncam];
        dst = P.off_pt + (t - ncam);
    } else if (t < ncam + npt + 4) {
        const int m = t - ncam - npt;
        cn = lin[2 + m * 4 - (m * (m - 1)) / 2];
        dst = P.off_k + m;
    }
    if (dst >= 0) scale[dst] = jacobi ? 1.0 / (1.0 + sqrt(cn)) : 1.0;
}

// ---------------------------------------------------------------- assembly
// Writes the camera/intrinsics (F-block) part of the damped, scaled normal
// equations into the lower triangle of S (row-major, npad stride) and rhs = J~^T f.
__global__ void k_assemble(DevProblem P, BaConsts c, const LmState* __restrict__ st, const double* __restrict__ camdata,
                           const double* __restrict__ lin, const double* __restrict__ scale, double* __restrict__ S,
                           double* __restrict__ rhs) {
    if (skip_step(st)) return;
    const double radius = st->radius;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const size_t ld = P.npad;
    const int kb = P.kb;
    const double* sk = scale + P.off_k;
    if (t < P.nac) {
        const int ac = t;
        const double* cd = camdata + (size_t)ac * CAMDATA;
        const double* sc = scale + 6 * ac;
        const int b = 6 * ac;
        int q = 0;
        for (int i = 0; i < 6; ++i)
            for (int j = i; j < 6; ++j, ++q) {
                double v = sc[i] * cd[q] * sc[j];
                if (i == j) v += fmin(fmax(v, c.min_diag), c.max_diag) / radius;
                S[(size_t)(b + j) * ld + b + i] = v;  // lower: row b+j >= col b+i
            }
        for (int i = 0; i < 6; ++i)
            for (int m = 0; m < 4; ++m) S[(size_t)(kb + m) * ld + b + i] = sc[i] * cd[21 + i * 4 + m] * sk[m];
        for (int i = 0; i < 6; ++i) rhs[b + i] = sc[i] * cd[45 + i];
    } else if (t == P.nac) {
        int q = 0;
        for (int m = 0; m < 4; ++m)
            for (int l = m; l < 4; ++l, ++q) {
                double v = sk[m] * lin[2 + q] * sk[l];
                if (l == m) v += fmin(fmax(v, c.min_diag), c.max_diag) / radius;
                S[(size_t)(kb + l) * ld + kb + m] = v;
            }
        for (int m = 0; m < 4; ++m) rhs[kb + m] = sk[m] * lin[12 + m];
        for (int r = P.n; r < P.npad; ++r) { S[(size_t)r * ld + r] = 1.0; rhs[r] = 0.0; }
    }
}

// Schur scatter for the OVERFLOW points (span > TILE_WIN cameras or repeated
// cameras): thread per listed observation, global f64 atomics.
template <bool O32>
__global__ __launch_bounds__(TPB) void k_obs_pairs(DevProblem P, BaConsts c, const LmState* __restrict__ st,
                                                   const double* __restrict__ scale,
                                                   const double* __restrict__ pdata, double* __restrict__ S,
                                                   double* __restrict__ rhs) {
    if (skip_step(st)) return;
    const int cur = st->cur;
    const int t = blockIdx.x * TPB + threadIdx.x;
    if (t >= P.n_ovf_obs) return;
    const int a = P.ovf_obs[t];
    const int ca = P.po_ac[a];
    if (ca < 0) return;
    const int ap = P.po_ap[a];
    const size_t ld = P.npad;
    const int kb = P.kb;
    const double* pd = pdata + (size_t)ap * PDATA;
    double Vf[9];
    vinv_from_g(pd, Vf);
    const double* sp = scale + P.off_pt + 3 * ap;
    const double* X = P.pts[cur] + 3 * P.pt_idx[ap];
    const double* K = P.K[cur];
    // W~_a = s_c (Jc^T Jp) s_p
    double Y[18];
    {
        const ObsRaw<O32> o = po_obs<O32>(P, a);
        ObsEval ev;
        double jc[18], jp[9], jk[8];
        lin_obs(c, P.cams[cur] + 7 * o.idx(), X, K, o.u(), o.v(), o.d(), ev, jc, jp, jk);
        const double* sc = scale + 6 * ca;
        double W[18];
        w_tilde(jc, jp, sc, sp, W);
#pragma unroll
        for (int d = 0; d < 6; ++d)
#pragma unroll
            for (int i = 0; i < 3; ++i)
                Y[d * 3 + i] = W[d * 3 + 0] * Vf[0 * 3 + i] + W[d * 3 + 1] * Vf[1 * 3 + i] + W[d * 3 + 2] * Vf[2 * 3 + i];
    }
    // rhs_c -= Y e ; border -= Y Kt^T
#pragma unroll
    for (int d = 0; d < 6; ++d) {
        atomicAdd(&rhs[6 * ca + d], -(Y[d * 3 + 0] * pd[6] + Y[d * 3 + 1] * pd[7] + Y[d * 3 + 2] * pd[8]));
#pragma unroll
        for (int m = 0; m < 4; ++m)
            atomicAdd(&S[(size_t)(kb + m) * ld + 6 * ca + d],
                      -(Y[d * 3 + 0] * pd[9 + m * 3 + 0] + Y[d * 3 + 1] * pd[9 + m * 3 + 1] + Y[d * 3 + 2] * pd[9 + m * 3 + 2]));
    }
    // pairs (a,b) with cam(b) > cam(a) or (same cam and b >= a)
    for (int b = P.pt_ptr[ap]; b < P.pt_ptr[ap + 1]; ++b) {
        const int cb = P.po_ac[b];
        if (cb < ca || (cb == ca && b < a)) continue;
        const ObsRaw<O32> o = po_obs<O32>(P, b);
        ObsEval ev;
        double jc[18], jp[9], jk[8];
        lin_obs(c, P.cams[cur] + 7 * o.idx(), X, K, o.u(), o.v(), o.d(), ev, jc, jp, jk);
        const double* sc = scale + 6 * cb;
        double W[18];
        w_tilde(jc, jp, sc, sp, W);
        // M = Y_a W_b^T  (block (ca, cb)); lower storage S[6cb + e][6ca + d]
        if (cb > ca) {
#pragma unroll
            for (int d = 0; d < 6; ++d)
#pragma unroll
                for (int e2 = 0; e2 < 6; ++e2)
                    atomicAdd(&S[(size_t)(6 * cb + e2) * ld + 6 * ca + d],
                              -(Y[d * 3 + 0] * W[e2 * 3 + 0] + Y[d * 3 + 1] * W[e2 * 3 + 1] + Y[d * 3 + 2] * W[e2 * 3 + 2]));
        } else {
            const bool self = (b == a);
#pragma unroll
            for (int d = 0; d < 6; ++d)
#pragma unroll
                for (int e2 = d; e2 < 6; ++e2) {
                    double m = Y[d * 3 + 0] * W[e2 * 3 + 0] + Y[d * 3 + 1] * W[e2 * 3 + 1] + Y[d * 3 + 2] * W[e2 * 3 + 2];
                    if (!self)
                        m += Y[e2 * 3 + 0] * W[d * 3 + 0] + Y[e2 * 3 + 1] * W[d * 3 + 1] + Y[e2 * 3 + 2] * W[d * 3 + 2];
                    atomicAdd(&S[(size_t)(6 * ca + e2) * ld + 6 * ca + d], -m);
                }
        }
    }
}

// Schur reduction over the TILED points (the common, banded case), on the f64 matrix cores.
// One workgroup per tile: a run of points (sorted by first camera) whose active cameras
// all lie in the window [base, base+span), span <= TILE_WIN. For a chunk of <= CHUNK_PTS
// points the tile's Schur term is a small dense product: with M' the (6 span + 5) x 3 npts
// matrix whose column (p, j) holds, for every camera c observing p, the rows
// 6c..6c+5 = Z_(p,c)[:, j] (Z = W~ G^T, zero where c does not observe p), then the
// 4 rows Zk = K~ G^T and one row ze = G e~,
//     S_cc -= M'_c M'_c^T,  S_kc -= M'_k M'_c^T,  rhs_c -= M'_c ze.
// Phase A (thread per observation / per point) writes M' k-major into LDS; phase B: each
// wave owns up to 4 of the (<= 15) lower 16x16 tiles of M' M'^T and runs 4 independent
// v_mfma_f64_16x16x4 chains over K = 3 npts, accumulating across chunks in registers.
// The tile is flushed into S / rhs once (f64 atomics, lower triangle). The intrinsics-
// intrinsics terms stay in k_point_prep, which also covers the overflow points.
__device__ __forceinline__ unsigned long long stamp_now() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
typedef double d4 __attribute__((ext_vector_type(4)));
static constexpr int SCH_K = 3 * CHUNK_PTS;   // K extent of one chunk
static constexpr int SCH_LDM = 80;            // rows of M' (6 * TILE_WIN + 5 <= 80)
static_assert(SCH_LDM * 6 * TILE_WIN == SCH_TBUF, "deterministic slab geometry");
static_assert(6 * TILE_WIN + 5 <= SCH_LDM, "M' rows exceed 5 MFMA tiles");
static_assert(CHUNK_OBS <= TPB, "phase A: one observation per thread");

// Envelope tiles riding in k_schur_tile (fused LM-loop path, n_env > 0): what env_tile needs. They add
// their values to an S (and rhs) that the previous back-substitution (k_final) zeroed, concurrently with the
// tiles' flushes, so every writer of S in that launch is an atomic add.
struct EnvArgs {
    const int2* tiles;
    int n_env;
    const double* camdata;
    const double* lin;
    int* chol_flag;
    const double* cpart;
    const double* seg_intr;
    double* camdata_w;
    double* lin_w;
    int fin;  // 1: unsharded (finish the camera sums, lin); 2: landmark shard (local terms for the exchange)
    // the small-window launch (k_schur_tile<..., FP>): the camera side and the non-tiled points ride in it
    double* pdata_w;   // the point records the tiles compute (for the back-substitution)
    double* part_w;    // per-tile gradient max / bad partials (k_final)
    double* cpart_w;   // camera-side sub-segment partials (written by the camera-side workgroups)
    double* seg_intr_w;
    unsigned* sw_cnt;  // camera-side workgroups finished (monotonic within a solve)
    unsigned sw_target;
    int n_cs, n_gb;    // camera-side workgroups (= n_seg), non-tiled point workgroups
};

// PF (small grids, where occupancy does not bound the launch): each chunk's point records (G, e~, K~) are loaded
// with the chunk's observation records — in the prologue, then a chunk ahead under the MFMAs — instead of at the
// start of phase A.
//
// FP (small windows, PF only; no k_lin_point in the LM loop): workgroups [0, n_tiles) are tiles that first compute
// their own points' point side (point_rec, one point per thread; also in the terminal stop_next iteration, for the
// gradient max): the records to pdata for phase A and the back-substitution, the intrinsics terms into S / rhs;
// workgroup n_tiles idles; then n_cs camera-side workgroups (cam_side_block, each counted in sw_cnt when done),
// n_gb workgroups for the non-tiled points (point_prep_block), and the envelope tiles, which wait until the
// camera side of this launch is counted (every workgroup of the launch is resident: the host launches FP only
// when they fit one round). A wait that times out raises FLAG_TIMEOUT (the iteration is re-run without FP).
// Polls before the wait gives up: sw_set_spin_limit (MIBA_BCR_SPIN_LIMIT forces the timeout path in the tests).
__device__ unsigned g_sw_spin_limit = 1u << 20;
__device__ __forceinline__ bool sw_wait(const unsigned* cnt, unsigned target) {
    const unsigned lim = g_sw_spin_limit;
    for (unsigned i = 0; i < lim; ++i) {
        // relaxed: the camera side's outputs are read past the L2 (env_tile pub), no invalidate needed
        if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}
template <bool STAMP, bool O32, bool PF, bool FP, bool SW>
__device__ __forceinline__ void schur_tile_body(DevProblem P, BaConsts c, const LmState* __restrict__ st,
                                                const double* __restrict__ scale, const double* __restrict__ pdata,
                                                double* __restrict__ S, double* __restrict__ rhs,
                                                unsigned long long* __restrict__ stamps, int nblk_pt,
                                                const double* __restrict__ part, double* __restrict__ tbuf, EnvArgs E) {
    static_assert(!SW || FP, "the small-window launch runs the point side in its tiles");
    __shared__ __attribute__((aligned(16))) double Mt[SCH_K * SCH_LDM];  // Mt[k][row] = M'[row][k]
    __shared__ double zeL[SCH_K];                                         // rhs row of M' when aside
    __shared__ double gL[FP ? 6 * CHUNK_PTS : 1];                         // FP: the chunk's G (phase A)
    // FP: the chunk's point records (phase A's per-point part) and each point thread's intrinsics terms, in LDS
    // rather than registers (the point side's registers would otherwise cost the tile its second workgroup per CU)
    __shared__ double qL[FP ? 21 * CHUNK_PTS : 1];
    __shared__ double kkL[FP ? 14 * CHUNK_PTS : 1];
    // FP: per-observation point sums, in M' before the chunk clears it
    static_assert(21 * CHUNK_OBS <= SCH_K * SCH_LDM, "the point sums fit M'");
    double* const psum = Mt;
    if constexpr (SW) {
        const int b = (int)blockIdx.x - P.n_tiles - 1;
        if (b >= 0 && b < E.n_cs) {  // camera side (gated on an accepted step), counted whatever it did
            // outputs stored past the L2 and drained by every thread, then counted: no release fence (an L2
            // write-back) between the camera side and the envelope tiles
            cam_side_block<O32>(P, c, st, 1, E.cpart_w, E.seg_intr_w, E.lin_w + 1, b, true);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0) __hip_atomic_fetch_add(E.sw_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        if (b >= E.n_cs && b < E.n_cs + E.n_gb) {  // non-tiled points (intrinsics terms into S unless stop_next)
            const bool sn = st->stop_next;
            point_prep_block<1, O32>(P, c, st, 1, scale, nullptr, E.pdata_w, E.part_w, P.n_tiles + b - E.n_cs,
                                     P.n_tiled_pts, b - E.n_cs, sn ? nullptr : S, rhs);
            return;
        }
        if (b >= E.n_cs + E.n_gb) {  // envelope tiles, after this launch's camera side
            if (st->done) return;
            __shared__ int sw_ok;
            if (threadIdx.x == 0) sw_ok = sw_wait(E.sw_cnt, E.sw_target) ? 1 : 0;
            __syncthreads();
            env_tile(P, c, st, b - E.n_cs - E.n_gb, E.tiles, E.camdata, E.lin, scale, S, rhs, E.chol_flag, E.fin,
                     E.cpart, E.seg_intr, E.camdata_w, E.lin_w, true, true);
            if (!sw_ok && threadIdx.x == 0) atomicOr(E.chol_flag, FLAG_TIMEOUT);
            return;
        }
        if (b == -1) return;  // (workgroup n_tiles: the tiles add the intrinsics terms themselves)
        if (st->done) return;
    } else {
    if ((int)blockIdx.x > P.n_tiles) {  // envelope tiles (fused path): also in the terminal stop_next iteration
        if (!st->done)
            env_tile(P, c, st, blockIdx.x - P.n_tiles - 1, E.tiles, E.camdata, E.lin, scale, S, rhs, E.chol_flag, E.fin,
                     E.cpart, E.seg_intr, E.camdata_w, E.lin_w, true);
        return;
    }
    if constexpr (FP) {  // (FP tiles run in the terminal stop_next iteration too: the decision needs their gradient max)
        if (st->done || ((int)blockIdx.x == P.n_tiles && st->stop_next)) return;
    } else if (skip_step(st)) return;
    }
    if (!SW && (int)blockIdx.x == P.n_tiles) {
        // last workgroup: S_kk += the points' intrinsics Schur terms (k_point_prep's per-workgroup partials,
        // fixed order), rhs_k likewise. No tile writes S_kk or rhs_k (FP: the non-tiled points' partials, slots
        // after the tiles'; the tiles add theirs).
        double acc[14];
#pragma unroll
        for (int q = 0; q < 14; ++q) acc[q] = 0.0;
        const int s0 = FP ? P.n_tiles : 0;
        for (int i = threadIdx.x; i < nblk_pt; i += TPB)
#pragma unroll
            for (int q = 0; q < 14; ++q) acc[q] += part[(PART_PT_KK + q) * P.part_stride + s0 + i];
        block_sum<14>(acc, Mt, Mt + 64);
        const double* out = Mt + 64;
        if (threadIdx.x < 10) {
            int m = 0, q = threadIdx.x;
            while (q >= 4 - m) { q -= 4 - m; ++m; }
            const int l = m + q;  // packed (m, l), l >= m
            if (E.n_env) atomicAdd(&S[(size_t)(P.kb + l) * P.npad + P.kb + m], out[threadIdx.x]);
            else S[(size_t)(P.kb + l) * P.npad + P.kb + m] += out[threadIdx.x];
        } else if (threadIdx.x < 14) {
            if (E.n_env) atomicAdd(&rhs[P.kb + threadIdx.x - 10], out[threadIdx.x]);
            else rhs[P.kb + threadIdx.x - 10] += out[threadIdx.x];
        }
        return;
    }
    unsigned long long t_prev = 0, st_acc[5] = {0, 0, 0, 0, 0}, sub_st[5] = {0, 0, 0, 0, 0};
#define SCH_STAMP(k)                                          \
    do {                                                      \
        if constexpr (STAMP) {                                \
            if (threadIdx.x == 0) {                           \
                const unsigned long long t_ = stamp_now();    \
                st_acc[k] += t_ - t_prev;                     \
                t_prev = t_;                                  \
            }                                                 \
        }                                                     \
    } while (0)
    if constexpr (STAMP) if (threadIdx.x == 0) t_prev = stamp_now();
    const int cur = st->cur;
    const int tile = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rr = lane & 15, kq = lane >> 4;
    const int base = P.tile_base[tile];
    const int span = P.tile_span[tile];
    const int kr = 6 * span, er = kr + 4;     // intrinsics rows, rhs row of M'
    // span <= 10 (the common tile: one run of points observed by the same 10 cameras): M' without its rhs
    // row fits 4 row tiles (60 camera + 4 intrinsics rows), so the MFMA product has 10 lower tiles instead of
    // 15; the rhs row's products rhs_c -= M'_c ze are a VALU dot product on wave 3 (2 of the 10 tiles)
    const bool rhs_aside = er <= 64;
    const int nrt = (er + (rhs_aside ? 0 : 1) + 15) >> 4;  // 16-row tiles of M'
    const int ntl = nrt * (nrt + 1) / 2;                     // lower tiles of M' M'^T
    // lower tiles in reverse row-major order, 4 consecutive per wave (operand rows shared within a
    // wave), or round-robin over the waves when the rhs row is aside (10 tiles: 3, 3, 2, 2); slots past
    // ntl duplicate tile (0,0) and are never flushed
    int tib[4], tjb[4];
    bool tok[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int u = rhs_aside ? wave + 4 * q : 4 * wave + q;
        tok[q] = u < ntl;
        int t = tok[q] ? ntl - 1 - u : 0, ib = 0;
        while (t > ib) { t -= ib + 1; ++ib; }
        tib[q] = ib;
        tjb[q] = t;
    }
    // the valid slots are a prefix; their count is wave-uniform (empty slots issue no MFMA)
    const int ntok = __builtin_amdgcn_readfirstlane((int)tok[0] + (int)tok[1] + (int)tok[2] + (int)tok[3]);
    // waves of the rhs-aside dot product: all four when the product has at most 4 tiles (one MFMA tile per wave at
    // most), else wave 3 alone (spread over the 2-tile waves 2-3 of the 10-tile shape it measured slower at C4)
    const int dw0 = ntl <= 4 ? 0 : 3;
    d4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = d4{0.0, 0.0, 0.0, 0.0};
    double rhs_acc = 0.0;
    const double* K = P.K[cur];
    // Software pipeline over the tile's chunks: the next chunk's bounds and level-1
    // observation records are loaded before this chunk's MFMAs, its level-2 operands
    // (pose, point, scales, G) right after them, so phase A starts with its data resident.
    const int ch_end = P.tile_chunk[tile + 1];
    int ch = P.tile_chunk[tile];
    int apb = P.chunk_ap[ch], ape = P.chunk_ap[ch + 1];
    int ob = P.pt_ptr[apb], oe = P.pt_ptr[ape];
    const int n_last = P.n_adm - 1;
    // the point records: FP writes them first (through a pointer that is not __restrict__) and reads them back
    const double* pdr = FP ? E.pdata_w : pdata;
    double fp_gmax = 0.0, fp_bad = 0.0;  // FP: the tile's points' gradient max, bad flag (point threads)
    if constexpr (FP)
        for (int i = tid; i < 14 * CHUNK_PTS; i += TPB) kkL[i] = 0.0;  // (first read after the first chunk's barrier)
    // level 1: observation record of this thread
    int r_ac, r_ap, r_pt;
    ObsRaw<O32> r_o;  // camera index, pixel, depth
    auto load_rec = [&](int qq) {
        const int qc = qq < n_last ? qq : n_last;
        r_ac = P.po_ac[qc]; r_ap = P.po_ap[qc]; r_pt = P.po_pt[qc];
        r_o = po_obs<O32>(P, qc);
    };
    // level 2: operands of the observation
    double o_pose[7], o_X[3], o_sc[6], o_sp[3], o_G[6];
    bool o_ok = false, o_in = false;
    // in: this thread has an observation of the chunk; ok: ... on an active camera (a column of M'). FP evaluates
    // every observation of the chunk (the point side's sums include the gauge camera's)
    auto load_ops = [&](bool in) {
        const bool ok = in && r_ac >= 0;
        o_ok = ok;
        o_in = in;
        const bool ev = FP ? in : ok;
        const int ac = ok ? r_ac : 0, ap = ok ? r_ap : 0;
        const double* pose = P.cams[cur] + 7 * (ev ? r_o.idx() : 0);
        const double* X = P.pts[cur] + 3 * (ev ? r_pt : 0);
#pragma unroll
        for (int k = 0; k < 7; ++k) o_pose[k] = pose[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) o_X[k] = X[k];
#pragma unroll
        for (int k = 0; k < 6; ++k) o_sc[k] = scale[6 * ac + k];
#pragma unroll
        for (int k = 0; k < 3; ++k) o_sp[k] = scale[P.off_pt + 3 * ap + k];
        if constexpr (!FP)  // FP: G from this chunk's point threads (gL)
#pragma unroll
            for (int k = 0; k < 6; ++k) o_G[k] = pdr[(size_t)ap * PDATA + k];
    };
    double q_pd[(PF && !FP) ? 21 : 1];
    auto load_pq = [&](int a0, int a1) {
        if constexpr (PF && !FP)  // (FP: the chunk's point threads compute them)
            if (tid < a1 - a0)
#pragma unroll
                for (int i = 0; i < 21; ++i) q_pd[i] = pdr[(size_t)(a0 + tid) * PDATA + i];
    };
    const double radius = FP ? st->radius : 0.0;
    if (FP && st->stop_next) {
        // terminal iteration: no step; the decision needs the points' gradient max (point_rec, one point per thread)
        for (int ap = apb + tid; ap < P.chunk_ap[ch_end]; ap += TPB) {
            double rec[PDATA], kkt[14];
            point_rec<O32>(P, c, cur, radius, scale, ap, rec, kkt, fp_gmax, fp_bad);
        }
        fp_gmax = block_max(fp_gmax, zeL);
        fp_bad = block_max(fp_bad, zeL);
        if (tid == 0) {
            E.part_w[PART_PT_GMAX * P.part_stride + tile] = fp_gmax;
            E.part_w[PART_PT_BAD * P.part_stride + tile] = fp_bad;
        }
        return;
    }
    load_rec(ob + tid);
    load_pq(apb, ape);
    load_ops(ob + tid < oe);
    for (;;) {
        const int npts = ape - apb;
        double Wt[FP ? 18 : 1];  // FP: this observation's W~, from its one Jacobian evaluation
        if constexpr (FP) {
            // the point side of the chunk's points from the same evaluation phase A uses: each observation's sums to
            // psum, then one thread per point adds its observations' in order (the sums of point_rec, bitwise)
            if (o_in) {
                ObsEval ev;
                double jc[18], jp[9], jk[8], a[21];
                lin_obs(c, o_pose, o_X, K, r_o.u(), r_o.v(), r_o.d(), ev, jc, jp, jk);
                if (o_ok) w_tilde(jc, jp, o_sc, o_sp, Wt);
#pragma unroll
                for (int i = 0; i < 21; ++i) a[i] = 0.0;
                point_accum(a, jp, jk, ev);
#pragma unroll
                for (int i = 0; i < 21; ++i) psum[i * CHUNK_OBS + tid] = a[i];
            }
            if constexpr (STAMP) if (tid == 0) sub_st[2] += stamp_now() - t_prev;
            __syncthreads();
            if constexpr (STAMP) if (tid == 0) sub_st[3] += stamp_now() - t_prev;
            if (tid < npts) {
                const int ap = apb + tid;
                const int q0 = P.pt_ptr[ap] - ob, q1 = P.pt_ptr[ap + 1] - ob;
                const double* Xp = P.pts[cur] + 3 * P.pt_idx[ap];
                double acc[21], rec[PDATA], kkt[14];
#pragma unroll
                for (int i = 0; i < 21; ++i) acc[i] = 0.0;
                for (int q = q0; q < q1; ++q)
#pragma unroll
                    for (int i = 0; i < 21; ++i) acc[i] += psum[i * CHUNK_OBS + q];
                point_tail(P, c, radius, scale, ap, Xp, acc, true, rec, kkt, fp_gmax, fp_bad);
#pragma unroll
                for (int i = 0; i < 14; ++i) kkL[14 * tid + i] += kkt[i];
#pragma unroll
                for (int i = 0; i < PDATA; ++i) E.pdata_w[(size_t)ap * PDATA + i] = rec[i];
#pragma unroll
                for (int i = 0; i < 21; ++i) qL[21 * tid + i] = rec[i];
#pragma unroll
                for (int k = 0; k < 6; ++k) gL[6 * tid + k] = rec[k];
            }
            if constexpr (STAMP) if (tid == 0) sub_st[4] += stamp_now() - t_prev;
            __syncthreads();  // (psum is M': read before the clear)
        }
        {
            // every thread the same number of 16-byte stores, unrolled: straight-line ds_write_b128 with immediate
            // offsets (the strided loop spent ~120 instructions of issue per thread on 15 stores)
            static_assert(SCH_K * SCH_LDM / 2 % TPB == 0, "zeroing: whole rounds");
            double2* M2 = reinterpret_cast<double2*>(Mt) + tid;
#pragma unroll
            for (int i = 0; i < SCH_K * SCH_LDM / 2 / TPB; ++i) M2[TPB * i] = double2{0.0, 0.0};
        }
        SCH_STAMP(4);  // zero stores issued (wave 0); slot 0 is then the barrier
        __syncthreads();
        SCH_STAMP(0);
        // ---- phase A
        if (tid < npts) {
            const double* pd = FP ? qL + 21 * tid : (PF ? q_pd : pdr + (size_t)(apb + tid) * PDATA);
            double G[6], Ks[12], es[3], zk[12], z3[3];
#pragma unroll
            for (int i = 0; i < 6; ++i) G[i] = pd[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) es[i] = pd[6 + i];
#pragma unroll
            for (int i = 0; i < 12; ++i) Ks[i] = pd[9 + i];
            zk_ze(G, Ks, es, zk, z3);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                double* col = Mt + (3 * tid + j) * SCH_LDM;
#pragma unroll
                for (int m = 0; m < 4; ++m) col[kr + m] = zk[m * 3 + j];
                if (rhs_aside) zeL[3 * tid + j] = z3[j]; else col[er] = z3[j];
            }
        }
        if (o_ok) {
            const int pl = r_ap - apb;
            double W[18];
            if constexpr (FP) {
#pragma unroll
                for (int i = 0; i < 18; ++i) W[i] = Wt[i];
#pragma unroll
                for (int k = 0; k < 6; ++k) o_G[k] = gL[6 * pl + k];
            } else {
                ObsEval ev;
                double jc[18], jp[9], jk[8];
                lin_obs(c, o_pose, o_X, K, r_o.u(), r_o.v(), r_o.d(), ev, jc, jp, jk);
                w_tilde(jc, jp, o_sc, o_sp, W);
            }
            const double g00 = o_G[0], g10 = o_G[1], g11 = o_G[2], g20 = o_G[3], g21 = o_G[4], g22 = o_G[5];
            double* c0 = Mt + (3 * pl) * SCH_LDM + 6 * (r_ac - base);
#pragma unroll
            for (int d = 0; d < 6; ++d) {
                c0[d] = W[d * 3 + 0] * g00;
                c0[SCH_LDM + d] = W[d * 3 + 0] * g10 + W[d * 3 + 1] * g11;
                c0[2 * SCH_LDM + d] = W[d * 3 + 0] * g20 + W[d * 3 + 1] * g21 + W[d * 3 + 2] * g22;
            }
        }
        __syncthreads();
        SCH_STAMP(1);
        // ---- prefetch: next chunk bounds + level-1 records
        const bool more = ch + 1 < ch_end;
        int ape_n = ape;
        if (more) {
            ape_n = P.chunk_ap[ch + 2];
            load_rec(oe + tid);
            load_pq(ape, ape_n);
        }
        // ---- rhs row aside: rhs_acc(r) += sum_k M'[r][k] ze[k] (lane = camera row r), the chunk's k-steps split
        // over the dot waves (waves dw0..3: all four when the product has few tiles, the two 2-tile waves of the
        // 10-tile shape); each wave four interleaved partial chains (k mod 4), its k-steps' loads issued together
        if (rhs_aside && dw0 == 3 && wave == 3 && lane < kr) {  // (the large tiles: wave 3 alone, k in order)
            const int nk = 3 * npts;
            double ra[4] = {0.0, 0.0, 0.0, 0.0};
            int k = 0;
            for (; k + 4 <= nk; k += 4)
#pragma unroll
                for (int u = 0; u < 4; ++u) ra[u] = __builtin_fma(Mt[(k + u) * SCH_LDM + lane], zeL[k + u], ra[u]);
            for (; k < nk; ++k) ra[0] = __builtin_fma(Mt[k * SCH_LDM + lane], zeL[k], ra[0]);
            rhs_acc += (ra[0] + ra[1]) + (ra[2] + ra[3]);
        } else if (rhs_aside && dw0 < 3 && lane < kr) {
            const int nk = 3 * npts, ns = (nk + 3) >> 2, nw = 4 - dw0, wi = wave - dw0;
            const int s0 = ns * wi / nw, s1 = ns * (wi + 1) / nw;
            double ra[4] = {0.0, 0.0, 0.0, 0.0};
            constexpr int UNR = 4;
            for (int sb = s0; sb < s1; sb += UNR) {
                double mv[UNR][4], zv[UNR][4];
#pragma unroll
                for (int q = 0; q < UNR; ++q)
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int k = 4 * (sb + q) + u;
                        const bool in = sb + q < s1 && k < nk;  // (zeL past the chunk's columns is stale)
                        mv[q][u] = in ? Mt[k * SCH_LDM + lane] : 0.0;
                        zv[q][u] = in ? zeL[k] : 0.0;
                    }
#pragma unroll
                for (int q = 0; q < UNR; ++q)
#pragma unroll
                    for (int u = 0; u < 4; ++u) ra[u] = __builtin_fma(mv[q][u], zv[q][u], ra[u]);
            }
            rhs_acc += (ra[0] + ra[1]) + (ra[2] + ra[3]);
        }
        if constexpr (STAMP && FP) if (tid == 0) sub_st[0] += stamp_now() - t_prev;
        // ---- phase B: acc[t] += M'[16 ib..][k] M'[16 jb..][k]^T over the chunk's K
        const int ksteps = (3 * npts + 3) >> 2;
        if ((rhs_aside && nrt == 4) || (!rhs_aside && nrt == 5)) {
            // the two common tile shapes, each wave running a fixed tile list (slot order as tib / tjb) and
            // loading only the row tiles its list reads, once per k-step (<= 5 LDS loads instead of 8):
            //   span <= 10, rhs aside (10 tiles, round-robin):
            //     wave 0: (3,3) (2,2) (1,0) | 1: (3,2) (2,1) (0,0) | 2: (3,1) (2,0) | 3: (3,0) (1,1)
            //   span 11 / 12 (15 tiles, 4 consecutive per wave in reverse row-major order):
            //     wave 0: (4,4) (4,3) (4,2) (4,1) | 1: (4,0) (3,3) (3,2) (3,1) | 2: (3,0) (2,2) (2,1) (2,0)
            //     wave 3: (1,1) (1,0) (0,0)
            const double* row = Mt + kq * SCH_LDM + rr;
            auto run = [&](auto ntag, auto wtag) {
                constexpr int NR = decltype(ntag)::value, W = decltype(wtag)::value;
                constexpr int TI[2][4][4] = {{{3, 2, 1, -1}, {3, 2, 0, -1}, {3, 2, -1, -1}, {3, 1, -1, -1}},
                                             {{4, 4, 4, 4}, {4, 3, 3, 3}, {3, 2, 2, 2}, {1, 1, 0, -1}}};
                constexpr int TJ[2][4][4] = {{{3, 2, 0, -1}, {2, 1, 0, -1}, {1, 0, -1, -1}, {0, 1, -1, -1}},
                                             {{4, 3, 2, 1}, {0, 3, 2, 1}, {0, 2, 1, 0}, {1, 0, 0, -1}}};
                constexpr int S = NR == 4 ? 0 : 1;
                constexpr auto uses = [](int r) {
                    for (int q = 0; q < 4; ++q)
                        if (TI[S][W][q] == r || TJ[S][W][q] == r) return true;
                    return false;
                };
                double rv[5], nv[5];
#pragma unroll
                for (int r = 0; r < 5; ++r) rv[r] = uses(r) ? row[16 * r] : 0.0;
                for (int s4 = 0; s4 < ksteps; ++s4) {
                    const double* nrow = row + (s4 + 1 < ksteps ? 4 * SCH_LDM : 0);
#pragma unroll
                    for (int r = 0; r < 5; ++r) nv[r] = uses(r) ? nrow[16 * r] : 0.0;
#pragma unroll
                    for (int q = 0; q < 4; ++q)  // (constant conditions once unrolled)
                        if (TI[S][W][q] >= 0)
                            acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(rv[TI[S][W][q] < 0 ? 0 : TI[S][W][q]],
                                                                         rv[TJ[S][W][q] < 0 ? 0 : TJ[S][W][q]], acc[q],
                                                                         0, 0, 0);
#pragma unroll
                    for (int r = 0; r < 5; ++r) rv[r] = nv[r];
                    row = nrow;
                }
            };
            using I0 = std::integral_constant<int, 0>;
            using I1 = std::integral_constant<int, 1>;
            using I2 = std::integral_constant<int, 2>;
            using I3 = std::integral_constant<int, 3>;
            if (nrt == 4) {
                switch (wave) {
                    case 0: run(std::integral_constant<int, 4>{}, I0{}); break;
                    case 1: run(std::integral_constant<int, 4>{}, I1{}); break;
                    case 2: run(std::integral_constant<int, 4>{}, I2{}); break;
                    default: run(std::integral_constant<int, 4>{}, I3{}); break;
                }
            } else {
                switch (wave) {
                    case 0: run(std::integral_constant<int, 5>{}, I0{}); break;
                    case 1: run(std::integral_constant<int, 5>{}, I1{}); break;
                    case 2: run(std::integral_constant<int, 5>{}, I2{}); break;
                    default: run(std::integral_constant<int, 5>{}, I3{}); break;
                }
            }
        } else if (ntl == 1) {
            // one 16 x 16 tile (span <= 2: the TUM windows' tiles), M'_0 M'_0^T: the chunk's k-steps split over the
            // four waves (a quarter each, partial products summed in wave order at the flush), each wave's operand
            // rows loaded in one block ahead of its MFMA chain (a wave alone on its SIMD waits out every LDS round
            // trip a one-step-ahead prefetch leaves exposed)
            const double* row = Mt + kq * SCH_LDM + rr;
            const int s0 = ksteps * wave / 4, s1 = ksteps * (wave + 1) / 4;
            constexpr int KB = 8;
            static_assert(KB * 4 >= SCH_K / 4, "a quarter of a chunk's k-steps in one block");
            double av[KB];
#pragma unroll
            for (int q = 0; q < KB; ++q) av[q] = s0 + q < s1 ? row[(s0 + q) * 4 * SCH_LDM] : 0.0;
#pragma unroll
            for (int q = 0; q < KB; ++q)
                if (s0 + q < s1) acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[q], av[q], acc[0], 0, 0, 0);
        } else {
            const double* row = Mt + kq * SCH_LDM + rr;
            double a[4], b[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) { a[t] = row[16 * tib[t]]; b[t] = row[16 * tjb[t]]; }
            for (int s4 = 0; s4 < ksteps; ++s4) {
                double an[4], bn[4];
                const double* nrow = row + (s4 + 1 < ksteps ? 4 * SCH_LDM : 0);
#pragma unroll
                for (int t = 0; t < 4; ++t) { an[t] = nrow[16 * tib[t]]; bn[t] = nrow[16 * tjb[t]]; }
#pragma unroll
                for (int t = 0; t < 4; ++t)
                    if (t < ntok) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t], b[t], acc[t], 0, 0, 0);
#pragma unroll
                for (int t = 0; t < 4; ++t) { a[t] = an[t]; b[t] = bn[t]; }
                row = nrow;
            }
        }
        if constexpr (STAMP && FP) if (tid == 0) sub_st[1] += stamp_now() - t_prev;
        if (!more) break;
        // ---- prefetch: level-2 operands of the next chunk
        const int oe_n = P.pt_ptr[ape_n];
        load_ops(oe + tid < oe_n);
        ++ch;
        apb = ape; ape = ape_n;
        ob = oe; oe = oe_n;
        __syncthreads();
        SCH_STAMP(2);
    }
    __syncthreads();
    SCH_STAMP(2);
    if ((rhs_aside && dw0 < 3) || ntl == 1) {  // (tile-uniform) partials summed in wave order, before any global
        // store of the flush (a barrier after them would wait for their acknowledgement): the dot waves' rhs rows on
        // wave 3; the one-tile product's k-quarters on wave 0
        if (rhs_aside && wave >= dw0 && wave < 3 && lane < kr) Mt[wave * 64 + lane] = rhs_acc;
        if (ntl == 1 && wave > 0)
#pragma unroll
            for (int g = 0; g < 4; ++g) Mt[256 + (wave - 1) * 256 + g * 64 + lane] = acc[0][g];
        __syncthreads();
        if (rhs_aside && wave == 3 && lane < kr) {
            double v = 0.0;
            for (int w = dw0; w < 3; ++w) v += Mt[w * 64 + lane];
            rhs_acc += v;
        }
        if (ntl == 1 && wave == 0)
#pragma unroll
            for (int g = 0; g < 4; ++g)
                acc[0][g] += (Mt[256 + g * 64 + lane] + Mt[512 + g * 64 + lane]) + Mt[768 + g * 64 + lane];
    }
    // ---- flush (lower triangle of S, row-major npad); C/D layout row = kq + 4g, col = rr
    const size_t ld = P.npad;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        if (!tok[t]) continue;
        const int r2 = 16 * tjb[t] + rr;
        if (r2 >= kr) continue;  // column must be a camera dof
        const int g2 = 6 * base + r2;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int r1 = 16 * tib[t] + kq + 4 * g;
            if (r1 < r2 || r1 > er || (rhs_aside && r1 == er)) continue;  // aside: wave 3 owns row er
            const double v = -acc[t][g];
            if (tbuf) {  // deterministic mode: the tile's own slab, summed in tile order by k_schur_gather
                tbuf[(size_t)tile * SCH_TBUF + r1 * SCH_TBUF_LD + r2] = v;
                continue;
            }
            if (r1 < kr) atomicAdd(&S[(size_t)(6 * base + r1) * ld + g2], v);
            else if (r1 < er) atomicAdd(&S[(size_t)(P.kb + r1 - kr) * ld + g2], v);
            else atomicAdd(&rhs[g2], v);
        }
    }
    if (rhs_aside && wave == 3 && lane < kr) {
        const double v = -rhs_acc;
        if (tbuf) tbuf[(size_t)tile * SCH_TBUF + er * SCH_TBUF_LD + lane] = v;
        else atomicAdd(&rhs[6 * base + lane], v);
    }
    if constexpr (FP) {
        // the tile's points: intrinsics terms into S / rhs, gradient max / bad for k_final. Only the point threads
        // (tid < CHUNK_PTS: wave 0) hold any, so wave 0 reduces them alone, without a workgroup barrier
        static_assert(CHUNK_PTS <= 64, "the point threads are wave 0's");
        if (wave == 0) {
            double fp_kk[14];
#pragma unroll
            for (int i = 0; i < 14; ++i) fp_kk[i] = lane < CHUNK_PTS ? kkL[14 * lane + i] : 0.0;
            // (DPP: the fused point side runs in default mode only, never in the deterministic solves whose obs32
            // and f64 instantiations are compared bit for bit)
            wave_sum_dpp<14>(fp_kk);
            fp_gmax = dpp_wave_max(fp_gmax);
            fp_bad = dpp_wave_max(fp_bad);
            if (lane == 0) {
#pragma unroll
                for (int i = 0; i < 14; ++i) zeL[i] = fp_kk[i];  // (zeL is free after the last chunk)
                E.part_w[PART_PT_GMAX * P.part_stride + tile] = fp_gmax;
                E.part_w[PART_PT_BAD * P.part_stride + tile] = fp_bad;
            }
            __builtin_amdgcn_wave_barrier();
            kk_add(P, zeL, S, rhs, true);  // (lanes 0..13)
        }
    }
    if constexpr (STAMP) {
        __syncthreads();
        SCH_STAMP(3);
        if (threadIdx.x == 0)
            for (int k = 0; k < 5; ++k) stamps[(size_t)blockIdx.x * 5 + k] = st_acc[k];
        if constexpr (FP) if (threadIdx.x == 0) {  // phase B on wave 0: after the rhs dot, after the MFMA loop
            for (int k = 0; k < 5; ++k) stamps[(size_t)5 * 256 + 5 * blockIdx.x + k] = sub_st[k];
        }
    }
#undef SCH_STAMP
}
#define SCH_ARGS                                                                                                       \
    DevProblem P, BaConsts c, const LmState *__restrict__ st, const double *__restrict__ scale,                       \
        const double *__restrict__ pdata, double *__restrict__ S, double *__restrict__ rhs,                           \
        unsigned long long *__restrict__ stamps, int nblk_pt, const double *__restrict__ part,                       \
        double *__restrict__ tbuf, EnvArgs E
template <bool STAMP, bool O32, bool PF = false, bool FP = false, bool SW = false>
__global__ __launch_bounds__(TPB) void k_schur_tile(SCH_ARGS) {
    schur_tile_body<STAMP, O32, PF, FP, SW>(P, c, st, scale, pdata, S, rhs, stamps, nblk_pt, part, tbuf, E);
}
// The fused point side on larger windows: held to two workgroups per CU (the LDS allows two; the registers the
// point side adds would otherwise leave one), a few spilled registers in exchange
template <bool O32>
__global__ __launch_bounds__(TPB, 2) void k_schur_tile_fpl(SCH_ARGS) {
    schur_tile_body<false, O32, false, true, false>(P, c, st, scale, pdata, S, rhs, stamps, nblk_pt, part, tbuf, E);
}
#undef SCH_ARGS

// Deterministic mode (ba_options.deterministic): every Schur tile wrote its flush into its own slab
// tbuf[tile] (rows: 6 span camera dofs | 4 intrinsics | rhs; columns: 6 span camera dofs) instead of
// f64 atomics into S. One workgroup per envelope tile of S sums, per element, the slabs of the tiles whose
// camera window covers it, in increasing tile order: bitwise reproducible S / rhs.
// trange[a] = [first tile with base >= a - (TILE_WIN - 1), first tile with base > a) (bases non-decreasing).
__global__ __launch_bounds__(TPB) void k_schur_gather(DevProblem P, const LmState* __restrict__ st,
                                                      const int2* __restrict__ tiles, const double* __restrict__ tbuf,
                                                      const int2* __restrict__ trange, double* __restrict__ S,
                                                      double* __restrict__ rhs) {
    if (skip_step(st)) return;
    const int2 ij = tiles[blockIdx.x];
    const int tid = threadIdx.x;
    const int r = 16 * ij.x + (tid >> 4), col = 16 * ij.y + (tid & 15);
    const int nd = 6 * P.nac, kb = P.kb;
    if (col < nd && col <= r && (r < nd || (r >= kb && r < kb + 4))) {
        const int b = col / 6;
        const bool cam_row = r < nd;
        const int a = cam_row ? r / 6 : b;
        const int t0 = trange[a].x, t1 = trange[b].y;
        double acc = 0.0;
        for (int t = t0; t < t1; ++t) {
            const int bs = P.tile_base[t], sp = P.tile_span[t];
            if (bs > b || bs + sp <= a) continue;
            const int r1 = cam_row ? r - 6 * bs : 6 * sp + (r - kb);
            acc += tbuf[(size_t)t * SCH_TBUF + r1 * SCH_TBUF_LD + (col - 6 * bs)];
        }
        S[(size_t)r * P.npad + col] += acc;
    }
    if (ij.x == ij.y && tid < 16) {
        const int rr = 16 * ij.x + tid;
        if (rr < nd) {
            const int a = rr / 6;
            double acc = 0.0;
            for (int t = trange[a].x; t < trange[a].y; ++t) {
                const int bs = P.tile_base[t], sp = P.tile_span[t];
                if (bs > a || bs + sp <= a) continue;
                acc += tbuf[(size_t)t * SCH_TBUF + (6 * sp + 4) * SCH_TBUF_LD + (rr - 6 * bs)];
            }
            rhs[rr] += acc;
        }
    }
}

// Deterministic overflow Schur terms (k_obs_pairs without atomics): ONE workgroup walks the overflow
// observations in their fixed order; every thread evaluates the (few) Jacobians itself, and each element
// of S / rhs is always updated by the same thread (S camera block element (e2, d) by thread 6 d + e2, rhs
// by 36 + d, border row m by 42 + 4 d + m), so the sums run in program order without barriers or atomics.
// Overflow points (spanning > TILE_WIN cameras or linking a camera twice) are rare; this path is for the
// reproducibility mode, not for speed.
template <bool O32>
__global__ __launch_bounds__(128) void k_obs_pairs_det(DevProblem P, BaConsts c, const LmState* __restrict__ st,
                                                       const double* __restrict__ scale,
                                                       const double* __restrict__ pdata, double* __restrict__ S,
                                                       double* __restrict__ rhs) {
    if (skip_step(st)) return;
    const int cur = st->cur;
    const int tid = threadIdx.x;
    const size_t ld = P.npad;
    const int kb = P.kb;
    const double* K = P.K[cur];
    auto wt = [&](int q, int ca, const double* sp, const double* X, double W[18]) {
        const ObsRaw<O32> o = po_obs<O32>(P, q);
        ObsEval ev;
        double jc[18], jp[9], jk[8];
        lin_obs(c, P.cams[cur] + 7 * o.idx(), X, K, o.u(), o.v(), o.d(), ev, jc, jp, jk);
        w_tilde(jc, jp, scale + 6 * ca, sp, W);
    };
    for (int i = 0; i < P.n_ovf_obs; ++i) {
        const int a = P.ovf_obs[i];
        const int ca = P.po_ac[a];
        if (ca < 0) continue;
        const int ap = P.po_ap[a];
        const double* pd = pdata + (size_t)ap * PDATA;
        const double* sp = scale + P.off_pt + 3 * ap;
        const double* X = P.pts[cur] + 3 * P.pt_idx[ap];
        double Vf[9], Wa[18], Y[18];
        vinv_from_g(pd, Vf);
        wt(a, ca, sp, X, Wa);
#pragma unroll
        for (int d = 0; d < 6; ++d)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                Y[d * 3 + j] = Wa[d * 3 + 0] * Vf[0 * 3 + j] + Wa[d * 3 + 1] * Vf[1 * 3 + j] + Wa[d * 3 + 2] * Vf[2 * 3 + j];
        if (tid >= 36 && tid < 42) {
            const int d = tid - 36;
            rhs[6 * ca + d] -= Y[d * 3 + 0] * pd[6] + Y[d * 3 + 1] * pd[7] + Y[d * 3 + 2] * pd[8];
        } else if (tid >= 42 && tid < 66) {
            const int d = (tid - 42) >> 2, m = (tid - 42) & 3;
            S[(size_t)(kb + m) * ld + 6 * ca + d] -=
                Y[d * 3 + 0] * pd[9 + m * 3 + 0] + Y[d * 3 + 1] * pd[9 + m * 3 + 1] + Y[d * 3 + 2] * pd[9 + m * 3 + 2];
        }
        for (int b = P.pt_ptr[ap]; b < P.pt_ptr[ap + 1]; ++b) {
            const int cb = P.po_ac[b];
            if (cb < ca || (cb == ca && b < a) || tid >= 36) continue;
            double W[18];
            wt(b, cb, sp, X, W);
            const int d = tid / 6, e2 = tid % 6;
            if (cb > ca) {
                S[(size_t)(6 * cb + e2) * ld + 6 * ca + d] -=
                    Y[d * 3 + 0] * W[e2 * 3 + 0] + Y[d * 3 + 1] * W[e2 * 3 + 1] + Y[d * 3 + 2] * W[e2 * 3 + 2];
            } else if (e2 >= d) {
                double m = Y[d * 3 + 0] * W[e2 * 3 + 0] + Y[d * 3 + 1] * W[e2 * 3 + 1] + Y[d * 3 + 2] * W[e2 * 3 + 2];
                if (b != a) m += Y[e2 * 3 + 0] * W[d * 3 + 0] + Y[e2 * 3 + 1] * W[d * 3 + 1] + Y[e2 * 3 + 2] * W[d * 3 + 2];
                S[(size_t)(6 * ca + e2) * ld + 6 * ca + d] -= m;
            }
        }
    }
}

// ---------------------------------------------------------------- Cholesky
// Envelope-blocked right-looking Cholesky of the npad x npad reduced system
// (lower triangle, row-major), then L z = b, L^T y = z (y overwrites b).
// One workgroup (4 waves). fcol[i]: first non-zero 16-block column of block row i;
// rows[rptr[k]..rptr[k+1]): block rows i > k with fcol[i] <= k.

__global__ __launch_bounds__(TPB) void k_chol(const LmState* __restrict__ st, double* __restrict__ A, int npad, int nb,
                                              const int* __restrict__ fcol,
                                              const int* __restrict__ rptr, const int* __restrict__ rows,
                                              double* __restrict__ b, int* __restrict__ flag) {
    if (skip_step(st)) return;
    __shared__ double Lkk[16][17];
    __shared__ double red[16][17];
    __shared__ int s_bad;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const size_t ld = npad;
    if (tid == 0) s_bad = 0;
    __syncthreads();
    for (int kb = 0; kb < nb; ++kb) {
        const size_t k0 = (size_t)kb * 16;
        // ---- potrf of the 16x16 diagonal tile, wave 0, lane r holds row r
        if (wave == 0) {
            double a[16];
            const int r = lane & 15;
#pragma unroll
            for (int j = 0; j < 16; ++j) a[j] = (j <= r) ? A[(k0 + r) * ld + k0 + j] : 0.0;
            bool bad = false;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                double djj = __shfl(a[j], j);
                if (!(djj > 0.0) || !isfinite(djj)) { bad = true; djj = 1.0; }
                const double d = sqrt(djj);
                double lrj = (r == j) ? d : (r > j ? a[j] / d : 0.0);
                a[j] = lrj;
#pragma unroll
                for (int k = j + 1; k < 16; ++k) {
                    const double lkj = __shfl(lrj, k);
                    if (r >= k) a[k] -= lrj * lkj;
                }
            }
            if (lane < 16) {
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    Lkk[r][j] = (j <= r) ? a[j] : 0.0;
                    if (j <= r) A[(k0 + r) * ld + k0 + j] = a[j];
                }
            }
            if (bad && lane == 0) s_bad = 1;
        }
        __syncthreads();
        const int r0 = rptr[kb], r1 = rptr[kb + 1];
        const int nr = r1 - r0;
        // ---- TRSM: L_ik = A_ik L_kk^{-T}, thread per row
        for (int t = tid; t < nr * 16; t += TPB) {
            const int i = rows[r0 + (t >> 4)];
            const int r = t & 15;
            double* row = A + ((size_t)i * 16 + r) * ld + k0;
            double x[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) x[j] = row[j];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                double s = x[j];
#pragma unroll
                for (int m = 0; m < j; ++m) s -= x[m] * Lkk[j][m];
                x[j] = s / Lkk[j][j];
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) row[j] = x[j];
        }
        __syncthreads();
        // ---- trailing update A_ij -= L_ik L_jk^T over tiles (p >= q) of the row list, MFMA f64
        const int ntiles = nr * (nr + 1) / 2;
        for (int t = wave; t < ntiles; t += 4) {
            // map t -> (p, q), q <= p
            int p = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
            while ((p + 1) * (p + 2) / 2 <= t) ++p;
            while (p * (p + 1) / 2 > t) --p;
            const int q = t - p * (p + 1) / 2;
            const int i = rows[r0 + p], j = rows[r0 + q];
            const double* Li = A + ((size_t)i * 16) * ld + k0;
            const double* Lj = A + ((size_t)j * 16) * ld + k0;
            d4 acc = {0.0, 0.0, 0.0, 0.0};
            const int rr = lane & 15, kk = lane >> 4;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const double av = Li[(size_t)rr * ld + 4 * s + kk];  // A[i=rr][k]
                const double bv = Lj[(size_t)rr * ld + 4 * s + kk];  // B[k][j=rr] = L_jk[rr][k]
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
            }
            double* Cij = A + ((size_t)i * 16) * ld + (size_t)j * 16;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int row = kk + 4 * g, col = rr;  // f64 C/D map: row = (lane>>4) + 4*reg
                Cij[(size_t)row * ld + col] -= acc[g];
            }
        }
        __syncthreads();
    }
    // ---- forward solve L z = b
    for (int i = 0; i < nb; ++i) {
        const int r = tid & 15, p = tid >> 4;  // 16 rows x 16 parts
        double s = 0.0;
        const size_t row = (size_t)i * 16 + r;
        for (int col = fcol[i] * 16 + p; col < i * 16; col += 16) s += A[row * ld + col] * b[col];
        red[p][r] = s;
        __syncthreads();
        if (wave == 0) {
            const int rr = lane & 15;
            double v = b[(size_t)i * 16 + rr];
#pragma unroll
            for (int q = 0; q < 16; ++q) v -= red[q][rr];
            // L_ii z = v, lane rr owns row rr
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const double lmm = A[((size_t)i * 16 + m) * ld + (size_t)i * 16 + m];
                double zm = __shfl(v, m) / lmm;
                if (rr > m) v -= A[((size_t)i * 16 + rr) * ld + (size_t)i * 16 + m] * zm;
                if (rr == m) v = zm;
            }
            if (lane < 16) b[(size_t)i * 16 + rr] = v;
        }
        __syncthreads();
    }
    // ---- backward solve L^T y = z
    for (int i = nb - 1; i >= 0; --i) {
        const int r = tid & 15, p = tid >> 4;
        double s = 0.0;
        const int r0 = rptr[i], r1 = rptr[i + 1];
        for (int t = r0; t < r1; ++t) {
            const int j = rows[t];
            // sum_c L[16j + c][16i + r] y[16j + c], c split over parts p
            const size_t rowj = (size_t)j * 16 + p;
            s += A[rowj * ld + (size_t)i * 16 + r] * b[rowj];
        }
        red[p][r] = s;
        __syncthreads();
        if (wave == 0) {
            const int rr = lane & 15;
            double v = b[(size_t)i * 16 + rr];
#pragma unroll
            for (int q = 0; q < 16; ++q) v -= red[q][rr];
            // L_ii^T y = v : y_m for m = 15..0 ; (L^T)[rr][m] = L[m][rr]
#pragma unroll
            for (int m = 15; m >= 0; --m) {
                const double lmm = A[((size_t)i * 16 + m) * ld + (size_t)i * 16 + m];
                double ym = __shfl(v, m) / lmm;
                if (rr < m) v -= A[((size_t)i * 16 + m) * ld + (size_t)i * 16 + rr] * ym;
                if (rr == m) v = ym;
            }
            if (lane < 16) b[(size_t)i * 16 + rr] = v;
        }
        __syncthreads();
    }
    if (tid == 0 && s_bad) *flag = 1;
}

// ---------------------------------------------------------------- banded Cholesky
// Reduced camera systems of sequential keyframe windows are block-banded
// (co-visibility of nearby keyframes) plus a dense border (the intrinsics block
// couples every camera: the last 16-row block). k_chol_band factors such a
// matrix (band of W 16x16 tiles below the diagonal) in ONE workgroup with the
// active band in LDS: a ring of W+1 block columns x (W+1 band tiles + 1 border
// tile). Column k+W+1 is prefetched into registers while column k is factored;
// the forward substitution L z = b is fused into the factorization and the
// backward solve L^T y = z streams the factor back with one column of prefetch.
// Trailing tile updates use v_mfma_f64_16x16x4_f64. Tiles are stored with an
// 18-double row stride (bank-conflict-free MFMA operand reads).
static constexpr int TLD = 18;          // LDS row stride of a 16x16 tile
static constexpr int TSZ = 16 * TLD;    // doubles per LDS tile
template <int W>
struct BandLds {
    static constexpr int TPS = W + 2;                 // tiles per ring slot (W+1 band + border)
    static constexpr int NT = (W + 1) * TPS + 2;      // + last diagonal tile + backward diagonal tile
    double tiles[NT][TSZ];
    double bring[W + 1][16];                          // rhs ring (band rows)
    double blast[16];                                 // rhs of the last block row
    double rdiag[16];
    double red[16][17];
};
static constexpr int BAND_MAX_NB = 2048;                // fcol staged in LDS (nb <= 2048)



template <int W, bool STAMP>
__global__ __launch_bounds__(TPB) void k_chol_band(const LmState* __restrict__ st, double* __restrict__ A, int npad, int nb,
                                                   const int* __restrict__ fcol,
                                                   double* __restrict__ b, int* __restrict__ flag,
                                                   unsigned long long* __restrict__ stamps) {
    if (skip_step(st)) return;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    BandLds<W>& L = *reinterpret_cast<BandLds<W>*>(smem);
    int* fc_s = reinterpret_cast<int*>(smem + sizeof(BandLds<W>));
    constexpr int TPS = BandLds<W>::TPS;
    unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0};
    unsigned long long t_prev = 0;
#define STAMP_AT(idx)                                  \
    if constexpr (STAMP) {                             \
        const unsigned long long t_ = stamp_now();    \
        st_acc[idx] += t_ - t_prev;                   \
        t_prev = t_;                                  \
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const size_t ld = npad;
    const int last = nb - 1;
    const int nbb = nb - 1;  // band block columns 0..nb-2
    for (int i = tid; i < nb; i += TPB) fc_s[i] = fcol[i];
    bool bad = false;
    // tile addressing: slot(j) = j % (W+1); band tile (i,j) at offset i-j, border (last,j) at W+1
    double* lastdiag = L.tiles[(W + 1) * TPS];
    double* bwdiag = L.tiles[(W + 1) * TPS + 1];
    const int er = tid >> 4, ec = tid & 15;  // element of a tile handled by this thread (copy loops)
    // ---- initial fill: columns 0..W, last diagonal tile, rhs
    for (int j = 0; j <= W; ++j) {
        const int sj = j % (W + 1);
        for (int bti = 0; bti < TPS; ++bti) {
            const int i = (bti == W + 1) ? last : j + bti;
            const bool ok = (j < nbb) && ((bti == W + 1) || (i < last));
            L.tiles[sj * TPS + bti][er * TLD + ec] = ok ? A[((size_t)i * 16 + er) * ld + (size_t)j * 16 + ec] : 0.0;
        }
        if (tid < 16) L.bring[sj][tid] = (j < nbb) ? b[(size_t)j * 16 + tid] : 0.0;
    }
    lastdiag[er * TLD + ec] = A[((size_t)last * 16 + er) * ld + (size_t)last * 16 + ec];
    if (tid < 16) L.blast[tid] = b[(size_t)last * 16 + tid];
    __syncthreads();
    if constexpr (STAMP) t_prev = stamp_now();
    // wave-0 helper: factor the diagonal tile held in `colk` (rows in registers), write it back,
    // and run the forward step z = L^-1 z on the rhs block `bz`.
    auto factor_diag = [&](double* Tk, double* bz) {
        const int r = lane & 15;
        double a[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) a[j] = (j <= r) ? Tk[r * TLD + j] : 0.0;
        potrf16_regs(a, L.rdiag, lane, bad);
        if (lane < 16)
#pragma unroll
            for (int j = 0; j < 16; ++j) Tk[r * TLD + j] = (j <= r) ? a[j] : 0.0;
        double v = bz[r];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const double zm = bcast(v, m) * L.rdiag[m];
            if (r > m) v -= a[m] * zm;
            if (r == m) v = zm;
        }
        if (lane < 16) bz[r] = v;
    };
    // prologue: factor tile (0,0)
    if (nbb > 0 && wave == 0) factor_diag(L.tiles[0], L.bring[0]);
    __syncthreads();
    for (int k = 0; k < nbb; ++k) {
        const int sk = k % (W + 1);
        double* colk = L.tiles[sk * TPS];
        const int kn = k + W + 1;
        // ---- prefetch column kn into registers
        double pre[TPS];
        double preb = 0.0;
#pragma unroll
        for (int bti = 0; bti < TPS; ++bti) {
            const int i = (bti == W + 1) ? last : kn + bti;
            const bool ok = (kn < nbb) && ((bti == W + 1) || (i < last));
            pre[bti] = ok ? A[((size_t)i * 16 + er) * ld + (size_t)kn * 16 + ec] : 0.0;
        }
        if (tid < 16 && kn < nbb) preb = b[(size_t)kn * 16 + tid];
        const int wk = min(W, last - 1 - k);  // band rows k+1..k+wk (fcol <= k), then the border
        STAMP_AT(0)
        // ---- 1. TRSM: L_ik = A_ik L_kk^-T (tile (k,k) factored by the previous look-ahead)
        if (tid < (W + 1) * 16) {
            const int bt = (tid >> 4) + 1;  // 1..W+1
            const int r = tid & 15;
            const bool border = (bt == W + 1);
            const int i = border ? last : k + bt;
            const bool act = border || (bt <= wk && fc_s[i] <= k);
            if (act) {
                double* T = L.tiles[sk * TPS + bt];
                double x[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) x[j] = T[r * TLD + j];
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    x[m] *= L.rdiag[m];
#pragma unroll
                    for (int j = m + 1; j < 16; ++j) x[j] -= x[m] * colk[j * TLD + m];
                }
#pragma unroll
                for (int j = 0; j < 16; ++j) T[r * TLD + j] = x[j];
            }
        }
        __syncthreads();
        STAMP_AT(1)
        // ---- 2. trailing update. Wave 0: look-ahead on block column k+1 (update + factor the
        //         diagonal tile (k+1,k+1), rhs of row k+1); waves 1..3: every other tile and rhs row.
        {
            const int nr = wk + 1;  // items: 0..wk-1 band rows k+1+idx, wk = border
            const int npairs = nr * (nr + 1) / 2;
            const bool la = (wk >= 1);  // look-ahead exists (band row k+1 < last)
            const int rr = lane & 15, kk = lane >> 4;
            auto tile_of = [&](int it) -> double* { return L.tiles[sk * TPS + ((it == wk) ? W + 1 : 1 + it)]; };
            if (wave == 0) {
                if (la) {
                    const int i1 = k + 1;
                    double* T11 = L.tiles[(i1 % (W + 1)) * TPS];
                    if (fc_s[i1] <= k) {
                        const double* Li = tile_of(0);
                        d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                        for (int s4 = 0; s4 < 4; ++s4)
                            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Li[rr * TLD + 4 * s4 + kk], Li[rr * TLD + 4 * s4 + kk],
                                                                      acc, 0, 0, 0);
#pragma unroll
                        for (int g = 0; g < 4; ++g) T11[(kk + 4 * g) * TLD + rr] -= acc[g];
                        // rhs row k+1
                        const int r = lane & 15, part = lane >> 4;
                        double sacc = 0.0;
#pragma unroll
                        for (int c = 0; c < 4; ++c) sacc += Li[r * TLD + part * 4 + c] * L.bring[sk][part * 4 + c];
                        sacc += __shfl_xor(sacc, 16);
                        sacc += __shfl_xor(sacc, 32);
                        if (lane < 16) L.bring[i1 % (W + 1)][lane] -= sacc;
                    }
                    factor_diag(T11, L.bring[i1 % (W + 1)]);
                }
            } else {
                constexpr int MAXU = ((W + 2) * (W + 1) / 2 + 2) / 3;
                d4 acc[MAXU];
                double* dst[MAXU];
#pragma unroll
                for (int u = 0; u < MAXU; ++u) {
                    acc[u] = d4{0.0, 0.0, 0.0, 0.0};
                    dst[u] = nullptr;
                    const int t = (wave - 1) + 3 * u + (la ? 1 : 0);  // skip pair 0 = (k+1,k+1) under look-ahead
                    if (t < npairs) {
                        int p = 0, rem = t;
                        while (rem > p) { rem -= p + 1; ++p; }
                        const int q = rem;
                        const int ip = (p == wk) ? last : k + 1 + p;
                        const int iq = (q == wk) ? last : k + 1 + q;
                        if ((ip == last || fc_s[ip] <= k) && (iq == last || fc_s[iq] <= k)) {
                            const double* Li = tile_of(p);
                            const double* Lj = tile_of(q);
                            dst[u] = (ip == last && iq == last)
                                         ? lastdiag
                                         : (ip == last ? L.tiles[(iq % (W + 1)) * TPS + W + 1]
                                                       : L.tiles[(iq % (W + 1)) * TPS + (ip - iq)]);
#pragma unroll
                            for (int s4 = 0; s4 < 4; ++s4)
                                acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(Li[rr * TLD + 4 * s4 + kk],
                                                                              Lj[rr * TLD + 4 * s4 + kk], acc[u], 0, 0, 0);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < MAXU; ++u)
                    if (dst[u])
#pragma unroll
                        for (int g = 0; g < 4; ++g) dst[u][(kk + 4 * g) * TLD + rr] -= acc[u][g];
                // rhs rows other than k+1
                for (int it = (la ? 1 : 0) + (wave - 1); it < nr; it += 3) {
                    const int i = (it == wk) ? last : k + 1 + it;
                    if (i != last && fc_s[i] > k) continue;
                    const double* Li = tile_of(it);
                    const int r = lane & 15, part = lane >> 4;
                    double sacc = 0.0;
#pragma unroll
                    for (int c = 0; c < 4; ++c) sacc += Li[r * TLD + part * 4 + c] * L.bring[sk][part * 4 + c];
                    sacc += __shfl_xor(sacc, 16);
                    sacc += __shfl_xor(sacc, 32);
                    if (lane < 16) {
                        if (it == wk) L.blast[lane] -= sacc; else L.bring[i % (W + 1)][lane] -= sacc;
                    }
                }
            }
        }
        __syncthreads();
        STAMP_AT(2)
        // ---- 3. retire column k to global (L and z), install the prefetched column kn
        for (int bti = 0; bti <= wk; ++bti) {
            const int i = k + bti;
            A[((size_t)i * 16 + er) * ld + (size_t)k * 16 + ec] = L.tiles[sk * TPS + bti][er * TLD + ec];
        }
        A[((size_t)last * 16 + er) * ld + (size_t)k * 16 + ec] = L.tiles[sk * TPS + W + 1][er * TLD + ec];
        if (tid < 16) b[(size_t)k * 16 + tid] = L.bring[sk][tid];
        __syncthreads();
#pragma unroll
        for (int bti = 0; bti < TPS; ++bti) L.tiles[sk * TPS + bti][er * TLD + ec] = pre[bti];
        if (tid < 16) L.bring[sk][tid] = preb;
        __syncthreads();
        STAMP_AT(3)
    }
    // ---- last diagonal tile: factor, forward and backward step
    if (wave == 0) {
        const int r = lane & 15;
        double a[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) a[j] = (j <= r) ? lastdiag[r * TLD + j] : 0.0;
        potrf16_regs(a, L.rdiag, lane, bad);
        double v = L.blast[r];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const double zm = bcast(v, m) * L.rdiag[m];
            if (r > m) v -= a[m] * zm;
            if (r == m) v = zm;
        }
        // y = L^-T z : (L^T)[r][m] = L[m][r] = lane m's a[r]
#pragma unroll
        for (int m = 15; m >= 0; --m) {
            const double ym = bcast(v, m) * L.rdiag[m];
            double lmr = 0.0;
#pragma unroll
            for (int q = 0; q < 16; ++q)
                if (q == r) lmr = bcast(a[q], m);  // L[m][r]
            if (r < m) v -= lmr * ym;
            if (r == m) v = ym;
        }
        if (lane < 16) {
            L.blast[r] = v;
            b[(size_t)last * 16 + r] = v;
#pragma unroll
            for (int j = 0; j < 16; ++j) A[((size_t)last * 16 + r) * ld + (size_t)last * 16 + j] = (j <= r) ? a[j] : 0.0;
        }
    }
    __syncthreads();
    // ---- backward solve over band columns k = nb-2 .. 0 ; y ring in L.bring, y_last in L.blast
    {
        const int r = tid & 15, p = tid >> 4;
        double cur[W + 1], nxt[W + 1];
        double dg_cur = 0.0, dg_nxt = 0.0, zk_cur = 0.0, zk_nxt = 0.0;
        auto load_col = [&](int k, double* v, double& dg, double& zk) {
#pragma unroll
            for (int it = 0; it <= W; ++it) {
                const int i = (it == W) ? last : k + 1 + it;
                const bool ok = (k >= 0) && ((it == W) || (i < last));
                v[it] = ok ? A[((size_t)i * 16 + p) * ld + (size_t)k * 16 + r] : 0.0;
            }
            dg = (k >= 0) ? A[((size_t)k * 16 + p) * ld + (size_t)k * 16 + r] : 0.0;
            zk = (k >= 0 && tid < 16) ? b[(size_t)k * 16 + tid] : 0.0;
        };
        load_col(nbb - 1, cur, dg_cur, zk_cur);
        for (int k = nbb - 1; k >= 0; --k) {
            load_col(k - 1, nxt, dg_nxt, zk_nxt);
            const int wk = min(W, last - 1 - k);
            double sacc = 0.0;
#pragma unroll
            for (int it = 0; it <= W; ++it) {
                const bool border = (it == W);
                const int i = border ? last : k + 1 + it;
                const bool act = border || (it < wk && fc_s[i] <= k);
                if (act) sacc += cur[it] * (border ? L.blast[p] : L.bring[i % (W + 1)][p]);
            }
            L.red[p][r] = sacc;
            bwdiag[p * TLD + r] = dg_cur;
            if (p == r) L.rdiag[r] = 1.0 / dg_cur;
            __syncthreads();
            if (wave == 0) {
                const int rr = lane & 15;
                double v = __shfl(zk_cur, rr);
#pragma unroll
                for (int q = 0; q < 16; ++q) v -= L.red[q][rr];
                // y_k = L_kk^-T v ; (L^T)[rr][m] = L[m][rr]
#pragma unroll
                for (int m = 15; m >= 0; --m) {
                    const double ym = bcast(v, m) * L.rdiag[m];
                    if (rr < m) v -= bwdiag[m * TLD + rr] * ym;
                    if (rr == m) v = ym;
                }
                if (lane < 16) {
                    L.bring[k % (W + 1)][lane] = v;
                    b[(size_t)k * 16 + lane] = v;
                }
            }
            __syncthreads();
#pragma unroll
            for (int it = 0; it <= W; ++it) cur[it] = nxt[it];
            dg_cur = dg_nxt;
            zk_cur = zk_nxt;
        }
    }
    STAMP_AT(4)
    if constexpr (STAMP) {
        if (tid == 0)
            for (int i = 0; i < 5; ++i) stamps[i] = st_acc[i];
    }
#undef STAMP_AT
    if (bad) *flag = 1;
}

// ---------------------------------------------------------------- update
// delta = -s * y over cameras and intrinsics; candidate poses; the camera / intrinsics terms of the
// model cost change and the candidate prior cost. part[PART_UPD_* * stride + block]
// Model cost change (Ceres ComputeTrustRegionStep: -(J d)^T (f + J d / 2)) from the normal equations:
// in scaled coordinates the step z = -y solves (A~ + D~) z = -g~ exactly (A~ = J~^T J~, g~ = J~^T f,
// D~ the LM diagonal; the Schur solve is exact), so -(J~ z)^T (f + J~ z / 2) = 0.5 (g~^T y + y^T D~ y):
// a sum of per-parameter terms (cameras and intrinsics here, points in k_backsub_chunk) that needs no
// second Jacobian evaluation per observation. g~ and D~ are the values k_env_assemble / k_point_prep
// put into the system, element for element.
__global__ void k_update_cams(DevProblem P, BaConsts c, const LmState* __restrict__ st, const double* __restrict__ scale,
                              const double* __restrict__ camdata, const double* __restrict__ lin,
                              const double* __restrict__ y, double* __restrict__ delta, double* __restrict__ part) {
    __shared__ double lds[4 * 4];
    __shared__ double out[4];
    if (skip_step(st)) return;
    const int cur = st->cur;
    const double radius = st->radius;
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};  // sn2, mcc, cand cost, |x_cand|^2
    if (t < P.nac)
        update_camera(P, c, cur, radius, scale, camdata, t, y + 6 * t, delta, acc);
    else if (t == P.nac)
        update_intrinsics(P, c, cur, radius, scale, lin, y + P.kb, delta, acc);
    block_sum<4>(acc, lds, out);
    if (threadIdx.x == 0) {
        part[PART_UPD_SN2 * P.part_stride + blockIdx.x] = out[0];
        part[PART_UPD_MCC * P.part_stride + blockIdx.x] = out[1];
        part[PART_UPD_COST * P.part_stride + blockIdx.x] = out[2];
        part[PART_UPD_XN2 * P.part_stride + blockIdx.x] = out[3];
    }
}

// Back-substitution over a chunk of points (backsub_body, ba_tail.h): one workgroup per chunk.
template <bool O32>
__global__ __launch_bounds__(TPB) void k_backsub_chunk(DevProblem P, BaConsts c, const LmState* __restrict__ st,
                                                       const double* __restrict__ scale,
                                                       const double* __restrict__ pdata, const double* __restrict__ y,
                                                       const double* __restrict__ delta, double* __restrict__ part,
                                                       const int2* __restrict__ ztiles, int n_ztiles,
                                                       double* __restrict__ Sz) {
    __shared__ BsLds L;
    backsub_body<O32>(P, c, st, scale, pdata, y, delta, part, ztiles, n_ztiles, Sz, blockIdx.x, gridDim.x, L);
}

// Clear the envelope tiles of S (every solver reads only these; the rest stays zero).
__global__ __launch_bounds__(TPB) void k_env_zero(const LmState* __restrict__ st, const int2* __restrict__ tiles, int npad,
                                                  double* __restrict__ S) {
    if (skip_step(st)) return;
    const int2 ij = tiles[blockIdx.x];
    S[(size_t)(16 * ij.x + (threadIdx.x >> 4)) * npad + 16 * ij.y + (threadIdx.x & 15)] = 0.0;
}

// ---------------------------------------------------------------- envelope clear + assembly
// One workgroup per envelope tile of S (16x16, one element per thread): every element is
// written once — the camera blocks s U s + D^2 (lower), the border s C s_k, the intrinsics
// block and the pad identity (rank 0; the landmark shards of other ranks contribute zeros),
// zero elsewhere — and the diagonal tiles write their 16 rows of rhs. Replaces k_env_zero +
// k_assemble + the chol_flag memset (same values as k_assemble, element for element).

// ---------------------------------------------------------------- final
// The deterministic reduction of the per-block partials + the LM decision (final_body, ba_tail.h).
template <int UNR>
__global__ __launch_bounds__(TPB_F) void k_final(DevProblem P, LmState* __restrict__ st, int nblk_pt, int nblk_upd,
                                               int nblk_bs, const double* __restrict__ part,
                                               const int* __restrict__ chol_flag, double* __restrict__ scal,
                                               LmParams prm, const double* __restrict__ lin, double* __restrict__ log,
                                               double* __restrict__ rhs_z, unsigned* __restrict__ bcr_epoch) {
    __shared__ FinLds L;
    final_body<UNR>(P, st, nblk_pt, nblk_upd, nblk_bs, part, chol_flag, scal, prm, lin, log, rhs_z, bcr_epoch, L);
}

// ---------------------------------------------------------------- landmark sharding
// Envelope of S (its 16x16 tiles) + rhs (+ camera / intrinsics sums) <-> one contiguous buffer for the
// all-reduce. unpack == 0: S, rhs, cam -> buf; unpack == 1: buf -> S, rhs. Workgroups < n_env move one tile
// each; the rest move the tail [rhs | cam] one element per thread (env_tail_blocks of them), so no workgroup
// walks a long serial copy.
__host__ __device__ inline int env_tail_blocks(int npad, int ncam) { return (npad + ncam + TPB - 1) / TPB; }
__global__ __launch_bounds__(TPB) void k_env_pack(const LmState* __restrict__ st, const int2* __restrict__ tiles, int n_env,
                                                  int npad, double* __restrict__ S, double* __restrict__ rhs,
                                                  double* __restrict__ buf, int unpack, const double* __restrict__ cam,
                                                  int ncam) {
    const int t = blockIdx.x;
    if (t < n_env) {
        if (skip_step(st)) return;
        const int2 ij = tiles[t];
        const int r = threadIdx.x >> 4, cc = threadIdx.x & 15;
        double* sp = S + (size_t)(16 * ij.x + r) * npad + 16 * ij.y + cc;
        double* bp = buf + (size_t)t * 256 + threadIdx.x;
        if (unpack) *sp = *bp; else *bp = *sp;
        return;
    }
    const int j = (t - n_env) * TPB + threadIdx.x;
    double* bp = buf + (size_t)n_env * 256 + j;
    if (j < npad) {
        if (skip_step(st)) return;
        if (unpack) rhs[j] = *bp; else *bp = rhs[j];
    } else if (j < npad + ncam) {  // folded exchange: this rank's camera-side and intrinsics sums (also when stop_next)
        if (st->done) return;
        *bp = cam[j - npad];
    }
}
// Folded exchange, after the all-reduce (landmark shards, fused LM loop): buf = [envelope tiles | rhs | camera
// sums (nac x CAMDATA) | intrinsics sums (SEGINTR)], each summed over the ranks. Workgroups < n_env: S tiles,
// plus the LM diagonal of the camera / intrinsics dofs and the IntrinsicsPrior diagonal (from the reduced camera
// and intrinsics sums: env_tile's rank-0 formulas); the next env_tail_blocks: rhs plus the prior's gradient and
// the camdata copy, one element per thread; the last: lin (cost, gradient max-norm, prior-augmented intrinsics
// block) for the step kernels and the decision.
__global__ __launch_bounds__(TPB) void k_env_unpack_fin(DevProblem P, BaConsts c, const LmState* __restrict__ st,
                                                        const int2* __restrict__ tiles, int n_env,
                                                        const double* __restrict__ buf, const double* __restrict__ scale,
                                                        double* __restrict__ S, double* __restrict__ rhs,
                                                        double* __restrict__ camdata, double* __restrict__ lin) {
    __shared__ double red[4];
    __shared__ double l16[LIN_N];
    const int t = blockIdx.x, tid = threadIdx.x;
    const int npad = P.npad, nd = 6 * P.nac, kb = P.kb;
    const double* cdg = buf + (size_t)n_env * 256 + npad;
    const double* iog = cdg + (size_t)P.nac * CAMDATA;
    const double* sk = scale + P.off_k;
    const double wk = c.sw_k * c.sw_k;
    const int ntail = env_tail_blocks(npad, P.nac * CAMDATA);
    if (t < n_env) {
        if (skip_step(st)) return;
        const int2 ij = tiles[t];
        const int r = 16 * ij.x + (tid >> 4), col = 16 * ij.y + (tid & 15);
        double v = buf[(size_t)t * 256 + tid];
        if (r == col) {
            const double radius = st->radius;
            if (r < nd) {
                const int ac = r / 6, i = r - 6 * ac;
                const double u = scale[r] * cdg[(size_t)ac * CAMDATA + 6 * i - i * (i - 1) / 2] * scale[r];
                v += fmin(fmax(u, c.min_diag), c.max_diag) / radius;
            } else if (r < kb + 4) {
                const int m = r - kb;
                const double u = sk[m] * (iog[4 * m - m * (m - 1) / 2] + wk) * sk[m];
                v += sk[m] * wk * sk[m] + fmin(fmax(u, c.min_diag), c.max_diag) / radius;
            }
        }
        S[(size_t)r * npad + col] = v;
    } else if (t < n_env + ntail) {
        const int j = (t - n_env) * TPB + tid;
        if (j < npad) {
            if (skip_step(st)) return;
            double b = buf[(size_t)n_env * 256 + j];
            if (j >= kb && j < kb + 4) {
                const int m = j - kb;
                b += sk[m] * (-c.sw_k) * (c.sw_k * (P.prior[m] - P.K[st->cur][m]));
            }
            rhs[j] = b;
        } else if (j < npad + P.nac * CAMDATA) {
            if (st->done) return;
            camdata[j - npad] = cdg[j - npad];
        }
    } else {
        if (st->done) return;
        const int cur = st->cur;
        double gm = 0.0;
        for (int ac = tid; ac < P.nac; ac += TPB) gm = fmax(gm, cam_gmax(P, cur, ac, cdg + (size_t)ac * CAMDATA + 45));
        gm = block_max(gm, red);
        if (tid == 0) {
            const double gi = intr_lin(P, c, P.K[cur], iog, l16);
            lin[0] = l16[0];
            lin[1] = fmax(gm, gi);
            for (int q = 2; q < LIN_N; ++q) lin[q] = l16[q];
        }
    }
}

// Sharded k_final: this rank's point-side sums / maxima and the (replicated) camera-side
// sums go to red[] for the all-reduce; k_combine assembles scal[] from the reduced values.
template <int UNR>
__global__ __launch_bounds__(TPB_F) void k_final_shard(DevProblem P, const LmState* __restrict__ st, int nblk_pt,
                                                       int nblk_upd, int nblk_bs, const double* __restrict__ part,
                                                       const int* __restrict__ chol_flag, double* __restrict__ red,
                                                       double* __restrict__ rhs_z, int nranks,
                                                       unsigned* __restrict__ bcr_epoch) {
    __shared__ double lds[NW_F * 8];
    __shared__ double out[8];
    __shared__ double rl[NW_F];
    // k_final's shape: every load up front, one memory round trip before the reductions
    const int cf = *chol_flag;
    const int done = __builtin_amdgcn_readfirstlane(st->done);
    double acc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};  // 0..3 local, 4..7 replicated
    double gm = 0.0, bad = 0.0;
    const size_t stp = P.part_stride;
#pragma unroll UNR
    for (int i = threadIdx.x; i < nblk_upd; i += TPB_F) {
        acc[4] += part[PART_UPD_SN2 * stp + i];
        acc[5] += part[PART_UPD_MCC * stp + i];
        acc[6] += part[PART_UPD_COST * stp + i];
        acc[7] += part[PART_UPD_XN2 * stp + i];
    }
#pragma unroll UNR
    for (int i = threadIdx.x; i < nblk_bs; i += TPB_F) {
        acc[0] += part[PART_BS_SN2 * stp + i];
        acc[1] += part[PART_BS_MCC * stp + i];
        acc[2] += part[PART_BS_COST * stp + i];
        acc[3] += part[PART_BS_XN2 * stp + i];
        bad = fmax(bad, part[PART_BS_BAD * stp + i]);
    }
#pragma unroll UNR
    for (int i = threadIdx.x; i < nblk_pt; i += TPB_F) {
        gm = fmax(gm, part[PART_PT_GMAX * stp + i]);
        bad = fmax(bad, 2.0 * part[PART_PT_BAD * stp + i]);
    }
    if (done) return;
    if (bcr_epoch && threadIdx.x == 0 && !st->stop_next) *bcr_epoch += 1;  // as in k_final
    if (rhs_z)  // fused path: y has been consumed; rhs is the next local assembly's atomic target
        for (int i = threadIdx.x; i < P.npad; i += TPB_F) rhs_z[i] = 0.0;
    // one SUM all-reduce carries both the sums and the maxima: each rank writes its two maxima into its own
    // slot pair of red[RED_X + 4 ...] and zeros into the others' (x + 0 is exact), k_combine takes the max
    double* x = red + RED_X;
    for (int i = 4 + threadIdx.x; i < 4 + 2 * nranks; i += TPB_F)
        if (((i - 4) >> 1) != P.rank) x[i] = 0.0;
    block_sum_nw<NW_F, 8>(acc, lds, out);
    gm = block_max_nw<NW_F>(gm, rl);
    bad = block_max_nw<NW_F>(bad, rl);
    if (threadIdx.x == 0) {
        for (int i = 0; i < 4; ++i) x[i] = out[i];
        x[4 + 2 * P.rank] = gm;
        // the factorisation flag is identical on every rank (replicated reduced solve) except for a hand-off
        // timeout, which is local: both ride the exchange, so every rank takes the same decision
        x[5 + 2 * P.rank] = bad + ((cf & FLAG_NOT_PD) ? 4.0 : 0.0) + ((cf & FLAG_TIMEOUT) ? SC_BAD_TIMEOUT : 0.0);
        for (int i = 0; i < 4; ++i) red[6 + i] = out[4 + i];
        red[10] = 0.0;
    }
}
__global__ void k_combine(LmState* __restrict__ st, const double* __restrict__ red, double* __restrict__ scal,
                          LmParams prm, const double* __restrict__ lin, double* __restrict__ log, int nranks) {
    if (threadIdx.x != 0) return;
    const LmState S0 = *st;
    const double lin0 = lin[0], lin1 = lin[1];
    const double* y = red + RED_X;  // the reduced exchange (in place)
    double r6[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) r6[i] = red[6 + i];
    double y4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) y4[i] = y[i];
    if (S0.done) return;
    double gm = 0.0, bad = 0.0;
    for (int r = 0; r < nranks; ++r) {
        gm = fmax(gm, y[4 + 2 * r]);
        const double b = y[5 + 2 * r];
        bad = (b != b || bad != bad) ? b + bad : fmax(bad, b);  // NaN propagates
    }
    double sc[SC_N] = {};
    sc[SC_SN2] = y4[0] + r6[0];
    sc[SC_MCC] = y4[1] + r6[1];
    sc[SC_CAND] = y4[2] + r6[2];
    sc[SC_XN2] = y4[3] + r6[3];
    sc[SC_GMAX_PT] = gm;
    sc[SC_BAD] = bad + r6[4];
#pragma unroll
    for (int k = 0; k < SC_N; ++k) scal[k] = sc[k];
    lm_decide_pre(S0, st, prm, lin0, lin1, sc, log);
}

// ---------------------------------------------------------------- LM control
// |x|^2 of the active parameter blocks (ambient) -> initial state; called once after
// the iteration-0 linearisation (lin[0] = cost, lin[1] = gmax of cams+intrinsics).
// |x|^2 at the start of a solve: per-block partial sums over the active cameras / points,
// then one block reduces the partials (fixed order) and initialises the LM state.
__global__ __launch_bounds__(TPB) void k_xnorm_part(DevProblem P, const LmState* __restrict__ st,
                                                    double* __restrict__ part) {
    __shared__ double lds[4];
    __shared__ double out[1];
    const int cur = st->cur;
    double a[1] = {0.0};
    const int t = blockIdx.x * TPB + threadIdx.x;
    if (t < P.nac && P.rank == 0) {  // cameras are replicated: counted once
        const double* x = P.cams[cur] + 7 * P.ac_cam[t];
#pragma unroll
        for (int j = 0; j < 7; ++j) a[0] += x[j] * x[j];
    }
    if (t < P.n_ap) {
        const double* x = P.pts[cur] + 3 * P.pt_idx[t];
        a[0] += x[0] * x[0] + x[1] * x[1] + x[2] * x[2];
    }
    block_sum<1>(a, lds, out);
    if (threadIdx.x == 0) part[PART_INIT_XN2 * P.part_stride + blockIdx.x] = out[0];
}

__global__ __launch_bounds__(TPB) void k_xnorm_init(DevProblem P, const double* __restrict__ lin,
                                                    LmState* __restrict__ st, double* __restrict__ log,
                                                    const double* __restrict__ part, int nparts,
                                                    unsigned* progress) {
    __shared__ double lds[4];
    __shared__ double out[1];
    const int cur = st->cur;
    double a[1] = {0.0};
    for (int t = threadIdx.x; t < nparts; t += TPB) a[0] += part[PART_INIT_XN2 * P.part_stride + t];
    block_sum<1>(a, lds, out);
    if (threadIdx.x == 0) {
        const double* K = P.K[cur];
        st->xnorm2 = out[0] + (P.rank == 0 ? K[0] * K[0] + K[1] * K[1] + K[2] * K[2] + K[3] * K[3] : 0.0);
        st->x_cost = lin[0];
        st->initial_cost = lin[0];
        st->final_cost = lin[0];
        st->gmax_ci = lin[1];
        log[0] = lin[0];
        log[1] = 0.0;
        log[3] = 0.0;
        log[4] = 0.0;
        log[5] = st->radius;
        log[6] = 1.0;
        if (!isfinite(lin[0])) {
            st->done = 1;
            st->termination = 2;  // FAILURE
            st->msg = MSG_EVAL_FAIL;
            // the host follows the progress word: publish the termination (no decision will run)
            if (progress) {
                const LmState S = *st;
                publish_progress(progress, S);
            }
        }
    }
}

__global__ void k_lm_decide(LmState* __restrict__ st, LmParams prm, const double* __restrict__ lin,
                            const double* __restrict__ scal, double* __restrict__ log) {
    if (threadIdx.x == 0) lm_decide_body(st, prm, lin, scal, log);
}

// ---------------------------------------------------------------- debug hook
// Per admissible observation (point-major order) residual + Jacobians, for the parity tests.
template <bool O32>
__global__ void k_debug_lin(DevProblem P, BaConsts c, const LmState* __restrict__ st, double* __restrict__ res,
                            double* __restrict__ jcam, double* __restrict__ jpt, double* __restrict__ jint) {
    const int cur = st->cur;
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= P.n_adm) return;
    const int ap = P.po_ap[a];
    const ObsRaw<O32> o = po_obs<O32>(P, a);
    ObsEval ev;
    double jc[18], jp[9], jk[8];
    lin_obs(c, P.cams[cur] + 7 * o.idx(), P.pts[cur] + 3 * P.pt_idx[ap], P.K[cur], o.u(), o.v(), o.d(), ev, jc, jp, jk);
    for (int i = 0; i < 3; ++i) res[3 * (size_t)a + i] = ev.f[i];
    for (int i = 0; i < 18; ++i) jcam[18 * (size_t)a + i] = jc[i];
    for (int i = 0; i < 9; ++i) jpt[9 * (size_t)a + i] = jp[i];
    for (int i = 0; i < 8; ++i) jint[8 * (size_t)a + i] = jk[i];
}

// ---------------------------------------------------------------- launchers
#define CK(x)                              \
    do {                                   \
        hipError_t e_ = (x);               \
        if (e_ != hipSuccess) return e_;   \
    } while (0)

static inline int nblocks(int n, int t) { return (n + t - 1) / t; }

#define PL(kid, ...)                        \
    do {                                    \
        if (pf) pf->begin(kid, s);          \
        hipLaunchKernelGGL(__VA_ARGS__);    \
        if (pf) pf->end(s);                 \
        CK(hipGetLastError());              \
    } while (0)

// the observation kernels' obs32 (record) instantiation on obs32 windows, the f64 one otherwise
#define OPL(kid, KT, KF, ...)                          \
    do {                                               \
        if (P.obs32) PL(kid, KT, __VA_ARGS__);         \
        else PL(kid, KF, __VA_ARGS__);                 \
    } while (0)

// all-reduce on the solver stream, timed as K_COMM
#define COMM(send, recv, n, t, op)                                             \
    do {                                                                        \
        if (pf) pf->begin(K_COMM, s);                                           \
        CK(comm_allreduce(W.comm, (send), (recv), (n), (t), (op), s));          \
        if (pf) pf->end(s);                                                     \
    } while (0)

int pp_lanes() {
    static const int lanes = [] {
        int l = 1;  // measured at C4: 1 lane per point beats 2 and 4 (the per-point tail dominates)
        if (const char* e = getenv("MIBA_PP_LANES")) {
            const int v = atoi(e);
            if (v == 1 || v == 2 || v == 4) l = v;
        }
        return l;
    }();
    return lanes;
}

// number of per-workgroup partials (PART_PT_*) the Schur preparation writes
int pp_parts(const DevProblem& P) { return P.n_ap > 0 ? pp_blocks(P.n_ap) : 0; }

static hipError_t launch_point_prep(const DevProblem& P, const BaConsts& c, int mode, DevWork& W, hipStream_t s, Prof* pf) {
    const int kid = mode == 0 ? K_POINT_COLNORM : K_POINT_PREP;
    const int nb = pp_blocks(P.n_ap);
    const int n_env = mode == 1 ? W.n_env : 0;  // mode 1: the envelope tiles of S ride along
    const int fin = W.comm.on() ? 0 : 1;         // unsharded: they also finish the camera-side sums
    const dim3 g(nb + n_env), b(PP_TPB);
    switch (pp_lanes()) {
        case 1: OPL(kid, (k_point_prep<1, true>), (k_point_prep<1, false>), g, b, 0, s, P, c, W.st, mode, W.scale, W.cnp, W.pdata, W.S, W.rhs, W.part, nb,
                   W.env_tile, W.camdata, W.lin, W.chol_flag, fin, W.camdata_part, W.seg_intr, W.camdata, W.lin); break;
        case 2: OPL(kid, (k_point_prep<2, true>), (k_point_prep<2, false>), g, b, 0, s, P, c, W.st, mode, W.scale, W.cnp, W.pdata, W.S, W.rhs, W.part, nb,
                   W.env_tile, W.camdata, W.lin, W.chol_flag, fin, W.camdata_part, W.seg_intr, W.camdata, W.lin); break;
        default: OPL(kid, (k_point_prep<4, true>), (k_point_prep<4, false>), g, b, 0, s, P, c, W.st, mode, W.scale, W.cnp, W.pdata, W.S, W.rhs, W.part, nb,
                    W.env_tile, W.camdata, W.lin, W.chol_flag, fin, W.camdata_part, W.seg_intr, W.camdata, W.lin); break;
    }
    return hipSuccess;
}

__global__ void k_dummy(const LmState* __restrict__ st) {
    if (st->done) return;
}

int schur_tile_slots() {
    int dev = 0, ncu = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_schur_tile<false, true>, TPB, 0) != hipSuccess) return 0;
    return per_cu * ncu;
}

// k_lin_point over nb point workgroups + the camera sub-segments (mode 1: LM loop, mode 0: IterationZero)
static hipError_t launch_lin_point(const DevProblem& P, const BaConsts& c, int mode, DevWork& W, hipStream_t s,
                                   Prof* pf) {
    // W.fpl (LM loop): the tiled points' point side runs in the Schur tiles; here only the non-tiled points
    const bool fpl = mode == 1 && W.fpl;
    const int ap0 = fpl ? P.n_tiled_pts : 0, slot0 = fpl ? P.n_tiles : 0;
    const int nb = pp_blocks(P.n_ap - ap0);
    const int kid = mode ? K_LIN_POINT : K_CAM_SIDE;
    if (nb + P.n_seg > 0) switch (pp_lanes()) {
        case 1: OPL(kid, (k_lin_point<1, true>), (k_lin_point<1, false>), dim3(nb + P.n_seg), dim3(TPB), 0, s, P, c, W.st, W.scale, W.cnp, W.pdata,
                   W.part, nb, W.camdata_part, W.seg_intr, W.lin + 1, mode, ap0, slot0); break;
        case 2: OPL(kid, (k_lin_point<2, true>), (k_lin_point<2, false>), dim3(nb + P.n_seg), dim3(TPB), 0, s, P, c, W.st, W.scale, W.cnp, W.pdata,
                   W.part, nb, W.camdata_part, W.seg_intr, W.lin + 1, mode, ap0, slot0); break;
        default: OPL(kid, (k_lin_point<4, true>), (k_lin_point<4, false>), dim3(nb + P.n_seg), dim3(TPB), 0, s, P, c, W.st, W.scale, W.cnp, W.pdata,
                    W.part, nb, W.camdata_part, W.seg_intr, W.lin + 1, mode, ap0, slot0); break;
    }
    return hipSuccess;
}

// IterationZero of the fused path: the points' column norms ride in the camera-side launch (k_lin_point
// mode 0), so launch_scale has no point pass of its own
static bool zero_fused(const DevProblem& P, const DevWork& W) { return W.fused && P.n_ap > 0; }

hipError_t launch_linearize(const DevProblem& P, const BaConsts& c, int gated, DevWork& W, hipStream_t s, Prof* pf) {
    if (gated && W.fused) return hipSuccess;  // the LM loop's camera side runs inside k_lin_point (launch_build)
    if (!gated && zero_fused(P, W)) {
        CK(launch_lin_point(P, c, 0, W, s, pf));
        if (P.n_seg == 0) CK(hipMemsetAsync(W.lin + 1, 0, sizeof(double), s));
    } else if (P.n_seg > 0)
        OPL(K_CAM_SIDE, k_cam_side<true>, k_cam_side<false>, dim3(P.n_seg), dim3(TPB), 0, s, P, c, W.st, gated, W.camdata_part, W.seg_intr,
           W.lin + 1);
    else
        CK(hipMemsetAsync(W.lin + 1, 0, sizeof(double), s));
    const size_t ncd = (size_t)P.nac * CAMDATA;
    if (!W.comm.on()) {  // camdata_loc == camdata unsharded
        // in the LM loop the envelope tiles (k_point_prep / k_env_assemble) finish the camera-side sums;
        // iteration 0 needs them before the Jacobi scale and the initial state
        if (!gated)
            PL(K_LIN_FINALIZE, k_cam_finalize, dim3(P.nac + 1), dim3(TPB), 0, s, P, c, W.st, gated, W.camdata_part,
               W.camdata_loc, W.seg_intr, W.lin, 0, (double*)nullptr);
        return hipSuccess;
    }
    // sharded: one all-reduce of [camdata | intrinsics partials] between the local sums and
    // the finalisation (camdata_loc is zero for cameras this shard does not observe)
    PL(K_LIN_FINALIZE, k_cam_finalize, dim3(P.nac + 1), dim3(TPB), 0, s, P, c, W.st, gated, W.camdata_part,
       W.camdata_loc, W.seg_intr, W.lin, 1, W.camdata_loc + ncd);
    COMM(W.camdata_loc, W.camdata, ncd + SEGINTR, COMM_F64, COMM_SUM);
    PL(K_LIN_FINALIZE, k_lin_finalize, dim3(1), dim3(TPB), 0, s, P, c, W.st, gated, W.camdata, W.seg_intr, W.lin, 2,
       W.camdata + ncd);
    return hipSuccess;
}

hipError_t launch_scale(const DevProblem& P, const BaConsts& c, int jacobi, DevWork& W, hipStream_t s, Prof* pf) {
    if (P.n_ap > 0 && !zero_fused(P, W))
        CK(launch_point_prep(P, c, 0, W, s, pf));
    const int nt = 6 * P.nac + 3 * P.n_ap + 4;
    PL(K_SCALE, k_scale, dim3(nblocks(nt, TPB)), dim3(TPB), 0, s, P, W.camdata, W.cnp, W.lin, jacobi, W.scale);
    return hipSuccess;
}

// Start of a solve: both parameter slots from the prepared initial values, and the fresh LM state
// (one launch instead of six copies and a host-to-device state copy); fused path: also zeroes S and rhs,
// the atomic targets of the first assembly (grid-stride, 16-byte stores).
__global__ __launch_bounds__(TPB) void k_reset(DevProblem P, LmState st0, LmState* __restrict__ st,
                                               const double* __restrict__ cams0, const double* __restrict__ pts0,
                                               const double* __restrict__ K0, int ncd, int npd,
                                               double* __restrict__ S, size_t nS2, double* __restrict__ rhs,
                                               int nrhs) {
    const int t = blockIdx.x * TPB + threadIdx.x;
    if (t < ncd) { const double v = cams0[t]; P.cams[0][t] = v; P.cams[1][t] = v; }
    if (t < npd) { const double v = pts0[t]; P.pts[0][t] = v; P.pts[1][t] = v; }
    if (t < 4) { const double v = K0[t]; P.K[0][t] = v; P.K[1][t] = v; }
    if (t == 0) *st = st0;
    if (t < nrhs) rhs[t] = 0.0;
    const size_t stride = (size_t)gridDim.x * TPB;
    for (size_t e = t; e < nS2; e += stride) reinterpret_cast<double2*>(S)[e] = double2{0.0, 0.0};
}

// ba_prepare: the observation layout the window uses, from the raw window (uploaded as the caller passed it) and
// the host plan's slots (ba_plan.cpp). Workgroups [0, nbo): one observation per thread in the caller's order, read
// once (coalesced) and scattered to its point-major and camera-major slots; the rest: one active point per thread,
// its slots' point indices. A gather by slot instead (round 3) read the raw arrays in a permuted order, every 4-16 B
// read pulling a whole line: 349 MB per launch at C4 for ~110 MB of data. The scatter's writes land in runs (each
// camera's slots and each point's slots are in the caller's index order), and consecutive workgroups of the range
// run on one XCD (dispatch is round-robin over the 8 XCDs), so a run's lines fill in one L2 before they are written.
// O32: the 16-byte records only (every observation kernel of an obs32 window reads those); else the f64 arrays.
template <bool O32>
__global__ __launch_bounds__(TPB) void k_prep_gather(DevProblem P, PrepRaw R, int nbo) {
    const int b = blockIdx.x, tid = threadIdx.x;
    if (b < nbo) {
        const int per = nbo >> 3, rem = nbo & 7, x = b & 7;
        const int lb = x * per + (x < rem ? x : rem) + (b >> 3);  // XCD x runs blocks [x per + min(x, rem), ...)
        const int k = lb * TPB + tid;
        if (k >= R.n_obs) return;
        const int pq = R.po_dest[k], cq = R.co_dest[k];
        if (pq < 0) return;  // not admissible (cq < 0 too)
        const int cam = R.cam[k], pt = R.pt[k];
        const double2 uv = R.uv[k];
        const double dep = R.depth[k];
        const_cast<int*>(P.po_ac)[pq] = R.cam_ac[cam];
        if constexpr (O32) {  // exact: the host checked that every admissible value is an f32
            const_cast<float4*>(P.po_rec)[pq] = float4{(float)uv.x, (float)uv.y, (float)dep, __int_as_float(cam)};
            const_cast<float4*>(P.co_rec)[cq] = float4{(float)uv.x, (float)uv.y, (float)dep, __int_as_float(pt)};
        } else {
            const_cast<int*>(P.po_cam)[pq] = cam;
            const_cast<double2*>(P.po_uv)[pq] = uv;
            const_cast<double*>(P.po_depth)[pq] = dep;
            const_cast<int*>(P.co_pt)[cq] = pt;
            const_cast<double2*>(P.co_uv)[cq] = uv;
            const_cast<double*>(P.co_depth)[cq] = dep;
        }
    } else {
        const int a = (b - nbo) * TPB + tid;
        if (a >= P.n_ap) return;
        const int pi = P.pt_idx[a];
        for (int q = P.pt_ptr[a]; q < P.pt_ptr[a + 1]; ++q) {
            const_cast<int*>(P.po_ap)[q] = a;
            const_cast<int*>(P.po_pt)[q] = pi;
        }
    }
}

hipError_t launch_prep_gather(const DevProblem& P, const PrepRaw& R, hipStream_t s) {
    const int nbo = nblocks(R.n_obs, TPB), nba = nblocks(P.n_ap, TPB);
    if (nbo + nba > 0) {
        if (P.obs32) hipLaunchKernelGGL(k_prep_gather<true>, dim3(nbo + nba), dim3(TPB), 0, s, P, R, nbo);
        else hipLaunchKernelGGL(k_prep_gather<false>, dim3(nbo + nba), dim3(TPB), 0, s, P, R, nbo);
    }
    return hipGetLastError();
}

hipError_t launch_reset(const DevProblem& P, DevWork& W, const LmState& st0, const double* cams0, const double* pts0,
                        const double* K0, int n_cams, int n_points, hipStream_t s) {
    if (W.sw_cnt) CK(hipMemsetAsync(W.sw_cnt, 0, sizeof(unsigned), s));  // the small-window launch's counter
    W.sw_seq = 0;
    if (W.tail_flags) CK(hipMemsetAsync(W.tail_flags, 0, 3 * sizeof(unsigned), s));  // the band tail's hand-offs
    W.tail_seq = 0;
    if (W.tail_y)  // both y buffers empty (the pattern's two 32-bit halves are equal)
        CK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(W.tail_y), (int)BCR_Y_EMPTY_D32, 2 * 2 * (size_t)P.npad, s));
    const int ncd = 7 * n_cams, npd = 3 * n_points;
    // fused path: S (npad^2, even: npad is a multiple of 16) and rhs are zeroed here too
    const size_t nS2 = W.fused ? (size_t)P.npad * P.npad / 2 : 0;
    const int nrhs = W.fused ? P.npad : 0;
    const int nb = std::max(nblocks(std::max({ncd, npd, nrhs, 4}), TPB), (int)std::min<size_t>(nS2 / (4 * TPB), 2048));
    hipLaunchKernelGGL(k_reset, dim3(nb), dim3(TPB), 0, s, P, st0, W.st, cams0, pts0, K0, ncd, npd, W.S, nS2, W.rhs,
                       nrhs);
    return hipGetLastError();
}

hipError_t launch_init_state(const DevProblem& P, DevWork& W, unsigned* progress, hipStream_t s, Prof* pf) {
    const int nparts = std::max(nblocks(std::max(P.nac, P.n_ap), TPB), 1);
    PL(K_XNORM, k_xnorm_part, dim3(nparts), dim3(TPB), 0, s, P, W.st, W.part);
    PL(K_XNORM, k_xnorm_init, dim3(1), dim3(TPB), 0, s, P, W.lin, W.st, W.log, W.part, nparts, progress);
    if (W.comm.on()) COMM(&W.st->xnorm2, &W.st->xnorm2, 1, COMM_F64, COMM_SUM);  // points of all shards
    return hipSuccess;
}

hipError_t launch_build(const DevProblem& P, const BaConsts& c, DevWork& W, hipStream_t s, Prof* pf) {
    // point records + intrinsics Schur partials, then the envelope of S: clear + camera / intrinsics
    // blocks, LM diagonal, pad (rank 0 only), the points' intrinsics terms, rhs, chol_flag
    EnvArgs E{};
    if (W.sw) {  // small window: one launch (k_schur_tile<..., FP>), no k_lin_point
        E = EnvArgs{W.env_tile, W.n_env, W.camdata, W.lin, W.chol_flag, W.camdata_part, W.seg_intr, W.camdata, W.lin, 1,
                    W.pdata, W.part, W.camdata_part, W.seg_intr, W.sw_cnt, (++W.sw_seq) * (unsigned)P.n_seg, P.n_seg,
                    pp_blocks(P.n_ap - P.n_tiled_pts, 1)};
        const int n_sch = P.n_tiles + 1 + E.n_cs + E.n_gb + E.n_env;
        static const int fp_stamps = env_on("MIBA_SCHUR_STAMPS");
        static DeviceScratch fst_buf;
        if (fp_stamps == 1 && P.obs32) {  // diagnostic: per-tile phase cycles (zero, A incl. the point side, B, flush)
            unsigned long long* fst = fst_buf.get<unsigned long long>(sizeof(unsigned long long) * 10 * 256);
            if (!fst) return hipErrorOutOfMemory;
            PL(K_SCHUR_TILE, (k_schur_tile<true, true, true, true, true>), dim3(n_sch), dim3(TPB), 0, s, P, c, W.st, W.scale,
               W.pdata, W.S, W.rhs, fst, 0, W.part, (double*)nullptr, E);
            std::vector<unsigned long long> h5((size_t)5 * P.n_tiles);
            CK(hipMemcpyAsync(h5.data(), fst, sizeof(h5[0]) * h5.size(), hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            double sum[5] = {0, 0, 0, 0, 0};
            for (int t = 0; t < P.n_tiles; ++t)
                for (int k = 0; k < 5; ++k) sum[k] += (double)h5[5 * t + k];
            std::vector<unsigned long long> hs((size_t)5 * P.n_tiles);
            CK(hipMemcpy(hs.data(), fst + 5 * 256, sizeof(hs[0]) * hs.size(), hipMemcpyDeviceToHost));
            double sb[5] = {0, 0, 0, 0, 0};
            for (int t = 0; t < P.n_tiles; ++t)
                for (int k = 0; k < 5; ++k) sb[k] += (double)hs[5 * t + k];
            fprintf(stderr, "  point side (thread 0, from the tile start): evaluated %.0f, barrier passed %.0f, point tail "
                    "done %.0f\n", sb[2] / P.n_tiles, sb[3] / P.n_tiles, sb[4] / P.n_tiles);
            fprintf(stderr, "schur_tile FP %d tiles, mean cycles/tile: point side + zero stores %.0f, barrier %.0f, phaseA %.0f, "
                    "phaseB %.0f (wave 0: rhs dot done %.0f, MFMA done %.0f), flush %.0f\n", P.n_tiles, sum[4] / P.n_tiles,
                    sum[0] / P.n_tiles, sum[1] / P.n_tiles, sum[2] / P.n_tiles, sb[0] / P.n_tiles, sb[1] / P.n_tiles,
                    sum[3] / P.n_tiles);
        } else
        OPL(K_SCHUR_TILE, (k_schur_tile<false, true, true, true, true>), (k_schur_tile<false, false, true, true, true>), dim3(n_sch),
            dim3(TPB), 0, s, P, c, W.st, W.scale, W.pdata, W.S, W.rhs, (unsigned long long*)nullptr, 0, W.part,
            (double*)nullptr, E);
        if (P.n_ovf_obs > 0)
            OPL(K_OBS_PAIRS, k_obs_pairs<true>, k_obs_pairs<false>, dim3(nblocks(P.n_ovf_obs, TPB)), dim3(TPB), 0, s, P, c,
                W.st, W.scale, W.pdata, W.S, W.rhs);
        return hipSuccess;
    }
    if (W.fused) {  // point side + gated camera side in one launch; the envelope tiles ride in k_schur_tile
        CK(launch_lin_point(P, c, 1, W, s, pf));
        // unsharded: the envelope tiles finish the camera sums and lin (fin 1); landmark shard: they write this
        // rank's terms and sums for the folded exchange (fin 2; camdata_loc = [camera sums | intrinsics sums])
        const int ncd = P.nac * CAMDATA;
        E = W.comm.on() ? EnvArgs{W.env_tile, W.n_env, W.camdata, W.lin, W.chol_flag, W.camdata_part, W.seg_intr,
                                  W.camdata_loc, W.camdata_loc + ncd, 2}
                        : EnvArgs{W.env_tile, W.n_env, W.camdata, W.lin, W.chol_flag, W.camdata_part, W.seg_intr,
                                  W.camdata, W.lin, 1};
        if (W.fpl) {  // the tiles write the point records and their partials
            E.pdata_w = W.pdata;
            E.part_w = W.part;
        }
    } else if (P.n_ap > 0)
        CK(launch_point_prep(P, c, 1, W, s, pf));  // + the envelope tiles
    else
        PL(K_ASSEMBLE, k_env_assemble, dim3(W.n_env), dim3(TPB), 0, s, P, c, W.st, W.env_tile, W.camdata, W.lin,
           W.scale, W.S, W.rhs, W.chol_flag, W.comm.on() ? 0 : 1, W.camdata_part, W.seg_intr, W.camdata, W.lin);
    // Schur tiles + one workgroup for the intrinsics Schur terms (when there are points)
    const int n_sch = P.n_tiles + ((P.n_ap > 0 || W.fused) ? 1 : 0) + E.n_env;
    if (n_sch > 0)
    {
        static const int smode = env_on("MIBA_SCHUR_STAMPS");
        static DeviceScratch sst_buf;
        if (smode == 1) {
            unsigned long long* sst = sst_buf.get<unsigned long long>(sizeof(unsigned long long) * 5 * std::max(P.n_tiles, 1));
            if (!sst) return hipErrorOutOfMemory;
            if (W.fpl)  // (the opt-in fused point side, stamped)
                OPL(K_SCHUR_TILE, (k_schur_tile<true, true, false, true>), (k_schur_tile<true, false, false, true>),
                    dim3(n_sch), dim3(TPB), 0, s, P, c, W.st, W.scale, W.pdata, W.S, W.rhs, sst,
                    pp_blocks(P.n_ap - P.n_tiled_pts), W.part, W.det_tbuf, E);
            else
            OPL(K_SCHUR_TILE, (k_schur_tile<true, true>), (k_schur_tile<true, false>), dim3(n_sch), dim3(TPB), 0, s, P, c, W.st, W.scale, W.pdata, W.S, W.rhs,
               sst, pp_parts(P), W.part, W.det_tbuf, E);
            std::vector<unsigned long long> h5((size_t)5 * P.n_tiles), h((size_t)4 * P.n_tiles);
            CK(hipMemcpyAsync(h5.data(), sst, sizeof(h5[0]) * h5.size(), hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            double sum[5] = {0, 0, 0, 0, 0}, mx = 0;
            for (int t = 0; t < P.n_tiles; ++t) {
                double tot = 0;
                for (int k = 0; k < 5; ++k) { sum[k] += (double)h5[5 * t + k]; tot += (double)h5[5 * t + k]; }
                for (int k = 0; k < 4; ++k) h[4 * t + k] = h5[5 * t + k] + (k == 0 ? h5[5 * t + 4] : 0ull);
                mx = std::max(mx, tot);
            }
            fprintf(stderr, "schur_tile %d tiles, mean cycles/tile: zero %.0f (stores %.0f, barrier %.0f) phaseA %.0f phaseB %.0f flush %.0f | max total %.0f\n",
                    P.n_tiles, (sum[0] + sum[4]) / P.n_tiles, sum[4] / P.n_tiles, sum[0] / P.n_tiles, sum[1] / P.n_tiles,
                    sum[2] / P.n_tiles, sum[3] / P.n_tiles, mx);
            // the slowest tiles: span, chunks, points (the kernel lasts as long as its slowest tile)
            std::vector<int> tspan(P.n_tiles), tch(P.n_tiles + 1), cap;
            CK(hipMemcpy(tspan.data(), P.tile_span, sizeof(int) * P.n_tiles, hipMemcpyDeviceToHost));
            CK(hipMemcpy(tch.data(), P.tile_chunk, sizeof(int) * (P.n_tiles + 1), hipMemcpyDeviceToHost));
            cap.resize(tch[P.n_tiles] + 1);
            CK(hipMemcpy(cap.data(), P.chunk_ap, sizeof(int) * cap.size(), hipMemcpyDeviceToHost));
            std::vector<std::pair<double, int>> tot(P.n_tiles);
            for (int t = 0; t < P.n_tiles; ++t)
                tot[t] = {(double)(h[4 * t] + h[4 * t + 1] + h[4 * t + 2] + h[4 * t + 3]), t};
            std::sort(tot.begin(), tot.end());
            for (int q = 0; q < 6 && q < P.n_tiles; ++q) {
                const int t = tot[P.n_tiles - 1 - q].second;
                fprintf(stderr, "  slow tile %d: %.0f cycles (zero %llu A %llu B %llu flush %llu) span %d chunks %d points %d\n", t,
                        tot[P.n_tiles - 1 - q].first, h[4 * t], h[4 * t + 1], h[4 * t + 2], h[4 * t + 3], tspan[t],
                        tch[t + 1] - tch[t], cap[tch[t + 1]] - cap[tch[t]]);
            }
            const int t50 = tot[P.n_tiles / 2].second;
            fprintf(stderr, "  median tile %d: %.0f cycles span %d chunks %d points %d\n", t50, tot[P.n_tiles / 2].first,
                    tspan[t50], tch[t50 + 1] - tch[t50], cap[tch[t50 + 1]] - cap[tch[t50]]);
        } else {
            if (W.fpl)  // the point side in the tiles (one Jacobian evaluation per observation); non-tiled points' partials
                OPL(K_SCHUR_TILE, (k_schur_tile_fpl<true>), (k_schur_tile_fpl<false>),
                    dim3(n_sch), dim3(TPB), 0, s, P, c, W.st, W.scale, W.pdata, W.S, W.rhs, (unsigned long long*)nullptr,
                    pp_blocks(P.n_ap - P.n_tiled_pts), W.part, W.det_tbuf, E);
            else if (n_sch <= 256)  // one round of resident workgroups whatever the register count
                OPL(K_SCHUR_TILE, (k_schur_tile<false, true, true>), (k_schur_tile<false, false, true>), dim3(n_sch), dim3(TPB), 0, s, P, c, W.st, W.scale, W.pdata, W.S,
                    W.rhs, (unsigned long long*)nullptr, pp_parts(P), W.part, W.det_tbuf, E);
            else
            OPL(K_SCHUR_TILE, (k_schur_tile<false, true>), (k_schur_tile<false, false>), dim3(n_sch), dim3(TPB), 0, s, P, c, W.st, W.scale, W.pdata, W.S,
               W.rhs, (unsigned long long*)nullptr, pp_parts(P), W.part, W.det_tbuf, E);
        }
        if (W.det_tbuf && P.n_tiles > 0)
            PL(K_SCHUR_TILE, k_schur_gather, dim3(W.n_env), dim3(TPB), 0, s, P, W.st, W.env_tile, W.det_tbuf,
               W.det_trange, W.S, W.rhs);
    }
    if (P.n_ovf_obs > 0) {
        if (W.det_tbuf)
            OPL(K_OBS_PAIRS, k_obs_pairs_det<true>, k_obs_pairs_det<false>, dim3(1), dim3(128), 0, s, P, c, W.st, W.scale,
                W.pdata, W.S, W.rhs);
        else
            OPL(K_OBS_PAIRS, k_obs_pairs<true>, k_obs_pairs<false>, dim3(nblocks(P.n_ovf_obs, TPB)), dim3(TPB), 0, s, P, c, W.st, W.scale,
               W.pdata, W.S, W.rhs);
    }
    if (W.comm.on() && W.fused) {
        // folded exchange: ONE all-reduce of [envelope | rhs | camera sums | intrinsics sums]; the LM diagonal,
        // the prior, camdata and lin follow from the reduced sums (k_env_unpack_fin)
        const int ncam = P.nac * CAMDATA + SEGINTR;
        const size_t ne = (size_t)W.n_env * 256 + P.npad + ncam;
        PL(K_COMM, k_env_pack, dim3(W.n_env + env_tail_blocks(P.npad, ncam)), dim3(TPB), 0, s, W.st, W.env_tile,
           W.n_env, P.npad, W.S, W.rhs, W.env_loc, 0, W.camdata_loc, ncam);
        COMM(W.env_loc, W.env_loc, ne, COMM_F64, COMM_SUM);  // in place (a 1-rank communicator copies nothing)
        PL(K_COMM, k_env_unpack_fin, dim3(W.n_env + env_tail_blocks(P.npad, P.nac * CAMDATA) + 1), dim3(TPB), 0, s,
           P, c, W.st, W.env_tile, W.n_env, W.env_loc, W.scale, W.S, W.rhs, W.camdata, W.lin);
    } else if (W.comm.on()) {  // S = sum over the landmark shards: envelope tiles + rhs
        const size_t ne = (size_t)W.n_env * 256 + P.npad;
        const int nt = W.n_env + env_tail_blocks(P.npad, 0);
        PL(K_COMM, k_env_pack, dim3(nt), dim3(TPB), 0, s, W.st, W.env_tile, W.n_env, P.npad, W.S, W.rhs, W.env_loc, 0,
           (const double*)nullptr, 0);
        COMM(W.env_loc, W.env_loc, ne, COMM_F64, COMM_SUM);
        PL(K_COMM, k_env_pack, dim3(nt), dim3(TPB), 0, s, W.st, W.env_tile, W.n_env, P.npad, W.S, W.rhs, W.env_loc,
           1, (const double*)nullptr, 0);
    }
    return hipSuccess;
}

template <int BW>
static hipError_t launch_band(const DevProblem& P, DevWork& W, hipStream_t s, Prof* pf) {
    const size_t lds = sizeof(BandLds<BW>) + sizeof(int) * BAND_MAX_NB;
    static DeviceOnce attr;
    static DeviceScratch stamp_buf;
    static const int stamp_mode = env_on("MIBA_CHOL_STAMPS");
    CK(attr([]() -> hipError_t {
        CK(hipFuncSetAttribute((const void*)k_chol_band<BW, false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        CK(hipFuncSetAttribute((const void*)k_chol_band<BW, true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        return hipSuccess;
    }));
    if (stamp_mode == 1) {
        unsigned long long* dst = stamp_buf.get<unsigned long long>(8 * sizeof(unsigned long long));
        if (!dst) return hipErrorOutOfMemory;
        PL(K_CHOL, (k_chol_band<BW, true>), dim3(1), dim3(TPB), lds, s, W.st, W.S, P.npad, P.npad / 16, W.fcol, W.rhs,
           W.chol_flag, dst);
        unsigned long long h[8];
        CK(hipMemcpyAsync(h, dst, sizeof(h[0]) * 5, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        fprintf(stderr, "chol_band<%d> nb=%d cycles: pre %llu trsm %llu update+lookahead %llu retire %llu backward %llu\n", BW,
                P.npad / 16, h[0], h[1], h[2], h[3], h[4]);
        return hipSuccess;
    }
    PL(K_CHOL, (k_chol_band<BW, false>), dim3(1), dim3(TPB), lds, s, W.st, W.S, P.npad, P.npad / 16, W.fcol, W.rhs,
       W.chol_flag, (unsigned long long*)nullptr);
    return hipSuccess;
}

hipError_t launch_factor(const DevProblem& P, const BaConsts& c, DevWork& W, hipStream_t s, Prof* pf) {
    if (P.solver == 2 && W.tail) return hipSuccess;  // the band solve runs in launch_update's tail launch
    if (P.solver == 2) return launch_bcr(P, c, W, W.bcr, s, pf);  // k_bcr_border also applies the camera step
    if (P.solver == 1) switch (P.band_w) {
        case 1: return launch_band<1>(P, W, s, pf);
        case 2: return launch_band<2>(P, W, s, pf);
        case 3: return launch_band<3>(P, W, s, pf);
        case 4: return launch_band<4>(P, W, s, pf);
        case 5: return launch_band<5>(P, W, s, pf);
        case 6: return launch_band<6>(P, W, s, pf);
        default: break;
    }
    PL(K_CHOL, k_chol, dim3(1), dim3(TPB), 0, s, W.st, W.S, P.npad, P.npad / 16, W.fcol, W.rptr, W.rows, W.rhs,
       W.chol_flag);
    return hipSuccess;
}

hipError_t launch_update(const DevProblem& P, const BaConsts& c, const LmParams& prm, DevWork& W, hipStream_t s,
                         Prof* pf) {
    // BCR: k_bcr_border already applied the camera / intrinsics step (one partial per BCR block)
    const bool fused_upd = P.solver == 2;
    const int nb_upd = fused_upd ? (P.nac + BCR_CAMS - 1) / BCR_CAMS : nblocks(P.nac + 1, TPB);
    static const int ndummy = [] {  // diagnostic: extra empty launches per iteration
        const char* e = getenv("MIBA_DUMMY_LAUNCHES");
        return e ? atoi(e) : 0;
    }();
    for (int k = 0; k < ndummy; ++k) PL(K_DUMMY, k_dummy, dim3(1), dim3(64), 0, s, W.st);
    if (W.tail) {  // band solve + back-substitution + decision in one launch (ba_band.hip k_band_tail)
        const int nb_pt = W.sw ? P.n_tiles + pp_blocks(P.n_ap - P.n_tiled_pts, 1) : pp_parts(P);
        return launch_band_tail(P, c, prm, W, W.bcr.band, nb_pt, nb_upd, s, pf);
    }
    if (!fused_upd)
        PL(K_UPDATE_CAMS, k_update_cams, dim3(nb_upd), dim3(TPB), 0, s, P, c, W.st, W.scale, W.camdata, W.lin, W.rhs,
           W.delta, W.part);
    const int nb_bs = P.n_bs_chunks;
    if (W.fused && P.n_ap == 0)  // an empty landmark shard: no back-substitution chunk zeroes S for the next assembly
        PL(K_MEMSET_S, k_env_zero, dim3(W.n_env), dim3(TPB), 0, s, W.st, W.env_tile, P.npad, W.S);
    // the points' gradient max / bad partials: per point workgroup, or per Schur tile + non-tiled point workgroup
    const int nb_pt = W.sw ? P.n_tiles + pp_blocks(P.n_ap - P.n_tiled_pts, 1)
                           : (W.fpl ? P.n_tiles + pp_blocks(P.n_ap - P.n_tiled_pts) : pp_parts(P));
    // the split BCR kernel's call epoch (the persistent kernel's is advanced by k_bcr_border)
    unsigned* const ep = (P.solver == 2 && W.bcr.persist >= 2) ? W.bcr.flags : nullptr;
    if (W.bsfin && P.n_ap > 0 && W.fused && !W.comm.on())  // back-substitution + decision in one launch (ba_band.hip)
        return launch_backsub_final(P, c, prm, W, nb_pt, nb_upd, ep, s, pf);
    if (P.n_ap > 0)
        OPL(K_BACKSUB_EVAL, k_backsub_chunk<true>, k_backsub_chunk<false>, dim3(nb_bs), dim3(TPB), 0, s, P, c, W.st, W.scale, W.pdata, W.rhs, W.delta,
           W.part, W.env_tile, W.fused ? W.n_env : 0, W.S);
    if (!W.comm.on()) {
        PL(K_FINAL, k_final<2>, dim3(1), dim3(TPB_F), 0, s, P, W.st, nb_pt, nb_upd, P.n_ap > 0 ? nb_bs : 0, W.part,
           W.chol_flag, W.scal, prm, W.lin, W.log, W.fused ? W.rhs : (double*)nullptr, ep);
        return hipSuccess;
    }
    PL(K_FINAL, k_final_shard<1>, dim3(1), dim3(TPB_F), 0, s, P, W.st, nb_pt, nb_upd, P.n_ap > 0 ? nb_bs : 0, W.part,
       W.chol_flag, W.red, W.fused ? W.rhs : (double*)nullptr, W.comm.nranks, ep);
    COMM(W.red + RED_X, W.red + RED_X, 4 + 2 * W.comm.nranks, COMM_F64, COMM_SUM);  // in place
    PL(K_FINAL, k_combine, dim3(1), dim3(64), 0, s, W.st, W.red, W.scal, prm, W.lin, W.log, W.comm.nranks);
    return hipSuccess;
}

hipError_t launch_decide(const DevProblem& P, const LmParams& prm, DevWork& W, hipStream_t s, Prof* pf) {
    PL(K_DECIDE, k_lm_decide, dim3(1), dim3(64), 0, s, W.st, prm, W.lin, W.scal, W.log);
    return hipSuccess;
}

hipError_t launch_debug_lin(const DevProblem& P, const BaConsts& c, DevWork& W, double* res, double* jc, double* jp,
                            double* jk, hipStream_t s) {
    if (P.n_adm > 0) {
        if (P.obs32) hipLaunchKernelGGL(k_debug_lin<true>, dim3(nblocks(P.n_adm, TPB)), dim3(TPB), 0, s, P, c, W.st, res, jc, jp, jk);
        else hipLaunchKernelGGL(k_debug_lin<false>, dim3(nblocks(P.n_adm, TPB)), dim3(TPB), 0, s, P, c, W.st, res, jc, jp, jk);
    }
    return hipGetLastError();
}

hipError_t sw_set_spin_limit(unsigned limit) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_sw_spin_limit), &limit, sizeof(limit));
}

}  // namespace miba
