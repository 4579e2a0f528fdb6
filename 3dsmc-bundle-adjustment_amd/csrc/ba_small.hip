// ba_small.hip — libmiba: the whole solve of a small window in ONE workgroup (gfx950 / MI355X, f64).
//
// The reference solves small windows: windowOptimize (/root/reference/src/OptimizationUtils.cpp:215-313)
// runs on 10-keyframe windows (BundleAdjustmentConfig.h:52-53) of ~1-2k observations and is called
// again for every frame (main.cpp:163-168). There the multi-launch LM iteration (ba_kernels.hip) is
// latency-bound: ~85 us per iteration, of which ~35 us is the reduced solve and the rest the seven
// dependent launches' own ramp and serial reductions. k_small_solve runs iteration 0 and every LM
// iteration of ceres::Solve (:300) in one launch of one 512-thread workgroup:
//   - linearisation (iteration 0 and after each accepted step): camera-side sums per sub-segment on the
//     waves (cam_accum + wave reduce-scatter), point sums V | e | Kt per point, and the per-observation
//     W_o = Jc^T Jp, all cached in global memory (L2-resident at these sizes), so a step re-reads
//     18 + 21 doubles instead of re-evaluating Jacobians;
//   - the damped, Jacobi-scaled reduced camera system S (npad <= SMALL_NPAD) is assembled in LDS:
//     camera / intrinsics blocks + LM diagonal (the envelope formula of env_tile), then the points'
//     Schur terms by *tasks* — one camera-pair block (a, b) or one camera's border rows — each owned
//     by one wave: the lanes take the task's observation pairs at a fixed stride, the wave reduces,
//     and the wave alone writes its block. No atomics: bitwise reproducible;
//   - Cholesky by 16x16 tiles in LDS (one wave factors the diagonal tile in registers, potrf16_regs;
//     row-parallel TRSM; MFMA trailing updates), the forward substitution fused into the factorisation,
//     blocked backward substitution;
//   - camera / intrinsics step (update_camera / update_intrinsics), point back-substitution and candidate
//     cost per point thread, fixed-order block sums, and the Ceres 2.0 decision (lm_decide_body) on
//     thread 0 between barriers.
// Same arithmetic as the multi-launch path element for element except for the summation order.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "ba_common.h"

namespace miba {

static constexpr int NT = SMALL_TPB;  // 512 threads
static constexpr int NW = NT / 64;    // 8 waves (2 per SIMD: up to 256 VGPRs per lane)
typedef double d4s __attribute__((ext_vector_type(4)));

// LDS: fixed part, then the reduced system S[npad][npad + 1] (odd stride: conflict-free column reads)
struct SmallLds {
    double red[NW * 64];        // block reductions / backward-solve partials
    double wout[NW][64];        // per-wave packed camera-side sums
    double lin[LIN_N];
    double io[SEGINTR];
    double kk[16];
    double yv[SMALL_NPAD];      // rhs -> z -> y
    double rdiag[SMALL_NPAD];   // 1 / diag(L)
    double gmax_pt;
    int bad;                    // Cholesky pivot failure
    LmState st;
};
size_t small_lds_bytes(int npad) { return sizeof(SmallLds) + sizeof(double) * (size_t)npad * (npad + 1); }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave reduce-scatter of N sums (WaveHalve); calls put(index, value) for the lane's share.
template <int N, class F>
__device__ __forceinline__ void wave_scatter(double (&v)[N], int lane, F put) {
    int base = 0, len = N;
    WaveHalve<N, 32>::run(v, lane, base, len);
    constexpr int R = HalveRemain<N, 32>::value;
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (j < len) put(base + j, v[j]);
}

// Diagnostic stamps (MIBA_SMALL_STAMPS=1): shader-clock cycles per phase, summed over the solve by
// thread 0 (after a barrier, so each phase's time is that of its slowest wave).
enum { SST_INIT = 0, SST_LIN, SST_POINT, SST_ASSEMBLE, SST_TASKS, SST_CHOL, SST_CAMS, SST_BACKSUB, SST_DECIDE,
       SST_CH_POTRF, SST_CH_TRSM, SST_CH_MFMA, SST_CH_BACK, SST_N };
__device__ __forceinline__ unsigned long long small_clock() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

// ---------------------------------------------------------------- linearisation at x = slot cur
// Camera-side sums per sub-segment (camdata_part / seg_intr, the k_cam_side layout), point sums
// (pv), W_o (wc), then per camera the in-order sum of its sub-segments (camdata), the intrinsics
// block (lin) and the gradient max-norm terms. Leaves L.lin / W.lin and L.gmax_pt.
__device__ void small_linearize(const DevProblem& P, const BaConsts& c, const DevWork& W, SmallLds& L, int cur) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const double* pts = P.pts[cur];
    const double* cams = P.cams[cur];
    const double* K = P.K[cur];
    // camera side: one sub-segment per wave at a time, the packed sums in two passes (U | g | cost, then
    // C | Ukk | gk) to stay within the registers of 2 waves per SIMD
    for (int s = wave; s < P.n_seg; s += NW) {
        const int ac = P.seg_ac[s];
        const double* pose = cams + 7 * P.seg_cam[s];
        double* wo = L.wout[wave];
        const int o0 = P.seg_ptr[s], o1 = P.seg_ptr[s + 1];
        {
            double acc[CAM_NZ_U];
#pragma unroll
            for (int i = 0; i < CAM_NZ_U; ++i) acc[i] = 0.0;
            for (int o = o0 + lane; o < o1; o += 64) {
                const double2 uv = P.co_uv[o];
                ObsEval e;
                double jc[18], jp[9], jk[8];
                lin_obs(c, pose, pts + 3 * P.co_pt[o], K, uv.x, uv.y, P.co_depth[o], e, jc, jp, jk);
                cam_accum_u(acc, jc, e.f, e.ok ? e.cost : __builtin_nan(""), ac >= 0);
            }
            wave_scatter<CAM_NZ_U>(acc, lane, [&](int i, double v) { wo[cam_nz_u_index(i)] = v; });
        }
        {
            double acc[CAM_NZ_C];
#pragma unroll
            for (int i = 0; i < CAM_NZ_C; ++i) acc[i] = 0.0;
            for (int o = o0 + lane; o < o1; o += 64) {
                const double2 uv = P.co_uv[o];
                ObsEval e;
                double jc[18], jp[9], jk[8];
                lin_obs(c, pose, pts + 3 * P.co_pt[o], K, uv.x, uv.y, P.co_depth[o], e, jc, jp, jk);
                cam_accum_c(acc, jc, jk, e.f, ac >= 0);
            }
            wave_scatter<CAM_NZ_C>(acc, lane, [&](int i, double v) { wo[cam_nz_c_index(i)] = v; });
        }
        wave_sync();
        for (int e = lane; e < CAMDATA + SEGINTR; e += 64) {
            const double v = cam_unpack(wo, e);
            if (e < CAMDATA) {
                if (ac >= 0) W.camdata_part[(size_t)s * CAMDATA + e] = v;
            } else {
                W.seg_intr[(size_t)s * SEGINTR + e - CAMDATA] = v;
            }
        }
        wave_sync();
    }
    // point side: one point per thread (k_point_prep's sums) + W_o of its active-camera observations
    double gmax = 0.0;
    const double one[6] = {1.0, 1.0, 1.0, 1.0, 1.0, 1.0};
    double* __restrict__ wcs = W.sm.wc;
    double* __restrict__ pvs = W.sm.pv;
    for (int ap = tid; ap < P.n_ap; ap += NT) {
        const double* X = pts + 3 * P.pt_idx[ap];
        double acc[21];
#pragma unroll
        for (int i = 0; i < 21; ++i) acc[i] = 0.0;
        for (int o = P.pt_ptr[ap]; o < P.pt_ptr[ap + 1]; ++o) {
            const double2 uv = P.po_uv[o];
            ObsEval ev;
            double jc[18], jp[9], jk[8];
            lin_obs(c, cams + 7 * P.po_cam[o], X, K, uv.x, uv.y, P.po_depth[o], ev, jc, jp, jk);
            acc[0] += jp[0] * jp[0] + jp[3] * jp[3] + jp[6] * jp[6];
            acc[1] += jp[0] * jp[1] + jp[3] * jp[4] + jp[6] * jp[7];
            acc[2] += jp[0] * jp[2] + jp[3] * jp[5] + jp[6] * jp[8];
            acc[3] += jp[1] * jp[1] + jp[4] * jp[4] + jp[7] * jp[7];
            acc[4] += jp[1] * jp[2] + jp[4] * jp[5] + jp[7] * jp[8];
            acc[5] += jp[2] * jp[2] + jp[5] * jp[5] + jp[8] * jp[8];
#pragma unroll
            for (int i = 0; i < 3; ++i) acc[6 + i] += jp[i] * ev.f[0] + jp[3 + i] * ev.f[1] + jp[6 + i] * ev.f[2];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                acc[9 + 0 * 3 + i] += jk[0] * jp[i];
                acc[9 + 1 * 3 + i] += jk[5] * jp[3 + i];
                acc[9 + 2 * 3 + i] += jk[2] * jp[i];
                acc[9 + 3 * 3 + i] += jk[7] * jp[3 + i];
            }
            if (P.po_ac[o] >= 0) {
                double w[18];
                w_tilde(jc, jp, one, one, w);  // unscaled: the step scales it (s_c W_o s_p)
                double* dst = wcs + (size_t)o * 18;
#pragma unroll
                for (int i = 0; i < 18; ++i) dst[i] = w[i];
            }
        }
        double* pv = pvs + (size_t)ap * 21;
#pragma unroll
        for (int i = 0; i < 21; ++i) pv[i] = acc[i];
#pragma unroll
        for (int i = 0; i < 3; ++i) gmax = fmax(gmax, fabs(X[i] - (X[i] + -acc[6 + i])));
    }
    gmax = block_max_nw<NW>(gmax, L.red);  // (barriers inside: the partials above are complete)
    if (tid == 0) L.gmax_pt = gmax;
    // camera sums in sub-segment order; intrinsics partials in segment order
    for (int e = tid; e < P.nac * CAMDATA; e += NT) {
        const int ac = e / CAMDATA, v = e - ac * CAMDATA;
        const int2 r = P.ac_seg[ac];
        double a = 0.0;
        for (int sg = r.x; sg < r.y; ++sg) a += W.camdata_part[(size_t)sg * CAMDATA + v];
        W.camdata[e] = a;
    }
    if (tid < SEGINTR) {
        double a = 0.0;
        for (int sg = 0; sg < P.n_seg; ++sg) a += W.seg_intr[(size_t)sg * SEGINTR + tid];
        L.io[tid] = a;
    }
    __syncthreads();
    double gm = 0.0;
    for (int ac = tid; ac < P.nac; ac += NT) gm = fmax(gm, cam_gmax(P, cur, ac, W.camdata + (size_t)ac * CAMDATA + 45));
    gm = block_max_nw<NW>(gm, L.red);
    if (tid == 0) {
        const double gk = intr_lin(P, c, K, L.io, L.lin);
        L.lin[1] = fmax(gm, gk);
        for (int q = 0; q < LIN_N; ++q) W.lin[q] = L.lin[q];
    }
    __syncthreads();
}

// ---------------------------------------------------------------- reduced system in LDS
// S (lower, stride ld) + rhs: the damped, scaled camera / intrinsics blocks, border and pad identity
// (env_tile's element formula, one landmark shard), then the points' intrinsics Schur sums.
__device__ __forceinline__ void small_assemble(const DevProblem& P, const BaConsts& c, const DevWork& W, SmallLds& L, double* S, int ld,
                               double radius, const double (&kk)[14]) {
    const int tid = threadIdx.x;
    const int npad = P.npad, nd = 6 * P.nac, kb = P.kb;
    const double* scale = W.scale;
    const double* sk = scale + P.off_k;
    const double* cd = W.camdata;
    for (int e = tid; e < npad * npad; e += NT) {
        const int r = e / npad, col = e - r * npad;
        if (col > r) continue;
        double v = 0.0;
        if (r < nd && r / 6 == col / 6) {
            const int ac = r / 6, i = col - 6 * ac, j = r - 6 * ac;
            const int q = 6 * i - i * (i - 1) / 2 + (j - i);
            const double* sc = scale + 6 * ac;
            v = sc[i] * cd[(size_t)ac * CAMDATA + q] * sc[j];
            if (i == j) v += fmin(fmax(v, c.min_diag), c.max_diag) / radius;
        } else if (r >= kb && r < kb + 4 && col < nd) {
            const int m = r - kb, ac = col / 6, i = col - 6 * ac;
            v = scale[6 * ac + i] * cd[(size_t)ac * CAMDATA + 21 + i * 4 + m] * sk[m];
        } else if (r >= kb && r < kb + 4 && col >= kb && col <= r) {
            const int m = col - kb, l = r - kb;
            const int q = 4 * m - m * (m - 1) / 2 + (l - m);
            v = sk[m] * L.lin[2 + q] * sk[l];
            if (l == m) v += fmin(fmax(v, c.min_diag), c.max_diag) / radius;
        } else if (r == col && r >= P.n) {
            v = 1.0;
        }
        S[r * ld + col] = v;
    }
    for (int r = tid; r < npad; r += NT) {
        double b = 0.0;
        if (r < nd) b = scale[r] * cd[(size_t)(r / 6) * CAMDATA + 45 + r % 6];
        else if (r < kb + 4) b = sk[r - kb] * L.lin[12 + r - kb];
        L.yv[r] = b;
    }
    double v[14];
#pragma unroll
    for (int q = 0; q < 14; ++q) v[q] = kk[q];
    block_sum_nw<NW, 14>(v, L.red, L.kk);  // (barriers inside: the envelope above is complete)
    if (tid < 10) {
        int m = 0, q = tid;
        while (q >= 4 - m) { q -= 4 - m; ++m; }
        S[(kb + m + q) * ld + kb + m] += L.kk[tid];
    } else if (tid < 14) {
        L.yv[kb + tid - 10] += L.kk[tid];
    }
}

// Points' Schur terms, one task per wave at a time (kind 0: camera-pair block, kind 1: border rows). The
// lanes take the task's observation pairs at a fixed stride, the wave reduce-scatters, and the wave alone
// writes the task's elements: no atomics, bitwise reproducible. (One thread per element with a serial loop
// over the entries measured 9x slower: every entry is a dependent L2 round trip.)
__device__ __forceinline__ void small_tasks(const DevProblem& P, const DevWork& W, double* S, int ld, double* yv) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const SmallWork& Z = W.sm;
    for (int t = wave; t < Z.n_task; t += NW) {
        const int4 tk = Z.task[t];
        const int e1 = Z.task_end[t];
        if (tk.z == 0) {
            double acc[36];
#pragma unroll
            for (int i = 0; i < 36; ++i) acc[i] = 0.0;
            for (int q = tk.w + lane; q < e1; q += 64) {
                const int2 uv = Z.entry[q];
                const double* zu = Z.zb + (size_t)uv.x * 18;
                const double* zv = Z.zb + (size_t)uv.y * 18;
                double a[18], b[18];
#pragma unroll
                for (int i = 0; i < 18; ++i) { a[i] = zu[i]; b[i] = zv[i]; }
#pragma unroll
                for (int d = 0; d < 6; ++d)
#pragma unroll
                    for (int e = 0; e < 6; ++e)
                        acc[d * 6 + e] += a[d * 3] * b[e * 3] + a[d * 3 + 1] * b[e * 3 + 1] + a[d * 3 + 2] * b[e * 3 + 2];
            }
            const int ra = 6 * tk.x, cb = 6 * tk.y;
            const bool diag = tk.x == tk.y;
            wave_scatter<36>(acc, lane, [&](int i, double v) {
                const int d = i / 6, e = i - 6 * d;
                if (!diag || e <= d) S[(ra + d) * ld + cb + e] -= v;
            });
        } else {
            double acc[30];
#pragma unroll
            for (int i = 0; i < 30; ++i) acc[i] = 0.0;
            for (int q = tk.w + lane; q < e1; q += 64) {
                const int u = Z.entry[q].x;
                const double* zu = Z.zb + (size_t)u * 18;
                const double* zp = Z.zk + (size_t)P.po_ap[u] * 15;
                double a[18], k[15];
#pragma unroll
                for (int i = 0; i < 18; ++i) a[i] = zu[i];
#pragma unroll
                for (int i = 0; i < 15; ++i) k[i] = zp[i];
#pragma unroll
                for (int m = 0; m < 4; ++m)
#pragma unroll
                    for (int d = 0; d < 6; ++d)
                        acc[m * 6 + d] += k[m * 3] * a[d * 3] + k[m * 3 + 1] * a[d * 3 + 1] + k[m * 3 + 2] * a[d * 3 + 2];
#pragma unroll
                for (int d = 0; d < 6; ++d)
                    acc[24 + d] += a[d * 3] * k[12] + a[d * 3 + 1] * k[13] + a[d * 3 + 2] * k[14];
            }
            const int ca = 6 * tk.x, kb = P.kb;
            wave_scatter<30>(acc, lane, [&](int i, double v) {
                if (i < 24) S[(kb + i / 6) * ld + ca + i % 6] -= v;
                else yv[ca + i - 24] -= v;
            });
        }
    }
}

// Cholesky of S (npad <= SMALL_NPAD, lower, stride ld) with the forward substitution fused
// (L z = b on the fly), then L^T y = z; y overwrites L.yv. Sets L.bad on a non-positive pivot.
template <bool STAMP>
__device__ __forceinline__ void small_cholesky(const DevProblem& P, SmallLds& L, double* S, int ld,
                                               unsigned long long* sacc) {
    unsigned long long tp = 0;
    auto mark = [&](int k) {
        if constexpr (STAMP) {
            __syncthreads();
            if (threadIdx.x == 0) {
                const unsigned long long t = small_clock();
                if (tp) sacc[k] += t - tp;
                tp = t;
            }
        }
    };
    mark(0);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rr = lane & 15, kq = lane >> 4;
    const int npad = P.npad, nb = npad / 16;
    bool bad = false;
    for (int kb = 0; kb < nb; ++kb) {
        const int k0 = 16 * kb;
        if (wave == 0) {
            // Pivot chain over the tall column block (rows k0 .. k0 + 63 on the 64 lanes): the diagonal tile and
            // the row panels below it in one pass, with the forward substitution (L z = b) fused: per pivot one
            // broadcast of the next pivot, v_rsq_f64 + one Newton step folded into l = a y (1 + e / 2), and the
            // next pivot's diagonal updated first (the k_bcr_split chain).
            const int row = k0 + lane;
            const bool live = row < npad;
            double a[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) a[j] = (live && (lane >= 16 || j <= lane)) ? S[row * ld + k0 + j] : 0.0;
            double yr = live ? L.yv[row] : 0.0;
            double my_inv = 0.0;
            double dn = bcast(a[0], 0);
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const double d = dn;
                bad = bad || !(d > 0.0 && d < INFINITY);
                const double y = __builtin_amdgcn_rsq(d);
                const double e = __builtin_fma(-d * y, y, 1.0);
                const double l = __builtin_fma(0.5 * a[j] * y, e, a[j] * y);
                const double inv = __builtin_fma(0.5 * y, e, y);
                my_inv = (lane == j) ? inv : my_inv;
                a[j] = l;
                const double zj = bcast(yr, j) * inv;
                yr = (lane == j) ? zj : (lane > j ? __builtin_fma(-l, zj, yr) : yr);
                if (j < 15) {
                    dn = bcast(__builtin_fma(-l, l, a[j + 1]), j + 1);
#pragma unroll
                    for (int k = j + 1; k < 16; ++k) a[k] = __builtin_fma(-l, bcast(l, k), a[k]);
                }
            }
            if (live) {
#pragma unroll
                for (int j = 0; j < 16; ++j) S[row * ld + k0 + j] = (lane >= 16 || j <= lane) ? a[j] : 0.0;
                L.yv[row] = yr;
            }
            if (lane < 16) L.rdiag[k0 + lane] = my_inv;
        }
        __syncthreads();
        mark(SST_CH_POTRF);
        // rows beyond the tall block (npad > k0 + 64): L_ik = A_ik L_kk^-T and their rhs update
        const int r0 = k0 + 64;
        if (r0 < npad) {
            for (int i = r0 + tid; i < npad; i += NT) {
                double x[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) x[j] = S[i * ld + k0 + j];
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    x[m] *= L.rdiag[k0 + m];
#pragma unroll
                    for (int j = m + 1; j < 16; ++j) x[j] -= x[m] * S[(k0 + j) * ld + k0 + m];
                }
                double sacc = 0.0;
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    S[i * ld + k0 + j] = x[j];
                    sacc += x[j] * L.yv[k0 + j];
                }
                L.yv[i] -= sacc;
            }
            __syncthreads();
        }
        mark(SST_CH_TRSM);
        // trailing tiles (ii, jj), kb < jj <= ii < nb, on the f64 matrix cores
        const int nr = nb - kb - 1, ntr = nr * (nr + 1) / 2;
        for (int t = wave; t < ntr; t += NW) {
            int p = 0, q = t;
            while (q > p) { q -= p + 1; ++p; }
            const int ii = 16 * (kb + 1 + p), jj = 16 * (kb + 1 + q);
            d4s acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s4 = 0; s4 < 4; ++s4)
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(S[(ii + rr) * ld + k0 + 4 * s4 + kq],
                                                           S[(jj + rr) * ld + k0 + 4 * s4 + kq], acc, 0, 0, 0);
#pragma unroll
            for (int g = 0; g < 4; ++g) S[(ii + kq + 4 * g) * ld + jj + rr] -= acc[g];
        }
        __syncthreads();
        mark(SST_CH_MFMA);
    }
    if (wave == 0) {
        const unsigned long long any = __ballot(bad);
        if (lane == 0 && any) L.bad = 1;
    }
    // backward: y_kb = L_kk^-T (z_kb - sum_{i >= k0 + 16} L_i,kb^T y_i)
    for (int kb = nb - 1; kb >= 0; --kb) {
        const int k0 = 16 * kb;
        {
            const int r = tid & 15, p = tid >> 4;  // 32 parts
            double s = 0.0;
            for (int i = k0 + 16 + p; i < npad; i += NT / 16) s += S[i * ld + k0 + r] * L.yv[i];
            L.red[p * 16 + r] = s;
        }
        __syncthreads();
        if (wave == 0) {
            double v = L.yv[k0 + rr];
            for (int p = 0; p < NT / 16; ++p) v -= L.red[p * 16 + rr];
#pragma unroll
            for (int m = 15; m >= 0; --m) {
                const double ym = bcast(v, m) * L.rdiag[k0 + m];
                if (rr < m) v -= S[(k0 + m) * ld + k0 + rr] * ym;
                if (rr == m) v = ym;
            }
            if (lane < 16) L.yv[k0 + rr] = v;
        }
        __syncthreads();
    }
    mark(SST_CH_BACK);
}


template <bool STAMP>
__global__ __launch_bounds__(NT) void k_small_solve(DevProblem P, BaConsts c, DevWork W, LmParams prm, int jacobi,
                                                    unsigned long long* __restrict__ stamps) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    unsigned long long t_prev = 0, st_acc[SST_N] = {};
#define SSTAMP(k)                                                   \
    do {                                                            \
        if constexpr (STAMP) {                                      \
            __syncthreads();                                        \
            if (threadIdx.x == 0) {                                 \
                const unsigned long long t_ = small_clock();        \
                st_acc[k] += t_ - t_prev;                           \
                t_prev = t_;                                        \
            }                                                       \
        }                                                           \
    } while (0)
    if constexpr (STAMP) if (threadIdx.x == 0) t_prev = small_clock();
    SmallLds& L = *reinterpret_cast<SmallLds*>(smem);
    double* S = reinterpret_cast<double*>(smem + sizeof(SmallLds));
    const int ld = P.npad + 1;
    const int tid = threadIdx.x;
    // ---- iteration 0: linearisation, Jacobi scale, |x|^2, initial state (k_cam_finalize, k_scale,
    //      k_xnorm_part / k_xnorm_init of the multi-launch path)
    int cur = W.st->cur;
    small_linearize(P, c, W, L, cur);
    SSTAMP(SST_LIN);
    {
        const int ncam = 6 * P.nac, npt = 3 * P.n_ap;
        for (int t = tid; t < ncam + npt + 4; t += NT) {
            double cn;
            int dst;
            if (t < ncam) {
                const int ac = t / 6, d = t % 6;
                cn = W.camdata[(size_t)ac * CAMDATA + d * 6 - (d * (d - 1)) / 2];
                dst = t;
            } else if (t < ncam + npt) {
                const int ap = (t - ncam) / 3, i = (t - ncam) % 3;
                cn = W.sm.pv[(size_t)ap * 21 + (i == 0 ? 0 : (i == 1 ? 3 : 5))];
                dst = P.off_pt + (t - ncam);
            } else {
                const int m = t - ncam - npt;
                cn = L.lin[2 + m * 4 - (m * (m - 1)) / 2];
                dst = P.off_k + m;
            }
            W.scale[dst] = jacobi ? 1.0 / (1.0 + sqrt(cn)) : 1.0;
        }
        double a[1] = {0.0};
        for (int ac = tid; ac < P.nac; ac += NT) {
            const double* x = P.cams[cur] + 7 * P.ac_cam[ac];
#pragma unroll
            for (int j = 0; j < 7; ++j) a[0] += x[j] * x[j];
        }
        for (int ap = tid; ap < P.n_ap; ap += NT) {
            const double* x = P.pts[cur] + 3 * P.pt_idx[ap];
            a[0] += x[0] * x[0] + x[1] * x[1] + x[2] * x[2];
        }
        block_sum_nw<NW, 1>(a, L.red, L.kk);
        if (tid == 0) {
            LmState* st = W.st;
            const double* K = P.K[cur];
            st->xnorm2 = L.kk[0] + K[0] * K[0] + K[1] * K[1] + K[2] * K[2] + K[3] * K[3];
            st->x_cost = L.lin[0];
            st->initial_cost = L.lin[0];
            st->final_cost = L.lin[0];
            st->gmax_ci = L.lin[1];
            double* log = W.log;
            log[0] = L.lin[0]; log[1] = 0.0; log[3] = 0.0; log[4] = 0.0; log[5] = st->radius; log[6] = 1.0;
            if (!isfinite(L.lin[0])) {
                st->done = 1;
                st->termination = 2;  // FAILURE
                st->msg = MSG_EVAL_FAIL;
            }
        }
    }
    SSTAMP(SST_INIT);
    // ---- LM iterations
    for (;;) {
        __syncthreads();
        if (tid == 0) L.st = *W.st;
        __syncthreads();
        if (L.st.done) break;
        cur = L.st.cur;
        if (L.st.need_lin) small_linearize(P, c, W, L, cur);
        SSTAMP(SST_LIN);
        double scal[SC_N];
#pragma unroll
        for (int i = 0; i < SC_N; ++i) scal[i] = 0.0;
        if (!L.st.stop_next) {
            const double radius = L.st.radius;
            // point records (G, e~, K~, D~) and Zk | ze, one point per thread
            double kk[14];
#pragma unroll
            for (int q = 0; q < 14; ++q) kk[q] = 0.0;
            double pbad = 0.0;
            {
                const double* __restrict__ pts = P.pts[cur];
                const double* __restrict__ pvs = W.sm.pv;
                double* __restrict__ pdata = W.pdata;
                double* __restrict__ zks = W.sm.zk;
                for (int ap = tid; ap < P.n_ap; ap += NT) {
                    const double* X = pts + 3 * P.pt_idx[ap];
                    double pv[21];
#pragma unroll
                    for (int i = 0; i < 21; ++i) pv[i] = pvs[(size_t)ap * 21 + i];
                    double rec[PDATA], kp[14], gdummy = 0.0;
                    point_tail(P, c, radius, W.scale, ap, X, pv, true, rec, kp, gdummy, pbad);
#pragma unroll
                    for (int i = 0; i < PDATA; ++i) pdata[(size_t)ap * PDATA + i] = rec[i];
#pragma unroll
                    for (int q = 0; q < 14; ++q) kk[q] += kp[q];
                    double zkp[12], zep[3];
                    zk_ze(rec, rec + 9, rec + 6, zkp, zep);
#pragma unroll
                    for (int i = 0; i < 12; ++i) zks[(size_t)ap * 15 + i] = zkp[i];
#pragma unroll
                    for (int i = 0; i < 3; ++i) zks[(size_t)ap * 15 + 12 + i] = zep[i];
                }
            }
            pbad = block_max_nw<NW>(pbad, L.red);  // (barriers inside: point records complete)
            // Z_o = W~_o G^T, one observation per thread (W~ = s_c W_o s_p, the k_schur_tile formula)
            {
                const double* __restrict__ wcs = W.sm.wc;
                const double* __restrict__ pdata = W.pdata;
                const double* __restrict__ scale = W.scale;
                double* __restrict__ zb = W.sm.zb;
                for (int o = tid; o < P.n_adm; o += NT) {
                    const int ac = P.po_ac[o];
                    if (ac < 0) continue;
                    const int ap = P.po_ap[o];
                    double wc[18], sc[6], sp[3], g[6];
#pragma unroll
                    for (int i = 0; i < 18; ++i) wc[i] = wcs[(size_t)o * 18 + i];
#pragma unroll
                    for (int i = 0; i < 6; ++i) sc[i] = scale[6 * ac + i];
#pragma unroll
                    for (int i = 0; i < 3; ++i) sp[i] = scale[P.off_pt + 3 * ap + i];
#pragma unroll
                    for (int i = 0; i < 6; ++i) g[i] = pdata[(size_t)ap * PDATA + i];
#pragma unroll
                    for (int d = 0; d < 6; ++d) {
                        const double w0 = sc[d] * wc[d * 3 + 0] * sp[0];
                        const double w1 = sc[d] * wc[d * 3 + 1] * sp[1];
                        const double w2 = sc[d] * wc[d * 3 + 2] * sp[2];
                        zb[(size_t)o * 18 + d * 3 + 0] = w0 * g[0];
                        zb[(size_t)o * 18 + d * 3 + 1] = w0 * g[1] + w1 * g[2];
                        zb[(size_t)o * 18 + d * 3 + 2] = w0 * g[3] + w1 * g[4] + w2 * g[5];
                    }
                }
            }
            if (tid == 0) L.bad = 0;
            SSTAMP(SST_POINT);
            small_assemble(P, c, W, L, S, ld, radius, kk);  // (barrier inside before its S_kk adds)
            SSTAMP(SST_ASSEMBLE);
            small_tasks(P, W, S, ld, L.yv);
            __syncthreads();
            SSTAMP(SST_TASKS);
            small_cholesky<STAMP>(P, L, S, ld, st_acc);
            SSTAMP(SST_CHOL);
            // camera / intrinsics step and their step-scalar terms
            double acc4[4] = {0.0, 0.0, 0.0, 0.0};  // |step|^2, model cost change, candidate cost, |x_cand|^2
            if (tid < P.nac) update_camera(P, c, cur, radius, W.scale, W.camdata, tid, L.yv + 6 * tid, W.delta, acc4);
            else if (tid == P.nac) update_intrinsics(P, c, cur, radius, W.scale, W.lin, L.yv + P.kb, W.delta, acc4);
            // back-substitution terms s_p W_o^T (s_c y_c), one observation per thread (into the Z slots)
            {
                const double* __restrict__ wcs = W.sm.wc;
                const double* __restrict__ scale = W.scale;
                double* __restrict__ cb = W.sm.zb;
                for (int o = tid; o < P.n_adm; o += NT) {
                    const int ac = P.po_ac[o];
                    if (ac < 0) continue;
                    const int ap = P.po_ap[o];
                    double wc[18], sy[6];
#pragma unroll
                    for (int i = 0; i < 18; ++i) wc[i] = wcs[(size_t)o * 18 + i];
#pragma unroll
                    for (int d = 0; d < 6; ++d) sy[d] = scale[6 * ac + d] * L.yv[6 * ac + d];
#pragma unroll
                    for (int i = 0; i < 3; ++i) {
                        double v = 0.0;
#pragma unroll
                        for (int d = 0; d < 6; ++d) v += wc[d * 3 + i] * sy[d];
                        cb[(size_t)o * 18 + i] = scale[P.off_pt + 3 * ap + i] * v;
                    }
                }
            }
            __syncthreads();  // candidate cameras / intrinsics and the back-substitution terms visible
            SSTAMP(SST_CAMS);
            // points: y_p = V~^-1 (e~ - K~^T y_k - sum_o c_o), the update and its step-scalar terms
            {
                const double* __restrict__ pdata = W.pdata;
                const double* __restrict__ cb = W.sm.zb;
                const double* __restrict__ pts = P.pts[cur];
                double* __restrict__ ptn = P.pts[cur ^ 1];
                const double* yk = L.yv + P.kb;
                for (int ap = tid; ap < P.n_ap; ap += NT) {
                    const int pi = P.pt_idx[ap];
                    double pd[PDATA], X[3];
#pragma unroll
                    for (int i = 0; i < PDATA; ++i) pd[i] = pdata[(size_t)ap * PDATA + i];
#pragma unroll
                    for (int i = 0; i < 3; ++i) X[i] = pts[3 * pi + i];
                    const double* sp = W.scale + P.off_pt + 3 * ap;
                    double t[3];
#pragma unroll
                    for (int i = 0; i < 3; ++i)
                        t[i] = pd[6 + i] - (pd[9 + 0 * 3 + i] * yk[0] + pd[9 + 1 * 3 + i] * yk[1] +
                                            pd[9 + 2 * 3 + i] * yk[2] + pd[9 + 3 * 3 + i] * yk[3]);
                    const int o0 = P.pt_ptr[ap], o1 = P.pt_ptr[ap + 1];
                    for (int o = o0; o < o1; ++o) {
                        if (P.po_ac[o] < 0) continue;
#pragma unroll
                        for (int i = 0; i < 3; ++i) t[i] -= cb[(size_t)o * 18 + i];
                    }
                    double Vf[9];
                    vinv_from_g(pd, Vf);
#pragma unroll
                    for (int i = 0; i < 3; ++i) {
                        const double yp = Vf[i * 3 + 0] * t[0] + Vf[i * 3 + 1] * t[1] + Vf[i * 3 + 2] * t[2];
                        acc4[1] += 0.5 * (pd[6 + i] * yp + pd[21 + i] * yp * yp);
                        const double xn = X[i] + -sp[i] * yp;
                        ptn[3 * pi + i] = xn;
                        const double df = X[i] - xn;
                        acc4[0] += df * df;
                        acc4[3] += xn * xn;
                    }
                }
            }
            __syncthreads();  // candidate points visible
            // candidate cost, one observation per thread
            double cbad = 0.0;
            {
                const double* __restrict__ ptn = P.pts[cur ^ 1];
                const double* __restrict__ camn = P.cams[cur ^ 1];
                const double* Kn = P.K[cur ^ 1];
                for (int o = tid; o < P.n_adm; o += NT) {
                    const double2 uv = P.po_uv[o];
                    ObsEval en;
                    eval_obs(c, camn + 7 * P.po_cam[o], ptn + 3 * P.po_pt[o], Kn, uv.x, uv.y, P.po_depth[o], en);
                    if (en.ok) acc4[2] += en.cost; else cbad = 1.0;
                }
            }
            if (!isfinite(acc4[0]) || !isfinite(acc4[1])) cbad = 1.0;
            block_sum_nw<NW, 4>(acc4, L.red, L.kk);
            cbad = block_max_nw<NW>(cbad, L.red);
            scal[SC_SN2] = L.kk[0];
            scal[SC_MCC] = L.kk[1];
            scal[SC_CAND] = L.kk[2];
            scal[SC_XN2] = L.kk[3];
            scal[SC_BAD] = fmax(cbad, 2.0 * pbad) + (L.bad ? 4.0 : 0.0);  // as k_final
            SSTAMP(SST_BACKSUB);
        }
        scal[SC_GMAX_PT] = L.gmax_pt;
        __syncthreads();
        if (tid == 0) {
            for (int i = 0; i < SC_N; ++i) W.scal[i] = scal[i];
            lm_decide_body(W.st, prm, W.lin, W.scal, W.log);
        }
        SSTAMP(SST_DECIDE);
    }
    if constexpr (STAMP)
        if (threadIdx.x == 0)
            for (int k = 0; k < SST_N; ++k) stamps[k] = st_acc[k];
#undef SSTAMP
}

hipError_t launch_small(const DevProblem& P, const BaConsts& c, const LmParams& prm, int jacobi, DevWork& W,
                        hipStream_t s, Prof* pf) {
    const size_t lds = small_lds_bytes(P.npad);
    static size_t attr = 0;
    static int stamp_mode = -1;
    static unsigned long long* dst = nullptr;
    if (lds > attr) {
        hipError_t e = hipFuncSetAttribute((const void*)k_small_solve<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)lds);
        if (e == hipSuccess)
            e = hipFuncSetAttribute((const void*)k_small_solve<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        attr = lds;
    }
    if (stamp_mode < 0) {
        const char* e = getenv("MIBA_SMALL_STAMPS");
        stamp_mode = (e && e[0] == '1') ? 1 : 0;
    }
    if (stamp_mode == 1) {
        if (!dst) {
            hipError_t e = hipMalloc(&dst, sizeof(unsigned long long) * SST_N);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k_small_solve<true>, dim3(1), dim3(NT), lds, s, P, c, W, prm, jacobi, dst);
        unsigned long long h[SST_N];
        hipError_t e = hipMemcpyAsync(h, dst, sizeof(h), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
        static const char* names[SST_N] = {"init", "linearize", "point", "assemble", "tasks", "cholesky", "cams",
                                           "backsub+eval", "decide", "[ch potrf", "ch trsm", "ch mfma", "ch back]"};
        fprintf(stderr, "small_solve cycles:");
        for (int k = 0; k < SST_N; ++k) fprintf(stderr, " %s %llu", names[k], h[k]);
        fprintf(stderr, "\n");
        return hipSuccess;
    }
    if (pf) pf->begin(K_SMALL, s);
    hipLaunchKernelGGL(k_small_solve<false>, dim3(1), dim3(NT), lds, s, P, c, W, prm, jacobi,
                       (unsigned long long*)nullptr);
    if (pf) pf->end(s);
    return hipGetLastError();
}

}  // namespace miba
