// ba_common.h — device-side helpers shared by the libmiba kernel translation units
// (ba_kernels.hip: the LM iteration; ba_bcr.hip: the reduced camera solve): reductions, the per-point
// Schur algebra, the in-register 16x16 Cholesky and the Ceres 2.0 trust-region decision.
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstddef>

#include "ba_device.h"
#include "ba_kernels.h"
#include "ba_solve_util.h"

namespace miba {

// ---------------------------------------------------------------- reductions
// The xor butterfly (ds_bpermute per step and half). Kept for the block sums of the kernels instantiated for both
// observation layouts (k_point_prep, k_backsub_chunk, the Schur tiles' intrinsics workgroup): with the DPP sum there,
// the obs32 and f64 instantiations of a deterministic solve stopped agreeing in the last bit
// (test_obs32_records_match_f64_arrays_bitwise, bisected to ba_tail.h's block_sum), for a reason not found.
template <int NV>
__device__ __forceinline__ void wave_sum(double (&v)[NV]) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] += __shfl_xor(v[i], off);
}
// DPP wave sums: the decision's reductions (block_sum_nw) and the band tail's chunk sums (block_sum_dpp)
template <int NV>
__device__ __forceinline__ void wave_sum_dpp(double (&v)[NV]) {
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = dpp_wave_sum(v[i]);
}

// Wave reduce-scatter by recursive halving: at the step with lane offset OFF a lane keeps
// one half of its N running sums (chosen by lane bit OFF) and adds its partner's copy of
// that half, so N values cost N/2 + N/4 + ... shuffles instead of 6 N. Afterwards lane l
// holds the wave sums of indices [base, base + len).
template <int N, int OFF>
struct WaveHalve {
    static __device__ __forceinline__ void run(double* v, int lane, int& base, int& len) {
        constexpr int H = (N + 1) / 2;
        const bool hi = (lane & OFF) != 0;
#pragma unroll
        for (int i = 0; i < H; ++i) {
            const double a = v[i];
            const double b = (i + H < N) ? v[i + H] : 0.0;
            const double keep = hi ? b : a;
            const double send = hi ? a : b;
            v[i] = keep + __shfl_xor(send, OFF);
        }
        if (hi) { base += H; len = len - H; } else { len = len < H ? len : H; }
        WaveHalve<H, OFF / 2>::run(v, lane, base, len);
    }
};

template <int N>
struct WaveHalve<N, 0> {
    static constexpr int kRemain = N;
    static __device__ __forceinline__ void run(double*, int, int&, int&) {}
};

template <int N, int OFF>
struct HalveRemain { static constexpr int value = HalveRemain<(N + 1) / 2, OFF / 2>::value; };

template <int N>
struct HalveRemain<N, 0> { static constexpr int value = N; };

// NW-wave variants (k_final runs 16 waves); lds holds NW * NV doubles. Wave sums added in wave order.
template <int NW, int NV>
__device__ __forceinline__ void block_sum_nw(double (&v)[NV], double* lds, double* out) {
    wave_sum_dpp<NV>(v);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) lds[wave * NV + i] = v[i];
    __syncthreads();
    if (threadIdx.x < NV) {
        double a = lds[threadIdx.x];
#pragma unroll
        for (int w = 1; w < NW; ++w) a += lds[w * NV + threadIdx.x];
        out[threadIdx.x] = a;
    }
    __syncthreads();
}

template <int NW>
__device__ __forceinline__ double block_max_nw(double v, double* lds) {
    v = dpp_wave_max(v);
    if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = lds[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) r = fmax(r, lds[w]);
    __syncthreads();
    return r;
}

// ---------------------------------------------------------------- point side
// G = L^-1 of the damped point block, packed lower (g00 g10 g11 g20 g21 g22).
__device__ __forceinline__ void zk_ze(const double G[6], const double Ks[12], const double es[3], double Zk[12],
                                      double ze[3]) {
    // Zk[m][k] = sum_{i<=k} K[m][i] G[k][i] ; ze[k] = sum_{i<=k} G[k][i] e[i]
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        Zk[m * 3 + 0] = Ks[m * 3 + 0] * G[0];
        Zk[m * 3 + 1] = Ks[m * 3 + 0] * G[1] + Ks[m * 3 + 1] * G[2];
        Zk[m * 3 + 2] = Ks[m * 3 + 0] * G[3] + Ks[m * 3 + 1] * G[4] + Ks[m * 3 + 2] * G[5];
    }
    ze[0] = G[0] * es[0];
    ze[1] = G[1] * es[0] + G[2] * es[1];
    ze[2] = G[3] * es[0] + G[4] * es[1] + G[5] * es[2];
}

// V~^-1 = G^T G (full 3x3)
__device__ __forceinline__ void vinv_from_g(const double* G, double Vf[9]) {
    const double g00 = G[0], g10 = G[1], g11 = G[2], g20 = G[3], g21 = G[4], g22 = G[5];
    Vf[0] = g00 * g00 + g10 * g10 + g20 * g20;
    Vf[1] = g10 * g11 + g20 * g21;
    Vf[2] = g20 * g22;
    Vf[4] = g11 * g11 + g21 * g21;
    Vf[5] = g21 * g22;
    Vf[8] = g22 * g22;
    Vf[3] = Vf[1]; Vf[6] = Vf[2]; Vf[7] = Vf[5];
}

// W~ (6x3) = s_c (Jc^T Jp) s_p  for one observation
__device__ __forceinline__ void w_tilde(const double jc[18], const double jp[9], const double* sc, const double* sp,
                                        double W[18]) {
    // structural zeros of jc skipped (cam_accum, ba_device.h): rows 0 / 1 / 2 have 5 / 5 / 3 nonzeros
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const double p0 = jp[i], p1 = jp[3 + i], p2 = jp[6 + i];
        double w[6];
        w[0] = jc[0] * p0;
        w[1] = jc[7] * p1;
        w[2] = jc[2] * p0 + jc[8] * p1 + jc[14] * p2;
        w[3] = jc[3] * p0 + jc[9] * p1 + jc[15] * p2;
        w[4] = jc[4] * p0 + jc[10] * p1 + jc[16] * p2;
        w[5] = jc[5] * p0 + jc[11] * p1;
#pragma unroll
        for (int d = 0; d < 6; ++d) W[d * 3 + i] = sc[d] * w[d] * sp[i];
    }
}

// J_c v for the three rows (structural zeros skipped)
__device__ __forceinline__ void jc_times(const double jc[18], const double v[6], double out[3]) {
    out[0] = jc[0] * v[0] + jc[2] * v[2] + jc[3] * v[3] + jc[4] * v[4] + jc[5] * v[5];
    out[1] = jc[7] * v[1] + jc[8] * v[2] + jc[9] * v[3] + jc[10] * v[4] + jc[11] * v[5];
    out[2] = jc[14] * v[2] + jc[15] * v[3] + jc[16] * v[4];
}

// The camera's share of the gradient max-norm ||x - Plus(x, -g)||_inf (Ceres 2.0 trust_region_minimizer).
__device__ __forceinline__ double cam_gmax(const DevProblem& P, int cur, int ac, const double* g) {
    const double* x = P.cams[cur] + 7 * P.ac_cam[ac];
    double ng[6], tp[7];
#pragma unroll
    for (int d = 0; d < 6; ++d) ng[d] = -g[d];
    se3_plus(x, ng, tp);
    double gm = 0.0;
#pragma unroll
    for (int j = 0; j < 7; ++j) gm = fmax(gm, fabs(x[j] - tp[j]));
    return gm;
}

// Max-accumulate a non-negative double (its bit pattern orders like its value).
__device__ __forceinline__ void atomic_max_nonneg(double* p, double v) {
    atomicMax((unsigned long long*)p, (unsigned long long)__double_as_longlong(v));
}

// From the summed intrinsics partials out[SEGINTR] and the IntrinsicsPrior block (OptimizationUtils.cpp:
// 117-125, squared loss): lin16[0] = cost, lin16[2..12) = Ukk packed (+ prior), lin16[12..16) = gk (+ prior);
// returns the intrinsics' gradient max-norm term.
__device__ inline double intr_lin(const DevProblem& P, const BaConsts& c, const double* K, const double* out, double* lin16) {
    double pc = 0.0, gm = 0.0;
    double gk[4];
    for (int m = 0; m < 4; ++m) {
        const double fk = c.sw_k * (P.prior[m] - K[m]);
        pc += fk * fk;
        gk[m] = out[10 + m] + (-c.sw_k) * fk;
        gm = fmax(gm, fabs(K[m] - (K[m] + -gk[m])));
    }
    lin16[0] = out[14] + 0.5 * pc;
    for (int q = 0; q < 10; ++q) lin16[2 + q] = out[q];
    int q = 0;
    for (int m = 0; m < 4; ++m)
        for (int l = m; l < 4; ++l, ++q)
            if (l == m) lin16[2 + q] += c.sw_k * c.sw_k;
    for (int m = 0; m < 4; ++m) lin16[12 + m] = gk[m];
    return gm;
}

// Point tail of the Schur preparation, from the point's sums acc = V packed (6) | e (3) | Kt (12):
// gradient max-norm term, scaled + LM-damped V~, G = chol(V~)^-1, e~, K~, D~ -> rec[PDATA]; with
// want_kk also the intrinsics Schur terms -Zk Zk^T (10 packed), -Zk ze (4) -> kk.
// 1/sqrt(x) to full f64 precision: v_rsq_f64 + two Newton steps
__device__ __forceinline__ double rsqrt_nr(double x) {
    double y = __builtin_amdgcn_rsq(x);
    y = y * (1.5 - 0.5 * x * y * y);
    y = y * (1.5 - 0.5 * x * y * y);
    return y;
}

__device__ __forceinline__ void point_tail(const DevProblem& P, const BaConsts& c, double radius,
                                           const double* __restrict__ scale, int ap, const double* X,
                                           const double* acc, bool want_kk, double* rec, double* kk, double& gmax,
                                           double& bad) {
    const double* V = acc;
    const double* e = acc + 6;
    const double* Kt = acc + 9;
    // gradient max-norm contribution (points: x - (x + -g))
#pragma unroll
    for (int i = 0; i < 3; ++i) gmax = fmax(gmax, fabs(X[i] - (X[i] + -e[i])));
    const double* sp = scale + P.off_pt + 3 * ap;
    const double* sk = scale + P.off_k;
    const double s0 = sp[0], s1 = sp[1], s2 = sp[2];
    // scaled, damped V  (Ceres: lm_diagonal = sqrt(clamp(diag(JtJ~)) / radius))
    double v00 = s0 * V[0] * s0, v01 = s0 * V[1] * s1, v02 = s0 * V[2] * s2;
    double v11 = s1 * V[3] * s1, v12 = s1 * V[4] * s2, v22 = s2 * V[5] * s2;
    rec[21] = fmin(fmax(v00, c.min_diag), c.max_diag) / radius;  // D~ (model cost change, k_backsub_chunk)
    rec[22] = fmin(fmax(v11, c.min_diag), c.max_diag) / radius;
    rec[23] = fmin(fmax(v22, c.min_diag), c.max_diag) / radius;
    v00 += rec[21];
    v11 += rec[22];
    v22 += rec[23];
    // V~ = L L^T ; G = L^-1 (lower), V~^-1 = G^T G
#pragma unroll
    for (int i = 0; i < 6; ++i) rec[i] = 0.0;  // g00 g10 g11 g20 g21 g22
    // the pivots' reciprocal square roots by v_rsq_f64 + two Newton steps (rsqrt_nr) instead of IEEE square roots
    // and divisions: ~40 dependent operations on the point's chain instead of ~80
    const bool pd = v00 > 0.0;
    const double i00 = rsqrt_nr(v00);  // 1 / L00
    const double L10 = v01 * i00, L20 = v02 * i00;
    const double l11 = v11 - L10 * L10;
    const double i11 = rsqrt_nr(l11);
    const double L21 = (v12 - L20 * L10) * i11;
    const double l22 = v22 - L20 * L20 - L21 * L21;
    const double i22 = rsqrt_nr(l22);
    if (pd && l11 > 0.0 && l22 > 0.0 && isfinite(l22)) {
        rec[0] = i00;
        rec[1] = -L10 * i00 * i11;
        rec[2] = i11;
        rec[4] = -L21 * i11 * i22;
        rec[3] = -(L20 * i00 + L21 * rec[1]) * i22;
        rec[5] = i22;
    } else {
        bad = 1.0;
    }
    const double* G = rec;
    double* es = rec + 6;
    double* Ks = rec + 9;
    es[0] = s0 * e[0]; es[1] = s1 * e[1]; es[2] = s2 * e[2];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        Ks[m * 3 + 0] = sk[m] * Kt[m * 3 + 0] * s0;
        Ks[m * 3 + 1] = sk[m] * Kt[m * 3 + 1] * s1;
        Ks[m * 3 + 2] = sk[m] * Kt[m * 3 + 2] * s2;
    }
    if (want_kk) {  // intrinsics Schur terms once per point: -Zk Zk^T (10 packed), -Zk ze (4)
        double Zk[12], ze[3];
        zk_ze(G, Ks, es, Zk, ze);
        int qq = 0;
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int l = m; l < 4; ++l, ++qq)
                kk[qq] = -(Zk[m * 3 + 0] * Zk[l * 3 + 0] + Zk[m * 3 + 1] * Zk[l * 3 + 1] + Zk[m * 3 + 2] * Zk[l * 3 + 2]);
#pragma unroll
        for (int m = 0; m < 4; ++m) kk[10 + m] = -(Zk[m * 3 + 0] * ze[0] + Zk[m * 3 + 1] * ze[1] + Zk[m * 3 + 2] * ze[2]);
    }
}

// Diagnostic stamps (separate build via STAMP=true, MIBA_CHOL_STAMPS=1): cycles per phase
// accumulated by thread 0: [0] prefetch issue, [1] trsm, [2] update || look-ahead potrf, [3] retire/install,
// [4] tail+backward.
// uniform broadcast of lane `l`'s double (v_readlane, no LDS round trip)
__device__ __forceinline__ double bcast(double v, int l) {
    const unsigned long long u = __double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
    return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// In-register 16x16 Cholesky by one wave: lane r (r < 16; replicated above) holds row r.
// Entries above the diagonal are scratch (never consumed; masked at write-back), so the
// rank-1 updates run unpredicated. rdiag[j] = 1 / L_jj.
__device__ __forceinline__ void potrf16_regs(double (&a)[16], double* rdiag, int lane, bool& bad) {
    const int r = lane & 15;
    double my_inv = 0.0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        double djj = bcast(a[j], j);
        const bool ok = (djj > 0.0) && (djj < INFINITY);
        bad = bad || !ok;
        djj = ok ? djj : 1.0;
        const double inv = rsqrt_nr(djj);
        const double lrj = a[j] * inv;  // lane j: sqrt(d_jj); lanes r > j: L_rj
        a[j] = lrj;
        my_inv = (r == j) ? inv : my_inv;
#pragma unroll
        for (int k = j + 1; k < 16; ++k) a[k] -= lrj * bcast(lrj, k);
    }
    if (lane < 16) rdiag[r] = my_inv;
}

// One thread: Ceres 2.0 TrustRegionMinimizer::Minimize bookkeeping for the step whose
// scalars k_final produced (model cost change, candidate cost, |step|, |x_cand|, flags).
// Same decisions, in the same order, as oracle_solve() (oracle/ba_oracle.c).
__device__ __forceinline__ void lm_decide_local(LmState& S, const LmParams& prm, double lin0, double lin1,
                                                const double* __restrict__ scal, double* __restrict__ log) {
    if (S.need_lin) {  // absorb the re-linearisation of the last accepted point
        S.need_lin = 0;
        S.x_cost = lin0;
        S.gmax_ci = lin1;
        log[S.iter * LOG_W + 0] = S.x_cost;
        if (!isfinite(S.x_cost)) {
            S.done = 1; S.termination = 2; S.msg = MSG_EVAL_FAIL;
            return;
        }
        S.final_cost = fmin(S.final_cost, S.x_cost);
    }
    const double gmax = fmax(S.gmax_ci, scal[SC_GMAX_PT]);
    log[S.iter * LOG_W + 2] = gmax;
    // FinalizeIterationAndCheckIfMinimizerCanContinue. The message operands are chosen by selects and stored
    // once: per-branch stores of msg_a / msg_b were merged into one store at a selected field offset, which
    // kept the state in scratch (24 B per lane in k_final / k_combine / k_lm_decide).
    {
        const bool t_iter = S.iter >= prm.max_iter;
        const bool t_grad = !t_iter && S.step_ok && gmax <= prm.gradient_tolerance;
        const bool t_rad = !t_iter && !t_grad && S.radius <= prm.min_radius;
        if (t_iter || t_grad || t_rad) {
            S.done = 1;
            S.termination = t_iter ? 1 : 0;
            S.msg = t_iter ? MSG_MAX_ITER : (t_grad ? MSG_GRAD_TOL : MSG_MIN_RADIUS);
            S.msg_a = t_iter ? (double)S.iter : (t_grad ? gmax : S.radius);
            S.msg_b = t_iter ? S.msg_b : (t_grad ? prm.gradient_tolerance : prm.min_radius);
            return;
        }
    }
    if (scal[SC_BAD] >= SC_BAD_TIMEOUT) {
        // a BCR hand-off timed out (the resident workgroups were not co-resident): this iteration computed no
        // step. Stop the device loop WITHOUT a termination (termination -1, the iteration not counted, x /
        // radius untouched): the host re-runs it with the per-level BCR launches and resumes the solve.
        S.done = 1; S.termination = -1; S.msg = MSG_TIMEOUT;
        return;
    }
    S.iter += 1;
    double* lg = log + S.iter * LOG_W;
    const double mcc = scal[SC_MCC];
    const bool lsf = scal[SC_BAD] >= 2.0;  // linear solver failure (point block or Cholesky not PD)
    const bool valid = !lsf && isfinite(mcc) && mcc > 0.0;
    if (!valid) {  // HandleInvalidStep
        S.n_unsucc += 1;
        if (++S.n_invalid >= prm.max_invalid) {
            S.done = 1; S.termination = 2; S.msg = MSG_INVALID; S.msg_a = prm.max_invalid;
        } else {
            S.radius /= S.decrease_factor;
            S.decrease_factor *= 2.0;
            S.step_ok = 0;
        }
        lg[0] = S.x_cost; lg[1] = 0.0; lg[3] = 0.0; lg[4] = 0.0; lg[5] = S.radius; lg[6] = 0.0;
        return;
    }
    S.n_invalid = 0;
    double cand = scal[SC_CAND];
    if (scal[SC_BAD] >= 1.0 || !isfinite(cand)) cand = DBL_MAX;
    const double step_norm = sqrt(scal[SC_SN2]);
    const double xnorm = sqrt(S.xnorm2);
    const double cost_change = S.x_cost - cand;
    const bool t_par = step_norm <= prm.parameter_tolerance * (xnorm + prm.parameter_tolerance);
    const bool t_fun = !t_par && fabs(cost_change) <= prm.function_tolerance * S.x_cost;
    if (t_par || t_fun) {
        S.done = 1; S.termination = 0; S.msg = t_par ? MSG_PARAM_TOL : MSG_FUNC_TOL;
        S.msg_a = t_par ? step_norm / (xnorm + prm.parameter_tolerance) : fabs(cost_change) / S.x_cost;
        S.msg_b = t_par ? prm.parameter_tolerance : prm.function_tolerance;
        lg[0] = cand; lg[1] = cost_change; lg[3] = step_norm; lg[4] = 0.0; lg[5] = S.radius; lg[6] = -1.0;
        return;
    }
    const double rho = (cand >= DBL_MAX) ? -DBL_MAX : cost_change / mcc;
    if (rho > prm.min_relative_decrease) {  // HandleSuccessfulStep + LM StepAccepted
        S.cur ^= 1;
        S.need_lin = 1;
        S.xnorm2 = scal[SC_XN2];
        const double t = 2.0 * rho - 1.0;
        S.radius = S.radius / fmax(1.0 / 3.0, 1.0 - t * t * t);
        S.radius = fmin(prm.max_radius, S.radius);
        S.decrease_factor = 2.0;
        S.step_ok = 1;
        S.n_succ += 1;
        lg[0] = cand; lg[6] = 1.0;  // cost re-evaluated at absorb time
    } else {  // HandleUnsuccessfulStep + LM StepRejected
        S.radius /= S.decrease_factor;
        S.decrease_factor *= 2.0;
        S.step_ok = 0;
        S.n_unsucc += 1;
        S.final_cost = fmin(S.final_cost, cand);
        lg[0] = cand; lg[6] = 0.0;
    }
    lg[1] = cost_change; lg[3] = step_norm; lg[4] = rho; lg[5] = S.radius;
}

// Publishes the LM progress to the host-mapped block (one thread): the terminal state first (8-byte
// system-scope stores, drained), then the word n_decide | done << 31.
// The state's 8-byte words field by field (no reinterpret_cast of the struct: that view kept the state in scratch,
// 24 B per lane in k_final / k_combine); the host copies the block back as an LmState.
static_assert(offsetof(LmState, msg_b) == 64 && offsetof(LmState, iter) == 72 && offsetof(LmState, n_decide) == 116 &&
                  sizeof(LmState) == 120,
              "publish_progress writes LmState's layout word by word");
__device__ __forceinline__ unsigned long long pack2(int lo, int hi) {
    return (unsigned long long)(unsigned)lo | ((unsigned long long)(unsigned)hi << 32);
}
__device__ inline void publish_progress(unsigned* progress, const LmState& S) {
    if (S.done) {
        const unsigned long long w[15] = {
            (unsigned long long)__double_as_longlong(S.radius), (unsigned long long)__double_as_longlong(S.decrease_factor),
            (unsigned long long)__double_as_longlong(S.x_cost), (unsigned long long)__double_as_longlong(S.xnorm2),
            (unsigned long long)__double_as_longlong(S.final_cost), (unsigned long long)__double_as_longlong(S.gmax_ci),
            (unsigned long long)__double_as_longlong(S.initial_cost), (unsigned long long)__double_as_longlong(S.msg_a),
            (unsigned long long)__double_as_longlong(S.msg_b), pack2(S.iter, S.n_succ), pack2(S.n_unsucc, S.n_invalid),
            pack2(S.step_ok, S.cur), pack2(S.need_lin, S.done), pack2(S.termination, S.msg),
            pack2(S.stop_next, S.n_decide)};
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(reinterpret_cast<char*>(progress) + PROG_STATE_OFF);
#pragma unroll
        for (int k = 0; k < 15; ++k) __hip_atomic_store(dst + k, w[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_store(progress, (unsigned)S.n_decide | (S.done ? 0x80000000u : 0u), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// The decision on a state the caller has already loaded (S0) and the step scalars in registers: one store
// of the new state, no global round trip between the reductions and the decision (k_final).
__device__ inline void lm_decide_pre(const LmState& S0, LmState* __restrict__ st, const LmParams& prm, double lin0,
                                     double lin1, const double* scal, double* __restrict__ log) {
    if (S0.done) return;
    LmState S = S0;
    lm_decide_local(S, prm, lin0, lin1, scal, log);
    S.n_decide += 1;
    S.stop_next = !S.done && S.iter >= prm.max_iter;
    *st = S;
    if (prm.progress) publish_progress(prm.progress, S);
}
__device__ inline void lm_decide_body(LmState* __restrict__ st, const LmParams& prm, const double* __restrict__ lin,
                                      const double* __restrict__ scal, double* __restrict__ log) {
    const LmState S0 = *st;
    lm_decide_pre(S0, st, prm, lin[0], lin[1], scal, log);
}

}  // namespace miba
