// ba_tail.h — the observation-record helpers and the bodies of the LM iteration's tail (libmiba, internal, HIP):
// the point back-substitution of one chunk and the final reduction + LM decision. ba_kernels.hip launches them as
// k_backsub_chunk / k_final; ba_band.hip runs them as roles of one launch behind the band solve (k_band_tail).
#pragma once
#include <hip/hip_runtime.h>

#include "ba_common.h"
#include "ba_device.h"
#include "ba_kernels.h"
#include "ba_solve_util.h"

namespace miba {

static constexpr int TPB = 256;

// Observation record as loaded (ObsRaw<O32>): O32 = the window's obs32 records (one 16-byte load), else the f64
// arrays; u / v / depth widen to f64 exactly, so both paths run the same arithmetic.
template <bool O32>
struct ObsRaw;
template <>
struct ObsRaw<true> {
    float4 r;
    __device__ __forceinline__ double u() const { return (double)r.x; }
    __device__ __forceinline__ double v() const { return (double)r.y; }
    __device__ __forceinline__ double d() const { return (double)r.z; }
    __device__ __forceinline__ int idx() const { return __float_as_int(r.w); }
};
template <>
struct ObsRaw<false> {
    double2 uv;
    double dep;
    int i;
    __device__ __forceinline__ double u() const { return uv.x; }
    __device__ __forceinline__ double v() const { return uv.y; }
    __device__ __forceinline__ double d() const { return dep; }
    __device__ __forceinline__ int idx() const { return i; }
};
// point-major observation o: pixel, depth, camera index
template <bool O32>
__device__ __forceinline__ ObsRaw<O32> po_obs(const DevProblem& P, int o) {
    if constexpr (O32) return ObsRaw<true>{P.po_rec[o]};
    else return ObsRaw<false>{P.po_uv[o], P.po_depth[o], P.po_cam[o]};
}
// camera-major observation o: pixel, depth, point index
template <bool O32>
__device__ __forceinline__ ObsRaw<O32> co_obs(const DevProblem& P, int o) {
    if constexpr (O32) return ObsRaw<true>{P.co_rec[o]};
    else return ObsRaw<false>{P.co_uv[o], P.co_depth[o], P.co_pt[o]};
}
template <bool O32>
__device__ __forceinline__ ObsRaw<O32> obs_zero() {
    if constexpr (O32) return ObsRaw<true>{float4{0.f, 0.f, 0.f, 0.f}};
    else return ObsRaw<false>{double2{0.0, 0.0}, 0.0, 0};
}


// Block (256 threads) sum of NV values; result valid in out[0..NV) after return (LDS).
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* lds /*4*NV*/, double* out /*NV*/) {
    wave_sum<NV>(v);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) lds[wave * NV + i] = v[i];
    __syncthreads();
    for (int i = threadIdx.x; i < NV; i += blockDim.x)
        out[i] = lds[0 * NV + i] + lds[1 * NV + i] + lds[2 * NV + i] + lds[3 * NV + i];
    __syncthreads();
}


// block_sum with the DPP wave sum (the band tail's chunks: default mode only, one instantiation per layout is never
// compared bitwise with the other)
template <int NV>
__device__ __forceinline__ void block_sum_dpp(double (&v)[NV], double* lds /*4*NV*/, double* out /*NV*/) {
    wave_sum_dpp<NV>(v);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) lds[wave * NV + i] = v[i];
    __syncthreads();
    for (int i = threadIdx.x; i < NV; i += blockDim.x)
        out[i] = lds[0 * NV + i] + lds[1 * NV + i] + lds[2 * NV + i] + lds[3 * NV + i];
    __syncthreads();
}


// Block (256 threads) sum of NV values via the wave reduce-scatter; out[0..NV) valid after return.
// lds must hold 4 * NV doubles. Fixed summation order (deterministic).
template <int NV>
__device__ __forceinline__ void block_sum_rs(double (&v)[NV], double* lds, double* out) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int base = 0, len = NV;
    WaveHalve<NV, 32>::run(v, lane, base, len);
    constexpr int R = HalveRemain<NV, 32>::value;
#pragma unroll
    for (int j = 0; j < R; ++j)
        if (j < len) lds[wave * NV + base + j] = v[j];
    __syncthreads();
    for (int i = threadIdx.x; i < NV; i += blockDim.x)
        out[i] = lds[0 * NV + i] + lds[1 * NV + i] + lds[2 * NV + i] + lds[3 * NV + i];
    __syncthreads();
}


__device__ __forceinline__ double block_max(double v, double* lds) {
    v = dpp_wave_max(v);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) lds[wave] = v;
    __syncthreads();
    const double r = fmax(fmax(lds[0], lds[1]), fmax(lds[2], lds[3]));
    __syncthreads();
    return r;
}

// Back-substitution over a chunk of <= BS_PTS points / <= BS_OBS observations (one
// workgroup; observation loads coalesced, one observation per thread):
//   phase 1 (obs):   c_o = s_p (Jp^T (Jc (s_c y_c)))  -> LDS slot of the observation
//   phase 2 (point): y_p = V~^-1 (e~ - Kt^T y_k - sum_o c_o) (fixed order), delta_p = -s_p y_p
//   phase 3 (obs):   candidate cost at x + delta
// The points' share of the model cost change, 0.5 (e~^T y_p + y_p^T D~_p y_p), is summed in phase 2
// (k_update_cams states the identity).
// A chunk holding a single point with more than BS_OBS observations sums c_o by block reduction.
// PUB (the band tail launch, ba_band.hip): values another workgroup of the same launch produced are read past the
// L2 (agent-scope relaxed loads), and the partials this one publishes are stored past it and drained, so no L2
// write-back / invalidate fence is needed on either side
__device__ __forceinline__ double tail_ld(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load((unsigned long long*)const_cast<double*>(p),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void tail_st(double* p, double v) {
    __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

struct BsLds {
    double co[BS_OBS][3];
    double xnl[BS_PTS][3];  // the chunk's candidate points x + delta (phase 2 -> phase 3: no point load in phase 3)
    double lds[4 * 5];
    double out[5];
};
// the band tail (BsPre): the chunk's point records, point scales and current points, loaded before the wait (in the
// tail launch's dynamic LDS after BsLds; k_backsub_chunk's static BsLds stays as it was)
struct BsPreLds {
    double pt[BS_PTS][PDATA + 6];
};
// Band tail (PUB): the candidate poses of every camera and the candidate intrinsics, computed by each chunk from y
// (the band solve publishes y BEFORE its camera step, which then runs beside the chunks instead of ahead of them).
// Before the wait: every camera's current pose (8 doubles per camera) and the active cameras' Jacobi scales; after it,
// one thread per active camera overwrites its pose with T exp(-s y) (se3_plus, the step's own arithmetic: the same
// values cam_step stores in the candidate slot) and one thread the intrinsics K - s_k y_k (intr_step's).
// Layout after BsLds + BsPreLds in the tail launch's dynamic LDS: pose[n_cams][8] | K[4] | sc[nac][6].
__host__ __device__ inline size_t cand_lds_doubles(int n_cams, int nac) { return 8 * (size_t)n_cams + 4 + 6 * (size_t)nac; }
template <bool O32>
__device__ __forceinline__ void cand_prefetch(const DevProblem& P, const LmState* __restrict__ st,
                                              const double* __restrict__ scale, double* __restrict__ CL) {
    if (skip_step(st)) return;
    const int cur = st->cur;
    const double* x = P.cams[cur];
    for (int e = threadIdx.x; e < 7 * P.n_cams; e += TPB) CL[(e / 7) * 8 + e % 7] = x[e];
    double* const sc = CL + 8 * (size_t)P.n_cams + 4;
    for (int e = threadIdx.x; e < 6 * P.nac; e += TPB) sc[e] = scale[e];
}
// after the wait (y published): the candidate poses / intrinsics in place; the caller's next barrier publishes them
// (YL: y is the chunk's LDS copy, plain loads; else y in memory, read past the L2)
template <bool YL = false>
__device__ __forceinline__ void cand_compute(const DevProblem& P, int cur, const double* __restrict__ scale,
                                             const double* __restrict__ y, double* __restrict__ CL);
// Band tail (PUB): what a back-substitution chunk can compute before the band solve's y exists — its observation
// records, each thread's first observation's y-free product A = diag(s_p) Jp^T Jc diag(s_c) (3 x 6; v = A y_c
// after the wait) and the chunk's point data in LDS — so only the y / candidate loads and short products follow it
template <bool O32>
struct BsPre {
    bool on;            // the chunk is not a single big point and the window's state says step
    int ac0;            // active camera of this thread's first observation (< 0: none / gauge)
    double A[18];
    int r_ap[BS_OBS / TPB];
    ObsRaw<O32> r_o[BS_OBS / TPB];
    int pi;             // point index of this thread's point (tid < the chunk's points): phase 2's store address
};
template <bool O32>
__device__ __forceinline__ void backsub_pre(const DevProblem& P, const BaConsts& c, const LmState* __restrict__ st,
                                            const double* __restrict__ scale, const double* __restrict__ pdata, int ch,
                                            BsPreLds& L, BsPre<O32>& B) {
    B.on = false;
    B.ac0 = -1;
    if (skip_step(st)) return;
    const int cur = st->cur;
    const int tid = threadIdx.x;
    const int apb = P.bs_chunk[ch], ape = P.bs_chunk[ch + 1];
    const int ob = P.pt_ptr[apb], oe = P.pt_ptr[ape];
    if (oe - ob > BS_OBS) return;  // a single big point: the plain path after the wait
    B.on = true;
    B.pi = tid < ape - apb ? P.pt_idx[apb + tid] : 0;
    constexpr int NR = BS_OBS / TPB;
    int it = 0;
    for (int o = ob + tid; o < oe; o += TPB, ++it) {
        const int ap = P.po_ap[o];
        const ObsRaw<O32> ro = po_obs<O32>(P, o);
#pragma unroll
        for (int k = 0; k < NR; ++k)
            if (k == it) { B.r_ap[k] = ap; B.r_o[k] = ro; }
        if (it == 0) {
            const int ac = P.po_ac[o];
            B.ac0 = ac;
            if (ac >= 0) {
                ObsEval ev;
                double jc[18], jp[9], jk[8];
                lin_obs(c, P.cams[cur] + 7 * ro.idx(), P.pts[cur] + 3 * P.pt_idx[ap], P.K[cur], ro.u(), ro.v(), ro.d(),
                        ev, jc, jp, jk);
                const double* sc = scale + 6 * ac;
                const double* sp = scale + P.off_pt + 3 * ap;
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int d = 0; d < 6; ++d)
                        B.A[i * 6 + d] = sp[i] * ((jp[i] * jc[d] + jp[3 + i] * jc[6 + d]) + jp[6 + i] * jc[12 + d]) * sc[d];
            }
        }
    }
    for (int e = tid; e < (ape - apb) * (PDATA + 6); e += TPB) {  // point data, coalesced by element
        const int pl = e / (PDATA + 6), q = e - pl * (PDATA + 6), ap = apb + pl;
        double v;
        if (q < PDATA) v = pdata[(size_t)ap * PDATA + q];
        else if (q < PDATA + 3) v = scale[P.off_pt + 3 * (size_t)ap + q - PDATA];
        else v = P.pts[cur][3 * (size_t)P.pt_idx[ap] + q - PDATA - 3];
        L.pt[pl][q] = v;
    }
}
// PUB_OUT alone (k_backsub_final, C4-size windows): y and the candidates come from the previous launch (plain loads),
// only the partials are stored past the L2 and drained for the decision workgroup of the same launch. YL (the band
// tail): y is the chunk's own LDS copy of the polled y (plain loads)
template <bool O32, bool PUB = false, bool PUB_OUT = PUB, bool YL = false>
__device__ __forceinline__ void backsub_body(const DevProblem& P, const BaConsts& c, const LmState* __restrict__ st,
                                             const double* __restrict__ scale, const double* __restrict__ pdata,
                                             const double* __restrict__ y, const double* __restrict__ delta,
                                             double* __restrict__ part, const int2* __restrict__ ztiles, int n_ztiles,
                                             double* __restrict__ Sz, int ch, int nch, BsLds& L,
                                             const BsPre<O32>& pre = BsPre<O32>{}, BsPreLds* PL = nullptr,
                                             double* __restrict__ CL = nullptr,
                                             unsigned long long* __restrict__ bst = nullptr) {
    auto bmark = [&](int k) {  // (diagnostic stamps: band tail, MIBA_BCR_STAMPS=1)
        if (bst && threadIdx.x == 0) bst[k] = realtime_now();
    };
    const bool use_pre = PL != nullptr;
    const bool PRE = use_pre && pre.on;  // (block-uniform)
    auto& co = L.co;
    auto& xnl = L.xnl;
    double* const lds = L.lds;
    double* const out = L.out;
    if (skip_step(st)) return;
    // fused path: the reduced solve has consumed S; zero this chunk's share of its envelope tiles for the next
    // iteration's atomic assembly (k_final zeroes rhs, which still holds y here)
    for (int t = ch * n_ztiles / nch; !PUB && t < (ch + 1) * n_ztiles / nch; ++t) {  // (PUB: the caller, after)
        // (k_backsub_final: S was read by the previous launch, so the chunks zero it here as k_backsub_chunk does)
        const int2 ij = ztiles[t];
        Sz[(size_t)(16 * ij.x + (threadIdx.x >> 4)) * P.npad + 16 * ij.y + (threadIdx.x & 15)] = 0.0;
    }
    const int cur = st->cur;
    const int tid = threadIdx.x;
    const int apb = P.bs_chunk[ch], ape = P.bs_chunk[ch + 1];
    const int ob = P.pt_ptr[apb], oe = P.pt_ptr[ape];
    const int npts = ape - apb;
    const bool big = oe - ob > BS_OBS;  // single point
    const double* K = P.K[cur];
    const double* Kn = P.K[cur ^ 1];
    double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};  // sn2, mcc, cost, bad, |x_cand|^2
    // each thread's observation records (<= BS_OBS / TPB of them) are read once, in phase 1, and kept in
    // registers for phase 3 (a single point with more observations re-reads its records in phase 3)
    constexpr int NR = BS_OBS / TPB;
    int r_ap[NR];
    ObsRaw<O32> r_o[NR];  // camera index, pixel, depth
    // this thread's point index for phase 2, loaded before phase 1 (phase 2 then gathers its point in one trip,
    // not pt_idx and then the point); the band tail's prologue loaded it already
    const int pi_ph2 = PRE ? pre.pi : (tid < npts ? P.pt_idx[apb + tid] : 0);
    // ---- phase 1
    double bsum[3] = {0.0, 0.0, 0.0};
    int it = 0;
    for (int o = ob + tid; o < oe; o += TPB, ++it) {
        if (PRE && it == 0) {  // the y-free product computed before the wait: v = A y_c
#pragma unroll
            for (int k = 0; k < NR; ++k) { r_ap[k] = pre.r_ap[k]; r_o[k] = pre.r_o[k]; }
            double v[3] = {0.0, 0.0, 0.0};
            const int ac = pre.ac0;
            if (ac >= 0) {
                double yv[6];
#pragma unroll
                for (int d = 0; d < 6; ++d) yv[d] = YL ? y[6 * ac + d] : tail_ld(y + 6 * ac + d);
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    double a = 0.0;
#pragma unroll
                    for (int d = 0; d < 6; ++d) a = __builtin_fma(pre.A[i * 6 + d], yv[d], a);
                    v[i] = a;
                }
            }
#pragma unroll
            for (int i = 0; i < 3; ++i) co[o - ob][i] = v[i];
            continue;
        }
        const int ac = P.po_ac[o];
        const int ap = P.po_ap[o];
        const ObsRaw<O32> ro = po_obs<O32>(P, o);
        const int cam = ro.idx();
#pragma unroll
        for (int k = 0; k < NR; ++k)  // register arrays: constant indices only
            if (k == it) { r_ap[k] = ap; r_o[k] = ro; }
        double v[3] = {0.0, 0.0, 0.0};
        if (ac >= 0) {
            ObsEval ev;
            double jc[18], jp[9], jk[8];
            // (the point through po_pt, loaded beside the record: one dependent load level less than pt_idx[ap])
            lin_obs(c, P.cams[cur] + 7 * cam, P.pts[cur] + 3 * P.po_pt[o], K, ro.u(), ro.v(), ro.d(), ev, jc, jp, jk);
            const double* sc = scale + 6 * ac;
            const double* yc = y + 6 * ac;
            const double* sp = scale + P.off_pt + 3 * ap;
            double jy[3], sy[6];
#pragma unroll
            for (int d = 0; d < 6; ++d) sy[d] = sc[d] * ((PUB && !YL) ? tail_ld(yc + d) : yc[d]);
            jc_times(jc, sy, jy);
#pragma unroll
            for (int i = 0; i < 3; ++i) v[i] = sp[i] * (jp[i] * jy[0] + jp[3 + i] * jy[1] + jp[6 + i] * jy[2]);
        }
        if (big) {
#pragma unroll
            for (int i = 0; i < 3; ++i) bsum[i] += v[i];
        } else {
#pragma unroll
            for (int i = 0; i < 3; ++i) co[o - ob][i] = v[i];
        }
    }
    // the band tail: this chunk's candidate poses / intrinsics from y (published by the barrier below / in block_sum)
    if (CL) cand_compute<YL>(P, cur, scale, y, CL);
    if (big) block_sum<3>(bsum, lds, out);  // out[0..3) valid for every thread after this
    __syncthreads();
    bmark(0);
    // ---- phase 2
    if (tid < npts) {
        const int ap = apb + tid;
        const int pi = pi_ph2;
        const double* X = PRE ? &PL->pt[tid][PDATA + 3] : P.pts[cur] + 3 * pi;
        double* Xn = P.pts[cur ^ 1] + 3 * pi;
        const double* pd = PRE ? &PL->pt[tid][0] : pdata + (size_t)ap * PDATA;
        const double* sp = PRE ? &PL->pt[tid][PDATA] : scale + P.off_pt + 3 * ap;
        double yk[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) yk[m] = (PUB && !YL) ? tail_ld(y + P.kb + m) : y[P.kb + m];
        double t[3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
            t[i] = pd[6 + i] - (pd[9 + 0 * 3 + i] * yk[0] + pd[9 + 1 * 3 + i] * yk[1] + pd[9 + 2 * 3 + i] * yk[2] +
                                pd[9 + 3 * 3 + i] * yk[3]);
        if (big) {
#pragma unroll
            for (int i = 0; i < 3; ++i) t[i] -= out[i];
        } else {
            for (int o = P.pt_ptr[ap]; o < P.pt_ptr[ap + 1]; ++o)
#pragma unroll
                for (int i = 0; i < 3; ++i) t[i] -= co[o - ob][i];
        }
        double Vf[9];
        vinv_from_g(pd, Vf);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double yp = Vf[i * 3 + 0] * t[0] + Vf[i * 3 + 1] * t[1] + Vf[i * 3 + 2] * t[2];
            acc[1] += 0.5 * (pd[6 + i] * yp + pd[21 + i] * yp * yp);
            const double dp = -sp[i] * yp;
            const double xn = X[i] + dp;
            Xn[i] = xn;
            xnl[tid][i] = xn;
            const double df = X[i] - xn;
            acc[0] += df * df;
            acc[4] += xn * xn;
        }
    }
    __syncthreads();
    bmark(1);
    // ---- phase 3
    (void)delta;
    it = 0;
    for (int o = ob + tid; o < oe; o += TPB, ++it) {
        int ap;
        ObsRaw<O32> ro;
        if (it < NR) {
#pragma unroll
            for (int k = 0; k < NR; ++k)  // register arrays: constant indices only
                if (k == it) { ap = r_ap[k]; ro = r_o[k]; }
        } else {
            ap = P.po_ap[o];
            ro = po_obs<O32>(P, o);
        }
        const int cam = ro.idx();
        const int pl = ap - apb;
        const double xn[3] = {xnl[pl][0], xnl[pl][1], xnl[pl][2]};  // X + delta_p, as phase 2 stored it
        ObsEval en;
        if (CL) {  // the band tail: the chunk's own candidate table (cand_compute)
            eval_obs(c, CL + 8 * cam, xn, CL + 8 * (size_t)P.n_cams, ro.u(), ro.v(), ro.d(), en);
        } else if constexpr (PUB) {
            double pose[7], kn[4];
#pragma unroll
            for (int k = 0; k < 7; ++k) pose[k] = tail_ld(P.cams[cur ^ 1] + 7 * cam + k);
#pragma unroll
            for (int k = 0; k < 4; ++k) kn[k] = tail_ld(Kn + k);
            eval_obs(c, pose, xn, kn, ro.u(), ro.v(), ro.d(), en);
        } else {
            eval_obs(c, P.cams[cur ^ 1] + 7 * cam, xn, Kn, ro.u(), ro.v(), ro.d(), en);
        }
        if (en.ok) acc[2] += en.cost; else acc[3] = 1.0;
    }
    if (!isfinite(acc[0]) || !isfinite(acc[1])) acc[3] = 1.0;
    bmark(2);
    if constexpr (PUB) block_sum_dpp<5>(acc, lds, out);
    else block_sum<5>(acc, lds, out);
    bmark(3);
    if (tid == 0) {
        const double pv[5] = {out[0], out[1], out[2], out[3] > 0.0 ? 1.0 : 0.0, out[4]};
        // (the band tail, PUB: the decision workgroup polls these slots for its values — no count on its path)
        const int slot[5] = {PUB ? PART_TAIL : PART_BS_SN2, PUB ? PART_TAIL + 1 : PART_BS_MCC,
                             PUB ? PART_TAIL + 2 : PART_BS_COST, PUB ? PART_TAIL + 3 : PART_BS_BAD,
                             PUB ? PART_TAIL + 4 : PART_BS_XN2};
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            double* q = part + slot[k] * P.part_stride + ch;
            if constexpr (PUB_OUT) tail_st(q, pv[k]); else *q = pv[k];
        }
        if constexpr (PUB_OUT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drained before the count
        bmark(4);
    }
}

template <bool YL>
__device__ __forceinline__ void cand_compute(const DevProblem& P, int cur, const double* __restrict__ scale,
                                             const double* __restrict__ y, double* __restrict__ CL) {
    const double* const sc = CL + 8 * (size_t)P.n_cams + 4;
    for (int t = threadIdx.x; t < P.nac; t += TPB) {
        double* const xc = CL + 8 * (size_t)P.ac_cam[t];
        double x[7], d[6], tp[7];
#pragma unroll
        for (int j = 0; j < 7; ++j) x[j] = xc[j];
#pragma unroll
        for (int k = 0; k < 6; ++k) d[k] = -(YL ? y[6 * t + k] : tail_ld(y + 6 * t + k)) * sc[6 * t + k];  // cam_step's delta
        se3_plus(x, d, tp);
#pragma unroll
        for (int j = 0; j < 7; ++j) xc[j] = tp[j];
    }
    if (threadIdx.x == TPB - 1) {  // intr_step's candidate: K + (-y_k s_k)
        double* const kc = CL + 8 * (size_t)P.n_cams;
#pragma unroll
        for (int m = 0; m < 4; ++m) kc[m] = P.K[cur][m] + (-(YL ? y[P.kb + m] : tail_ld(y + P.kb + m)) * scale[P.off_k + m]);
    }
}

// scal[SC_MCC], [SC_CAND], [SC_SN2], [SC_GMAX_PT], [SC_BAD]; then the LM decision (k_lm_decide's
// body, fused: one launch less per iteration)
// 4 waves (16 measured 1 us slower at C4: more waves to start and to reduce than loads saved). UNR: unroll of
// the partial-sum loops (C4 rocprof: k_final 9.2 / 6.9 / 7.5 us at 1 / 2 / 8; k_final_shard with twice the
// accumulators 6.7 / 11.0 / 12.8 us at 1 / 4 / 8)
static constexpr int TPB_F = 256, NW_F = TPB_F / 64;
struct FinLds {
    double lds[NW_F * 4];
    double out[4];
    double red[NW_F];
};
// The band tail's decision (POLL): the back-substitution chunks' partials are not counted and then loaded — each
// thread polls its chunks' PART_TAIL slots until they hold values (flag-free: an empty slot holds BCR_Y_EMPTY, which no
// f64 arithmetic produces), so the reduction starts one store-to-load hop after the last chunk's store instead of a
// drain, a count, a poll of the count and a load round trip; then it empties the slots for the next launch. A poll
// past the spin bound raises FLAG_TIMEOUT (the iteration is re-run with the separate launches) and waits for the
// chunks' count (every chunk done) before anything is emptied or zeroed.
struct TailPoll {
    unsigned lim;            // polls before the timeout
    const unsigned* count;   // the chunks' count word
    unsigned target;         // its value once every chunk of this launch has counted
};
template <int UNR, bool PUB = false, bool POLL = false>
__device__ __forceinline__ void final_body(const DevProblem& P, LmState* __restrict__ st, int nblk_pt, int nblk_upd,
                                           int nblk_bs, const double* __restrict__ part,
                                           const int* __restrict__ chol_flag, double* __restrict__ scal,
                                           const LmParams& prm, const double* __restrict__ lin, double* __restrict__ log,
                                           double* __restrict__ rhs_z, unsigned* __restrict__ bcr_epoch, FinLds& L,
                                           unsigned long long* __restrict__ fst = nullptr, TailPoll tp = TailPoll{}) {
    double* const lds = L.lds;
    double* const out = L.out;
    double* const red = L.red;
    auto LD = [](const double* q) { return PUB ? tail_ld(q) : *q; };
    // every load up front (the state, the flag, lin and all partials), so the reductions and the decision
    // wait for one memory round trip instead of one per loop trip
    LmState S0;
    int cf = 0;
    double lin0 = 0.0, lin1 = 0.0;
    if (threadIdx.x == 0) {
        S0 = *st;
        if constexpr (!POLL)  // (POLL: after the chunks' partials, which follow any chunk's timeout flag)
            cf = PUB ? __hip_atomic_load(const_cast<int*>(chol_flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : *chol_flag;
        lin0 = lin[0];
        lin1 = lin[1];
    }
    const int done = __builtin_amdgcn_readfirstlane(st->done);
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    double gm = 0.0, bad = 0.0;
    const size_t stp = P.part_stride;
#pragma unroll UNR
    for (int i = threadIdx.x; i < nblk_upd; i += TPB_F) {
        acc[0] += LD(part + PART_UPD_SN2 * stp + i);
        acc[1] += LD(part + PART_UPD_MCC * stp + i);
        acc[2] += LD(part + PART_UPD_COST * stp + i);
        acc[3] += LD(part + PART_UPD_XN2 * stp + i);
    }
    if constexpr (POLL) {
        // (skip_step: the chunks stored nothing; the partials are not read)
        const bool skip = done || __builtin_amdgcn_readfirstlane(st->stop_next);
        bool ok = true;
        for (int i = threadIdx.x; i < nblk_bs && !skip; i += TPB_F) {
            unsigned long long u[5];
            const unsigned long long* q[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) q[k] = reinterpret_cast<const unsigned long long*>(part + (PART_TAIL + k) * stp + i);
            for (unsigned n = 0;; ++n) {
                bool pend = false;
#pragma unroll
                for (int k = 0; k < 5; ++k) {
                    u[k] = __hip_atomic_load(const_cast<unsigned long long*>(q[k]), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
                    pend = pend || u[k] == BCR_Y_EMPTY;
                }
                if (!pend) break;
                if (n >= tp.lim) { ok = false; break; }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!ok) break;
            acc[0] += __longlong_as_double((long long)u[0]);
            acc[1] += __longlong_as_double((long long)u[1]);
            acc[2] += __longlong_as_double((long long)u[2]);
            acc[3] += __longlong_as_double((long long)u[4]);
            bad = fmax(bad, __longlong_as_double((long long)u[3]));
        }
        __shared__ int fin_ok;
        if (threadIdx.x == 0) fin_ok = 1;
        __syncthreads();
        if (!ok) fin_ok = 0;
        __syncthreads();
        if (!fin_ok && threadIdx.x == 0) {
            raise_flag(const_cast<int*>(chol_flag), FLAG_TIMEOUT);
            for (unsigned n = 0; n < (1u << 26); ++n) {  // every chunk done before the slots are emptied, rhs zeroed
                if (__hip_atomic_load(const_cast<unsigned*>(tp.count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
                    tp.target)
                    break;
                __builtin_amdgcn_s_sleep(2);
            }
        }
        if (!fin_ok) __syncthreads();
        if (!skip)  // the slots empty again for the next launch (its chunks store after this launch has ended)
            for (int i = threadIdx.x; i < nblk_bs; i += TPB_F)
#pragma unroll
                for (int k = 0; k < 5; ++k) tail_st(const_cast<double*>(part) + (PART_TAIL + k) * stp + i,
                                                    __longlong_as_double((long long)BCR_Y_EMPTY));
        if (threadIdx.x == 0)
            cf = __hip_atomic_load(const_cast<int*>(chol_flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
#pragma unroll UNR
    for (int i = threadIdx.x; i < nblk_bs; i += TPB_F) {
        acc[0] += LD(part + PART_BS_SN2 * stp + i);
        acc[1] += LD(part + PART_BS_MCC * stp + i);
        acc[2] += LD(part + PART_BS_COST * stp + i);
        acc[3] += LD(part + PART_BS_XN2 * stp + i);
        bad = fmax(bad, LD(part + PART_BS_BAD * stp + i));
    }
    }
#pragma unroll UNR
    for (int i = threadIdx.x; i < nblk_pt; i += TPB_F) {
        gm = fmax(gm, part[PART_PT_GMAX * stp + i]);
        bad = fmax(bad, 2.0 * part[PART_PT_BAD * stp + i]);
    }
    if (done) return;
    // k_bcr_split ran this iteration (it skips exactly when done | stop_next): the next launch's epoch. Advanced
    // here, in stream order behind it, so no workgroup of that launch can still be reading the current one.
    if (bcr_epoch && threadIdx.x == 0 && !S0.stop_next) *bcr_epoch += 1;
    if (rhs_z)  // fused path: y has been consumed; rhs is the next assembly's atomic target
        for (int i = threadIdx.x; i < P.npad; i += TPB_F) rhs_z[i] = 0.0;
    if (fst && threadIdx.x == 0) fst[0] = realtime_now();  // (diagnostic stamps: band tail, MIBA_BCR_STAMPS=1)
    block_sum_nw<NW_F, 4>(acc, lds, out);
    gm = block_max_nw<NW_F>(gm, red);
    bad = block_max_nw<NW_F>(bad, red);
    if (fst && threadIdx.x == 0) fst[1] = realtime_now();
    if (threadIdx.x == 0) {
        double sc[SC_N] = {};
        sc[SC_XN2] = out[3];
        sc[SC_SN2] = out[0];
        sc[SC_MCC] = out[1];
        sc[SC_CAND] = out[2];
        sc[SC_GMAX_PT] = gm;
        sc[SC_BAD] = bad + ((cf & FLAG_NOT_PD) ? 4.0 : 0.0) + ((cf & FLAG_TIMEOUT) ? SC_BAD_TIMEOUT : 0.0);
#pragma unroll
        for (int k = 0; k < SC_N; ++k) scal[k] = sc[k];
        lm_decide_pre(S0, st, prm, lin0, lin1, sc, log);
        if (fst) fst[2] = realtime_now();
    }
}

}  // namespace miba
