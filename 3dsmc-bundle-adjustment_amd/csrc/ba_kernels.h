// ba_kernels.h — device data layout and kernel launchers of libmiba (internal).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdlib>
#include <mutex>

#include "ba_comm.h"
#include "ba_device.h"

namespace miba {

// per-active-camera linearisation record: U upper-packed (21) | C 6x4 (24) | g (6)
static constexpr int CAMDATA = 51;
// per camera-segment intrinsics partial: Ukk packed (10) | gk (4) | cost (1)
static constexpr int SEGINTR = 15;
// per active point Schur record: G = chol(V~)^-1 packed lower (6) | e~ (3) | K~ 4x3 (12) | LM diagonal D~ (3)
static constexpr int PDATA = 24;
// tiled Schur reduction geometry
static constexpr int TILE_WIN = 12;    // cameras per tile window
static constexpr int CHUNK_PTS = 32;   // points per Schur chunk (K = 3 * CHUNK_PTS of the MFMA product)
static constexpr int CHUNK_OBS = 256;
// deterministic mode: per-tile Schur slab, rows of M' (80) x the window's camera dofs (6 * TILE_WIN)
static constexpr int SCH_TBUF_LD = 6 * TILE_WIN;
static constexpr int SCH_TBUF = 80 * SCH_TBUF_LD;
static constexpr int SUBSEG_OBS = 1024;  // observations per camera-side sub-segment (one workgroup)
static constexpr int SUBSEG_OBS_SMALL = 256;  // ... on windows of < 4096 observations
static constexpr int SUBSEG_OBS_LARGE = 1700;  // the same on windows of >= 200k observations
static constexpr int BS_PTS = 128;    // points per back-substitution chunk (C4: 64 / 512 29.4 us, 128 / 1024 27.6, 256 / 2048 33.1)
static constexpr int BS_OBS = 1024;   // observations per back-substitution chunk (a single point may exceed)
// k_point_prep: PP_LANES lanes per active point (one aligned lane group), each taking every
// PP_LANES-th observation of the point; the group sums by xor-shuffles (fixed order)
static constexpr int PP_LANES_MAX = 4;
static constexpr int PP_TPB = 256;
int pp_lanes();  // lanes per point of k_point_prep (MIBA_PP_LANES: 1, 2 or 4)
inline int pp_blocks(int n_ap, int lanes) { return (n_ap * lanes + PP_TPB - 1) / PP_TPB; }
inline int pp_blocks(int n_ap) { return pp_blocks(n_ap, pp_lanes()); }

// partial-sum slots (each slot holds part_stride doubles, one per producing block)
enum {
    PART_PT_GMAX = 0,
    PART_PT_BAD,
    PART_UPD_SN2,
    PART_UPD_MCC,
    PART_UPD_COST,
    PART_BS_SN2,
    PART_BS_MCC,
    PART_BS_COST,
    PART_BS_BAD,
    PART_UPD_XN2,
    PART_BS_XN2,
    PART_INIT_XN2,
    PART_PT_KK,                     // 14 slots: intrinsics Schur terms of k_point_prep (10 packed + 4)
    // 5 slots: the band tail's back-substitution partials (sn2, mcc, cost, bad, |x_cand|^2), handed to its decision
    // workgroup flag-free — an empty slot holds BCR_Y_EMPTY (set at prepare, re-set by the decision after reading)
    PART_TAIL = PART_PT_KK + 14,
    PART_NSLOTS = PART_TAIL + 5
};
// final scalars
enum { SC_MCC = 0, SC_CAND, SC_SN2, SC_GMAX_PT, SC_BAD, SC_XN2, SC_N = 8 };
// lin record: [0] cost(x), [1] gmax cams+intr, [2..12) Ukk packed (+prior), [12..16) gk (+prior)
static constexpr int LIN_N = 16;

// Flattened window on the device (all indices 32-bit).
struct DevProblem {
    double* cams[2];  // [n_cams*7]  x and candidate (ping-pong)
    double* pts[2];   // [n_points*3]
    double* K[2];     // [4]
    const double* prior;
    // admissible observations grouped by active point (point-major)
    const int* po_cam;     // camera index
    const int* po_ac;      // active camera index or -1 (gauge / unobserved)
    const double2* po_uv;  // pixel
    const double* po_depth;
    const int* po_ap;      // active point index
    const int* po_pt;      // point index (= pt_idx[po_ap])
    const int* pt_ptr;     // [n_ap+1]
    const int* pt_idx;     // active point -> point index
    // admissible observations grouped by camera (camera-major)
    const int* co_pt;
    const double2* co_uv;
    const double* co_depth;
    // obs32 windows — every admissible pixel coordinate and depth exactly representable in f32, as the reference's
    // are (cv::KeyPoint::pt is float, the depth comes from a float image: OptimizationUtils.cpp:261-262,
    // Map3D.cpp:85-88): one 16-byte record per observation, {u, v, depth, camera index} point-major and
    // {u, v, depth, point index} camera-major (the index as the float's bits), read in one load instead of the
    // f64 arrays po_cam / po_uv / po_depth and co_pt / co_uv / co_depth (28 -> 16 bytes per observation and sweep)
    const float4* po_rec;
    const float4* co_rec;
    int obs32;
    const int* seg_ptr;  // [n_seg+1]
    const int* seg_cam;  // [n_seg]
    const int* seg_ac;   // [n_seg]
    const int2* ac_seg;  // [nac]: sub-segment range [x, y) of each active camera (camera-major order)
    const int* ac_cam;   // active camera -> camera index
    // tiled Schur reduction: tile t = chunks [tile_chunk[t], tile_chunk[t+1]),
    // chunk c = active points [chunk_ap[c], chunk_ap[c+1]); camera window [tile_base, +tile_span)
    const int* tile_chunk;
    const int* tile_base;
    const int* tile_span;
    const int* chunk_ap;
    const int* bs_chunk;   // back-substitution chunks: active-point boundaries (<= BS_PTS points, <= BS_OBS obs)
    int n_bs_chunks;
    const int* ovf_obs;  // point-major obs of overflow points (active camera only)
    int n_tiles, n_ovf_obs;
    int n_tiled_pts;  // active points [0, n_tiled_pts) belong to Schur tiles
    int n_seg, n_ap, n_adm, nac;
    int n_cams;  // cameras of the window (the band tail's candidate-pose table)
    int n;     // reduced system size 6*nac + 4
    int npad;  // n rounded up to 16
    int kb;    // first intrinsics row = 6*nac
    int off_pt, off_k;  // scale-vector offsets
    int part_stride;
    int band_w;  // 16x16 tiles below the diagonal in the camera band; <=0 or >6: dense envelope kernel
    int cam_band;  // max over active cameras of (camera - first co-visible camera)
    int solver;    // 0 dense envelope, 1 band, 2 block cyclic reduction
    int rank, nranks;  // landmark shard of this context (ba_comm_init); rank 0 adds the camera/intrinsics terms
    int xcd_map;       // camera-side workgroups take the sub-segments by XCD band (xcd_seg, ba_kernels.hip)
};

// Block cyclic reduction (ba_bcr.hip): nblk blocks of BCR_CAMS cameras (64 dofs).
static constexpr int BCR_CAMS = 10;
// Block cyclic reduction workspace, per 64-dof block i:
//   Cf   Cholesky factor of the block at its elimination                  64x64
//   X    [XL | XR | x] = Cf^-1 [A[i][i-s] | A[i][i+s] | R_i]              64x136
//   UL   XL^T XL  (Schur contribution to the left survivor, lower tiles) 64x64
//   UR   XR^T XR  (to the right survivor, lower tiles)                    64x64
//   F    -XR^T XL (fill coupling right survivor -> left one)              64x64
//   rL   XL^T x, rR = XR^T x                                              64x8 each
//   Dacc, Racc  survivor's diagonal block / rhs with the contributions of
//               all levels <= its elimination level - 2 folded in         64x64, 64x8
//   Y    solution rows [u | V]                                            64x8
//   Bp   border partial B_i^T Y_i (4x5)                                   32
//   rd   1 / diag(Cf)                                                     64
// plus one global slot: bk = [b_k (4) | S_kk lower (10)].
struct BcrWork {
    double *Cf, *X, *UL, *UR, *F, *rL, *rR, *Dacc, *Racc, *Y, *Bp, *rd, *bk;
    double* F2;  // k_bcr_split: the published XR rows of odd epochs (flag-free pull hand-off)
    // persistent path: flags[0] = call epoch, flags[16 + i] = block i eliminated (helper A's part
    // when split 3-way), flags[16 + nblk + i] = block i back-substituted, [16 + 2 nblk + i] panels
    // published, [16 + 3 nblk + i] helper B's part, [16 + 4 nblk + i] fill F, [16 + 5 nblk + i] XL
    // (each holds the epoch that set it; panels 4 * epoch + panel)
    unsigned* flags;  // flags[0] (the epoch) is advanced by k_final after every BCR launch that ran
    int nblk, levels;
    int voff, vroot, vlevels;  // k_bcr_split: balanced tree on v = i + voff, root block vroot, depth vlevels + 1
    int persist;  // 3 = factor + two helper workgroups per block (k_bcr_split<.., 2>), 2 = factor + one
                  // helper (k_bcr_split<.., 1>), 1 = one resident workgroup per block (k_bcr_persist),
                  // 0 = one launch per level
    int dense1;   // one-block window solved by k_bcr_dense1 (bcr_dense1_ok)
    int band;     // narrow-band window solved in one workgroup by k_bcr_band (ba_band.hip): cameras per block
                  // (1..3 = max(camera band, 1)), 0 = off (bcr_band_ok)
    int xmap;     // k_bcr_split on XCDs 0-3 only (one I/O die: 385 vs 510-580 ns per cross-workgroup hop,
                  // tools/handoff_probe.hip): launch workgroup b runs on XCD b mod 8, those on XCDs 4-7 exit
};
// k_bcr_split's flag-free back-substitution hand-off: y rows double-buffered by epoch parity (Y even,
// Racc odd — Racc belongs to the per-level path only); an empty slot holds this signalling-NaN pattern,
// which no f64 operation produces (they return quiet NaNs). INVARIANT: every value published through a
// flag-free slot (y rows, panels, fills) is the result of f64 arithmetic in the producing kernel, never
// raw input bits copied through (an input holding this exact pattern would read as "not yet stored");
// a future publication of copied values must canonicalise them first (v + 0.0 quiets a signalling NaN).
static constexpr unsigned BCR_Y_EMPTY_D32 = 0xFFF7A5A5u;
static constexpr unsigned long long BCR_Y_EMPTY = 0xFFF7A5A5FFF7A5A5ull;
// [XL | XR | x] row stride (136 columns; padding to 144 for conflict-free operand rows measured no gain)
static constexpr int BCR_XW = 136;
static constexpr size_t BCR_BLOCK_DOUBLES = (size_t)5 * 64 * 64 + 64 * BCR_XW + 4 * 64 * 8 + 32 + 64;

// Device-resident Levenberg-Marquardt state (Ceres 2.0 TrustRegionMinimizer +
// LevenbergMarquardtStrategy bookkeeping, owned by k_lm_decide).
struct LmState {
    double radius, decrease_factor, x_cost, xnorm2, final_cost, gmax_ci, initial_cost;
    double msg_a, msg_b;
    int iter, n_succ, n_unsucc, n_invalid, step_ok, cur, need_lin, done, termination, msg;
    // the next decision terminates at max_num_iterations before it looks at a step (Ceres checks the
    // iteration count before ComputeTrustRegionStep): that iteration only re-linearises, so the step
    // kernels (assembly, Schur, reduced solve, back-substitution) exit at once, like after `done`
    int stop_next;
    int n_decide;  // decisions taken (host progress word)
};
__device__ __forceinline__ bool skip_step(const LmState* st) { return st->done | st->stop_next; }
// Camera / intrinsics step application (k_update_cams, or fused into k_bcr_border): delta = -s*y,
// Sophus T*exp(delta) into the candidate slot, and the block's terms of the step scalars
// acc = {|step|^2, model cost change 0.5 (g~ y + D~ y^2), candidate prior cost, |x_cand|^2}.
// The operands of one camera's step (update_camera; k_bcr_dense1 loads them ahead of its factorization).
struct CamStepOps {
    int cam;
    double x[7], sc[6], ud[6], g[6];  // pose, Jacobi scale, diag of U, gradient g = Jc^T f
};
__device__ __forceinline__ void load_cam_step_ops(const DevProblem& P, int cur, const double* __restrict__ scale,
                                                  const double* __restrict__ camdata, int t, CamStepOps& o) {
    o.cam = P.ac_cam[t];
    const double* cd = camdata + (size_t)t * CAMDATA;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        o.sc[k] = scale[6 * t + k];
        o.ud[k] = cd[k * 6 - (k * (k - 1)) / 2];
        o.g[k] = cd[45 + k];
    }
    const double* x = P.cams[cur] + 7 * o.cam;
#pragma unroll
    for (int j = 0; j < 7; ++j) o.x[j] = x[j];
}
// PUB: a store past the L2 (agent-scope relaxed 8-byte atomic store), for a consumer of the same launch on another
// XCD that reads with agent-scope loads once the producer has drained its stores (the band tail launch)
template <bool PUB>
__device__ __forceinline__ void st_opt(double* p, double v) {
    if constexpr (PUB)
        __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    else
        *p = v;
}
template <bool PUB = false>
__device__ __forceinline__ void cam_step(const DevProblem& P, const BaConsts& c, int cur, double radius,
                                         const CamStepOps& o, int t, const double* yv, double* __restrict__ delta,
                                         double acc[4]) {
    double d[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const double sc = o.sc[k], yk = yv[k];
        d[k] = -yk * sc;
        st_opt<PUB>(delta + 6 * t + k, d[k]);
        const double u = sc * o.ud[k] * sc;  // diag of s U s (k_env_assemble)
        const double dd = fmin(fmax(u, c.min_diag), c.max_diag) / radius;
        acc[1] += 0.5 * ((sc * o.g[k]) * yk + dd * yk * yk);
    }
    double* xn = P.cams[cur ^ 1] + 7 * o.cam;
    double tp[7];
    se3_plus(o.x, d, tp);
#pragma unroll
    for (int j = 0; j < 7; ++j) {
        st_opt<PUB>(xn + j, tp[j]);
        const double df = o.x[j] - tp[j];
        acc[0] += df * df;
        acc[3] += tp[j] * tp[j];
    }
}
__device__ __forceinline__ void update_camera(const DevProblem& P, const BaConsts& c, int cur, double radius,
                                              const double* __restrict__ scale, const double* __restrict__ camdata,
                                              int t, const double* yv, double* __restrict__ delta, double acc[4]) {
    CamStepOps o;
    load_cam_step_ops(P, cur, scale, camdata, t, o);
    cam_step(P, c, cur, radius, o, t, yv, delta, acc);
}
// The intrinsics' step operands (update_intrinsics) and the step from them.
struct IntrStepOps {
    double K[4], sk[4], uk[4], gk[4], prior[4];  // K, Jacobi scale, diag of the prior-augmented Ukk, gk, prior
};
__device__ __forceinline__ void load_intr_step_ops(const DevProblem& P, int cur, const double* __restrict__ scale,
                                                   const double* __restrict__ lin, IntrStepOps& o) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        o.K[m] = P.K[cur][m];
        o.sk[m] = scale[P.off_k + m];
        o.uk[m] = lin[2 + 4 * m - (m * (m - 1)) / 2];
        o.gk[m] = lin[12 + m];
        o.prior[m] = P.prior[m];
    }
}
template <bool PUB = false>
__device__ __forceinline__ void intr_step(const DevProblem& P, const BaConsts& c, int cur, double radius,
                                          const IntrStepOps& o, const double* yk4, double* __restrict__ delta,
                                          double acc[4]) {
    double* Kn = P.K[cur ^ 1];
    for (int m = 0; m < 4; ++m) {
        const double sk = o.sk[m], ym = yk4[m];
        const double dk = -ym * sk;
        st_opt<PUB>(delta + P.kb + m, dk);
        const double kn = o.K[m] + dk;
        st_opt<PUB>(Kn + m, kn);
        const double df = o.K[m] - kn;
        acc[0] += df * df;
        const double u = sk * o.uk[m] * sk;  // Ukk incl. the prior block
        const double dd = fmin(fmax(u, c.min_diag), c.max_diag) / radius;
        acc[1] += 0.5 * ((sk * o.gk[m]) * ym + dd * ym * ym);
        const double fn = c.sw_k * (o.prior[m] - kn);
        acc[2] += 0.5 * fn * fn;
        acc[3] += kn * kn;
    }
}
__device__ __forceinline__ void update_intrinsics(const DevProblem& P, const BaConsts& c, int cur, double radius,
                                                  const double* __restrict__ scale, const double* __restrict__ lin,
                                                  const double* yk4, double* __restrict__ delta, double acc[4]) {
    IntrStepOps o;
    load_intr_step_ops(P, cur, scale, lin, o);
    intr_step(P, c, cur, radius, o, yk4, delta, acc);
}

struct LmParams {
    double min_relative_decrease, max_radius, min_radius, function_tolerance, gradient_tolerance,
        parameter_tolerance;
    int max_iter, max_invalid;
    unsigned* progress;  // host-mapped word: n_decide | done << 31 after every decision (nullptr: none)
};
// Host-mapped progress block (LmParams::progress): the word at byte 0 and, at byte PROG_STATE_OFF, a copy of
// the terminal LmState, stored (system scope, drained) before the word's done bit: the host reads the summary
// there instead of a device-to-host copy behind a stream synchronisation.
static constexpr int PROG_STATE_OFF = 64;
static constexpr int PROG_BYTES = PROG_STATE_OFF + (int)((sizeof(LmState) + 63) / 64 * 64);
static_assert(sizeof(LmState) % 8 == 0, "LmState is copied as 8-byte words");
enum LmMsg { MSG_NONE = 0, MSG_MAX_ITER, MSG_GRAD_TOL, MSG_MIN_RADIUS, MSG_PARAM_TOL, MSG_FUNC_TOL, MSG_INVALID,
             MSG_EVAL_FAIL, MSG_TIMEOUT };
// chol_flag bits: the reduced-system factorisation hit a non-positive pivot (a linear-solver failure,
// Ceres' invalid step), or an inter-workgroup hand-off of the resident BCR kernels timed out (the
// workgroups were not co-resident: the decision stops the device loop without a termination and the host
// re-runs that iteration with the per-level BCR launches, which have no inter-workgroup waits)
static constexpr int FLAG_NOT_PD = 1;
static constexpr int FLAG_TIMEOUT = 2;
// scal[SC_BAD] >= SC_BAD_TIMEOUT: some workgroup's hand-off timed out
static constexpr double SC_BAD_TIMEOUT = 8.0;
// offset of the sharded scalar exchange in DevWork::red
static constexpr int RED_X = 16;
// per-iteration log row: cost, cost_change, |gradient|_inf, |step|, tr_ratio, tr_radius, accepted
static constexpr int LOG_W = 8;

struct DevWork {
    double* camdata;
    double* seg_intr;
    double* lin;
    double* scale;
    double* cnp;
    double* pdata;
    double* S;
    double* rhs;  // rhs in, y out (after factor)
    double* delta;
    double* part;
    double* scal;
    int* chol_flag;
    int* fcol;
    int* rptr;
    int* rows;
    LmState* st;
    double* log;  // [(max_iter + 2) * LOG_W]
    BcrWork bcr;
    // landmark sharding (nranks > 1): this rank's camera-side partials, the packed envelope
    // of S (+ rhs) before / after the all-reduce, and the step-scalar exchange buffer
    Comm comm;
    double* camdata_loc;   // [nac * CAMDATA + 16]; == camdata when unsharded
    double* camdata_part;  // [n_seg * CAMDATA]: per sub-segment camera partials
    const int2* env_tile;  // (block row, block col) of every 16x16 envelope tile of S
    int n_env;
    double* env_loc;       // [n_env * 256 + npad (+ camera sums)]: the exchange, reduced in place
    double* red;           // [RED_X + 4 + 2 * nranks]: 6..9 replicated sums, 10 chol flag; at RED_X the exchange
                           // (4 local sums, then a (gmax, bad) slot pair per rank), reduced in place
    // deterministic mode (ba_options.deterministic): per-tile Schur slabs + each active camera's tile range;
    // nullptr: the tiles flush with f64 atomics
    double* det_tbuf = nullptr;
    const int2* det_trange = nullptr;
    // fused LM-loop linearisation (unsharded, default mode): k_lin_point (point side + camera side in one
    // launch), the envelope tiles as atomic adds inside k_schur_tile onto an S / rhs zeroed by the previous
    // iteration's k_backsub_chunk / k_final
    int fused = 0;
    // small windows (one resident round of the Schur launch, unsharded, default mode): the point side in the Schur
    // tiles themselves and the camera side + non-tiled points as extra workgroups of that launch, so the LM loop
    // has no k_lin_point (k_schur_tile<..., FP>). sw_cnt: camera-side workgroups finished (monotonic within a
    // solve; reset by launch_reset), sw_seq: Schur launches of this solve (host side)
    int sw = 0;
    // larger windows (unsharded, default mode): the tiled points' point side in the Schur tiles (k_schur_tile<..., FP>,
    // one Jacobian evaluation per observation for it and M'), k_lin_point runs the camera side + the non-tiled points
    int fpl = 0;
    unsigned* sw_cnt = nullptr;
    unsigned sw_seq = 0;
    // the band solve's tail (small unsharded windows, default mode): the back-substitution chunks and the final
    // reduction + decision as workgroups of the band solve's launch (k_band_tail), behind two hand-off words
    // tail_flags[0] (the solve's launch number: y published), [1] (back-substitution chunks done, monotonic within a
    // solve) and [2] (the solve's camera step published; all three reset by launch_reset); tail_seq: tail launches of
    // this solve (host side)
    int tail = 0;
    // larger unsharded fused windows: the back-substitution chunks and the final reduction + decision in one launch
    // (k_backsub_final), counted on tail_flags[1] / tail_seq like the band tail (never both)
    int bsfin = 0;
    unsigned* tail_flags = nullptr;
    unsigned tail_seq = 0;
    // the band tail's y, handed to its back-substitution chunks flag-free: buffer (tail_seq & 1) of two npad-double
    // buffers, an unwritten value holding BCR_Y_EMPTY; the solve workgroup empties the other buffer (read by the
    // previous launch) for the next launch, launch_reset empties both at a solve's start
    double* tail_y = nullptr;
};

// kernel ids for per-launch HIP-event profiling (ba_kernel_stats)
enum KernelId {
    K_CAM_SIDE = 0, K_LIN_FINALIZE, K_POINT_COLNORM, K_SCALE, K_MEMSET_S, K_ASSEMBLE, K_POINT_PREP, K_SCHUR_TILE,
    K_OBS_PAIRS, K_CHOL, K_UPDATE_CAMS, K_BACKSUB_EVAL, K_FINAL, K_DECIDE, K_XNORM, K_BCR_ELIM, K_BCR_CONTRIB,
    K_BCR_BACK, K_BCR_BORDER, K_COMM, K_CAM_REDUCE, K_BCR_PERSIST, K_PP_REDUCE, K_DUMMY, K_LIN_POINT, K_COUNT
};
static const char* const kKernelNames[K_COUNT] = {
    "cam_side", "lin_finalize", "point_colnorm", "scale", "memset_S", "assemble", "point_prep", "schur_tile",
    "obs_pairs", "chol", "update_cams", "backsub_eval", "final", "lm_decide", "xnorm", "bcr_elim", "bcr_contrib",
    "bcr_back", "bcr_border", "comm", "cam_reduce", "bcr_persist", "pp_reduce", "dummy", "lin_point"};

// Records an event pair around each launch on the launch stream.
struct Prof {
    static constexpr int MAXP = 640;
    int on = 0;
    int n = 0;
    int id[MAXP];
    hipEvent_t ev[2 * MAXP];
    unsigned mask = 0;  // bit k: record kernel id k (0 = every kernel)
    bool open_ = false;
    void begin(int k, hipStream_t s) {
        open_ = on && n < MAXP && (mask == 0 || ((mask >> k) & 1u));
        if (open_) { (void)hipEventRecord(ev[2 * n], s); id[n] = k; }
    }
    void end(hipStream_t s) {
        if (open_) { (void)hipEventRecord(ev[2 * n + 1], s); ++n; }
        open_ = false;
    }
};

// All kernels read cur / radius / done from W.st (device), so an LM iteration is a
// fixed launch sequence the host can enqueue without reading anything back.
// ---------------------------------------------------------------- per-device launch setup (host)
// hipFuncSetAttribute (the 160 KB dynamic LDS opt-in) applies to the CURRENT device only, and the API allows one
// context per host thread on any device (include/ba.h): the one-time setup of a launch path runs once per device,
// under a lock, and is retried if it failed. Diagnostic stamp buffers are kept per device the same way.
struct DeviceOnce {
    static constexpr int MAXDEV = 64;
    std::atomic<unsigned long long> done{0};
    std::mutex mu;
    template <class F>
    hipError_t operator()(F&& setup) {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        if (dev < 0 || dev >= MAXDEV) return hipErrorInvalidDevice;
        const unsigned long long bit = 1ull << dev;
        if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
        std::lock_guard<std::mutex> lock(mu);
        if (done.load(std::memory_order_relaxed) & bit) return hipSuccess;
        e = setup();
        if (e == hipSuccess) done.fetch_or(bit, std::memory_order_release);
        return e;
    }
};

// A device buffer per device (stamp diagnostics), grown to `bytes` on first use; nullptr on failure.
struct DeviceScratch {
    std::mutex mu;
    void* p[DeviceOnce::MAXDEV] = {};
    size_t cap[DeviceOnce::MAXDEV] = {};
    template <class T>
    T* get(size_t bytes) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= DeviceOnce::MAXDEV) return nullptr;
        std::lock_guard<std::mutex> lock(mu);
        if (cap[dev] < bytes) {
            if (p[dev]) (void)hipFree(p[dev]);
            p[dev] = nullptr;
            cap[dev] = 0;
            if (hipMalloc(&p[dev], bytes) != hipSuccess) return nullptr;
            cap[dev] = bytes;
        }
        return static_cast<T*>(p[dev]);
    }
};

// "1" in a MIBA_* diagnostic switch (read once per process: thread-safe function-local statics at the call sites)
inline int env_on(const char* name) {
    const char* e = std::getenv(name);
    return (e && e[0] == '1') ? 1 : 0;
}

hipError_t launch_linearize(const DevProblem& P, const BaConsts& c, int gated, DevWork& W, hipStream_t s, Prof* pf);
hipError_t launch_scale(const DevProblem& P, const BaConsts& c, int jacobi, DevWork& W, hipStream_t s, Prof* pf);
// progress: the host-mapped LM progress word (LmParams::progress), published with the done bit when the
// initial evaluation is non-finite (nullptr: none)
hipError_t launch_init_state(const DevProblem& P, DevWork& W, unsigned* progress, hipStream_t s, Prof* pf);
// ba_prepare's device side: the raw window as the caller passed it + the host plan's orderings (ba_plan.h)
struct PrepRaw {
    const int* cam;       // [n_obs] obs_cam
    const int* pt;        // [n_obs] obs_pt
    const double2* uv;    // [n_obs]
    const double* depth;  // [n_obs]
    const int* cam_ac;    // [n_cams] camera -> active index or -1
    const int* po_dest;   // [n_obs] observation -> point-major slot (-1: not admissible)
    const int* co_dest;   // [n_obs] observation -> camera-major slot (-1: not admissible)
    int n_obs;
};
// fills P.po_* (and po_ap / po_pt from pt_ptr / pt_idx) and P.co_* from R
hipError_t launch_prep_gather(const DevProblem& P, const PrepRaw& R, hipStream_t s);
// solve start: x and candidate slots <- prepared initial parameters, LM state <- st0
hipError_t launch_reset(const DevProblem& P, DevWork& W, const LmState& st0, const double* cams0, const double* pts0,
                        const double* K0, int n_cams, int n_points, hipStream_t s);
hipError_t launch_build(const DevProblem& P, const BaConsts& c, DevWork& W, hipStream_t s, Prof* pf);
hipError_t launch_factor(const DevProblem& P, const BaConsts& c, DevWork& W, hipStream_t s, Prof* pf);
// back-substitution, candidate evaluation, step scalars and the LM decision (k_final fuses k_lm_decide)
hipError_t launch_update(const DevProblem& P, const BaConsts& c, const LmParams& prm, DevWork& W, hipStream_t s,
                         Prof* pf);
hipError_t launch_decide(const DevProblem& P, const LmParams& prm, DevWork& W, hipStream_t s, Prof* pf);
// (Bw.persist drops to 0 when the device refuses the split kernel's cooperative launch)
hipError_t launch_bcr(const DevProblem& P, const BaConsts& c, DevWork& W, BcrWork& Bw, hipStream_t s, Prof* pf);
// 2 when the 2 * nblk workgroups of k_bcr_split can all be resident on the current device, else 1
// when the nblk workgroups of k_bcr_persist can, else 0
int bcr_persist_ok(int nblk);
int bcr_xmap_ok(int nblk, int persist);
int bcr_dense1_ok(int nblk, int kb);
// cameras per block of the one-workgroup band solve for this window (0: not eligible; MIBA_BCR_BAND)
// (one_block: also windows of one 64-dof block, where the band solve runs with its tail launch)
int bcr_band_ok(int nac, int cam_band, int kb, bool one_block);
hipError_t launch_bcr_band(const DevProblem& P, const BaConsts& c, DevWork& W, int bc, hipStream_t s, Prof* pf);
// the band solve + back-substitution + final decision in one launch (W.tail): nb_pt / nb_upd / nb_bs as k_final's
hipError_t launch_band_tail(const DevProblem& P, const BaConsts& c, const LmParams& prm, DevWork& W, int bc, int nb_pt,
                            int nb_upd, hipStream_t s, Prof* pf);
// workgroups of the tail launch (0: the window does not fit one resident round)
int band_tail_blocks(const DevProblem& P, int bc);
// the back-substitution chunks + the final reduction and decision in one launch (W.bsfin, unsharded fused windows)
hipError_t launch_backsub_final(const DevProblem& P, const BaConsts& c, const LmParams& prm, DevWork& W, int nb_pt,
                                int nb_upd, unsigned* bcr_epoch, hipStream_t s, Prof* pf);
hipError_t tail_set_spin_limit(unsigned limit);
// k_bcr_split's pull slots: empty (split = true, Bw.persist >= 2) or zero (the per-level / persistent paths)
hipError_t bcr_reset_pull_slots(const BcrWork& Bw, bool split, hipStream_t s);
// spin bound of the resident BCR kernels' inter-workgroup waits (default 1 << 22 polls; tests force a
// tiny bound to exercise the timeout path)
hipError_t bcr_set_spin_limit(unsigned limit);
// the small-window launch's wait for its camera side (ba_kernels.hip sw_wait)
hipError_t sw_set_spin_limit(unsigned limit);
// workgroups of k_schur_tile resident at once on the current device (CUs x blocks per CU)
int schur_tile_slots();
hipError_t launch_debug_lin(const DevProblem& P, const BaConsts& c, DevWork& W, double* res, double* jc, double* jp,
                            double* jk, hipStream_t s);

}  // namespace miba
