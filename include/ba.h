/*
 * ba.h — C-ABI of libmiba, the MI355X-native windowed bundle-adjustment solver.
 *
 * This is the drop-in boundary for the reference's hot path
 *
 *   bool windowOptimize(ceresGlobalProblem&, int kf_i, int kf_f,
 *                       vector<KeyFrame>&, Map3D&,
 *                       const Vector4d& intrinsics_initial,
 *                       Vector4d& intrinsics_optimized);
 *     declared  /root/reference/headers/OptimizationUtils.h:55
 *     defined   /root/reference/src/OptimizationUtils.cpp:215-313
 *
 * whose entire compute is `ceres::Solve(globalProblem.options, &problem, &summary)`
 * (src/OptimizationUtils.cpp:300) over the residual blocks built at :236-294.
 * The caller (a host adapter, see INTEGRATION.md and include/ba_window.hpp)
 * flattens the window into the SoA `ba_problem` below, calls ba_solve(), and
 * maps the results back (reference :303-310).
 *
 * Conventions
 *  - Plain C types only; every pointer is a caller-owned HOST buffer.
 *  - Poses use Sophus::SE3d storage order [qx,qy,qz,qw,tx,ty,tz]
 *    (reference headers/sophus/se3.hpp:469-479), T_w_c (camera -> window frame).
 *  - Updated in place: cams, points, intr (reference mutates T_w_c, map points
 *    and intrinsics_optimized in place, OptimizationUtils.cpp:248,274,236).
 *  - Return value: 0 = ok, <0 = error (see BA_E_*); ba_last_error() has text.
 *    The reference has no error convention (always returns true, :312); a
 *    Ceres-level failure (e.g. initial evaluation non-finite) is reported in
 *    ba_summary.termination_type exactly as Ceres would, with return 0.
 *  - One context per host thread; contexts cache device buffers across calls
 *    (the reference re-optimizes the same window repeatedly, main.cpp:163-168).
 */
#ifndef MIBA_BA_H
#define MIBA_BA_H

#include <stddef.h>
#include <stdint.h>
#include <string.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Version history:
 *   1  (rounds 1-5) ba_summary / ba_prepare_info without a size field; ba_prepare_info grew lin_path (r4),
 *      plan_device and tail (r5) under the same version.
 *   2  ba_summary and ba_prepare_info lead with `struct_size`: the caller sets it to sizeof() of ITS struct
 *      (BA_SUMMARY_INIT / BA_PREPARE_INFO_INIT), the library writes only that many bytes (fields a newer
 *      library added past the caller's size stay untouched) and rejects a size below the *_MIN_SIZE of this
 *      version with BA_E_INVALID. */
#define BA_API_VERSION 2

/* error codes */
#define BA_OK 0
#define BA_E_INVALID (-1)   /* bad argument / malformed problem */
#define BA_E_DEVICE (-2)    /* HIP runtime error / no device */
#define BA_E_NOMEM (-3)     /* allocation failed */
#define BA_E_COMM (-4)      /* RCCL / multi-device error */
#define BA_E_INTERNAL (-5)

/* Ceres 2.0 ceres::TerminationType values (types.h), mirrored numerically. */
#define BA_CONVERGENCE 0
#define BA_NO_CONVERGENCE 1
#define BA_FAILURE 2

/* Solver configuration.
 * Field-for-field mirror of ceresGlobalProblem
 * (/root/reference/headers/BundleAdjustmentConfig.h:44-69) plus the Ceres 2.0
 * Solver::Options defaults that the reference leaves untouched. */
typedef struct ba_options {
    /* ceresGlobalProblem constants, BundleAdjustmentConfig.h:47-50 */
    double hub_p_repr;         /* HUB_P_REPR = 1e-3: Huber a for reprojection blocks */
    double hub_p_unpr;         /* HUB_P_UNPR = 1e-3: Huber a for depth-prior blocks  */
    double weight_intrinsics;  /* WEIGHT_INTRINSICS = 1e-6 (IntrinsicsPrior weight)   */
    double weight_unpr;        /* WEIGHT_UNPR = 10 (depth prior weight numerator)     */
    /* Solver::Options set in initialize_options(), BundleAdjustmentConfig.h:61-67 */
    int32_t max_num_iterations;           /* 75 */
    int32_t minimizer_progress_to_stdout; /* 1 -> Ceres-style iteration table */
    double eta;                           /* 1e-6 (no effect on a direct Schur solve) */
    /* Ceres 2.0 defaults (not set by the reference) */
    double initial_trust_region_radius; /* 1e4  */
    double max_trust_region_radius;     /* 1e16 */
    double min_trust_region_radius;     /* 1e-32 */
    double min_relative_decrease;       /* 1e-3 */
    double min_lm_diagonal;             /* 1e-6 */
    double max_lm_diagonal;             /* 1e32 */
    int32_t max_num_consecutive_invalid_steps; /* 5 */
    int32_t jacobi_scaling;             /* 1 */
    double function_tolerance;          /* 1e-6 */
    double gradient_tolerance;          /* 1e-10 */
    double parameter_tolerance;         /* 1e-8 */
    /* MI355X execution knobs (no reference counterpart) */
    int32_t device;          /* HIP device ordinal for this context; -1 = current */
    int32_t deterministic;   /* 1 = fixed-order reductions only (no float atomics): bitwise-reproducible
                                solves (the Schur tiles write per-tile slabs summed in tile order; the
                                overflow Schur terms run in one workgroup), at some speed cost */
    int32_t profile_kernels; /* 1 = HIP-event timing of kernel launches (ba_kernel_stats) */
    int32_t profile_mask;    /* with profile_kernels: bit k selects kernel id k of ba_kernel_stats order; 0 = all */
    int32_t shard_min_obs;   /* landmark shards (ba_comm_init*): a window with fewer admissible observations
                                over all shards is gathered onto every rank at ba_prepare and solved there
                                alone (no per-iteration collectives, deterministic mode), each rank keeping
                                its own points; 0 = always run the sharded exchange. Default 262144 */
    int32_t small_window;    /* ignored: kept for layout compatibility (the round-2 single-workgroup small-window
                                kernel measured slower than the multi-launch path and was removed) */
    int32_t rebuild_plan;    /* 0 (default): ba_prepare / ba_solve reuse the context's host plan and device
                                structure when the window's structure is unchanged since the last prepare
                                (same sizes, fixed_cam, obs_cam, obs_pt, admissibility mask; the reference
                                re-optimises the same window every frame, main.cpp:163-168) and upload only the
                                parameters and the observation values that changed; 1 = rebuild every call.
                                Unsharded contexts only (landmark shards always rebuild) */
    int32_t reserved[1];
} ba_options;

/* One window, flattened. Mirrors what windowOptimize feeds to Ceres
 * (OptimizationUtils.cpp:236-294). Observations with depth <= 1e-15 are
 * skipped and excluded from the 1/N weight normaliser exactly like the
 * reference (countConstraints :184-213 and the skip at :265-268). */
typedef struct ba_problem {
    int32_t n_cams;
    int32_t n_points;
    int32_t n_obs;
    int32_t fixed_cam;        /* gauge: SetParameterBlockConstant(kf_i) (:299); -1 = none */
    double* cams;             /* [n_cams*7]  qx,qy,qz,qw,tx,ty,tz   (in/out) */
    double* points;           /* [n_points*3] (in/out) */
    double* intr;             /* [4] fx,fy,cx,cy (intrinsics_optimized, in/out) */
    const double* intr_prior; /* [4] intrinsics_initial (IntrinsicsPrior target, :238) */
    const int32_t* obs_cam;   /* [n_obs] camera index of each observation */
    const int32_t* obs_pt;    /* [n_obs] point index of each observation  */
    const double* obs_uv;     /* [n_obs*2] keypoint pixel (u,v)  (:262) */
    const double* obs_depth;  /* [n_obs] measured depth z (:261) */
} ba_problem;

/* Result summary (subset of ceres::Solver::Summary + per-phase device timings). */
/* ba_summary.linear_solver */
#define BA_LS_DENSE 0 /* dense-envelope LDS Cholesky */
#define BA_LS_BAND 1  /* banded LDS Cholesky (6x6 block band <= 6) */
#define BA_LS_BCR 2   /* block cyclic reduction over 64-dof camera blocks */

typedef struct ba_summary {
    int32_t struct_size;            /* in: sizeof(ba_summary) of the caller's header (BA_SUMMARY_INIT) */
    int32_t reserved0;
    double initial_cost;
    double final_cost;
    int32_t num_successful_steps;   /* Ceres convention: includes iteration 0 */
    int32_t num_unsuccessful_steps;
    int32_t num_iterations;         /* LM steps computed = iterations after 0 */
    int32_t termination_type;       /* BA_CONVERGENCE / BA_NO_CONVERGENCE / BA_FAILURE */
    int32_t num_obs_admissible;     /* N of countConstraints */
    int32_t num_active_cams;
    int32_t num_active_points;
    int32_t reduced_system_size;    /* 6*active_cams + 4 */
    int32_t linear_solver;          /* reduced-system solver used: BA_LS_DENSE / _BAND / _BCR */
    int32_t camera_band;            /* max |cam_a - cam_b| over coupled active cameras */
    double time_setup_ms;           /* host prep + H2D + structure build */
    double time_lm_ms;              /* LM loop wall time (device work + host control) */
    double time_linearize_ms;       /* device: camera-side / point-side linearisation */
    double time_schur_ms;           /* device: Schur reduction over points */
    double time_factor_ms;          /* device: reduced camera system factor + solve */
    double time_update_ms;          /* device: back-substitution + candidate evaluation */
    double time_total_ms;
    char message[160];
} ba_summary;
/* the smallest struct_size ba_solve / ba_solve_prepared accept: every field before `message` */
#define BA_SUMMARY_MIN_SIZE ((int32_t)offsetof(ba_summary, message))
#define BA_SUMMARY_INIT(s) (memset(&(s), 0, sizeof(s)), (s).struct_size = (int32_t)sizeof(s))

/* Library / API identification. */
int32_t ba_api_version(void);
const char* ba_build_info(void);

/* Defaults = ceresGlobalProblem() + Ceres 2.0 defaults. */
void ba_default_options(ba_options* opts);

/* Context lifecycle. Returns NULL on failure (ba_last_error(NULL) explains). */
typedef struct ba_context ba_context;
ba_context* ba_create(const ba_options* opts);
void ba_destroy(ba_context* ctx);
/* Text of the context's last failed call; after a successful ba_solve / ba_solve_prepared it is empty, or a
 * note (e.g. LM iterations re-run with the per-level BCR launches after a resident-kernel hand-off timeout). */
const char* ba_last_error(const ba_context* ctx);
/* Replace the solver options of a live context (device buffers are kept;
 * opts->device must equal the context's device or be -1). */
int32_t ba_set_options(ba_context* ctx, const ba_options* opts);

/* Solve one window in place (the replacement of ceres::Solve at :300).
 * Equivalent to ba_prepare() followed by ba_solve_prepared(). summary->struct_size must be set
 * (BA_SUMMARY_INIT); min(struct_size, sizeof(ba_summary)) bytes are written. */
int32_t ba_solve(ba_context* ctx, ba_problem* prob, ba_summary* summary);

/* Split form of ba_solve for callers that re-solve a resident window:
 * ba_prepare() validates the window, builds the point-/camera-major orderings
 * and the reduced-system envelope on the host and uploads everything to HBM;
 * ba_solve_prepared() runs the LM loop on the resident window starting from the
 * parameters uploaded by the last ba_prepare() and writes the result into prob
 * (which must be the same window, same sizes). */
int32_t ba_prepare(ba_context* ctx, const ba_problem* prob);
int32_t ba_solve_prepared(ba_context* ctx, ba_problem* prob, ba_summary* summary);

/* What the last ba_prepare (or the prepare inside ba_solve / the debug hooks) did. */
typedef struct ba_prepare_info {
    int32_t struct_size;     /* in: sizeof(ba_prepare_info) of the caller's header (BA_PREPARE_INFO_INIT) */
    int32_t plan_reused;     /* 1: the window's structure matched the context's last plan (no plan rebuild) */
    int32_t obs_uploaded;    /* 1: observation values were uploaded (always on a rebuild; on a reuse only when
                                some pixel / depth value changed) */
    int32_t host_threads;    /* host plan threads (MIBA_HOST_THREADS, else min(16, OMP_NUM_THREADS, affinity)) */
    int32_t bcr_path;        /* reduced-solve path of the prepared window: 5 = narrow camera band (<= 3), the
                                whole system cyclic-reduced in one workgroup's LDS; 4 = one-block window, dense
                                single-workgroup solve; 3 / 2 = resident split kernel with two / one helper
                                workgroups per block, 1 = resident one-workgroup kernel, 0 = per-level launches,
                                -1 = not the block cyclic reduction (band / dense) */
    double compare_ms;       /* structure / value comparison against the last prepare (reuse check) */
    double plan_ms;          /* host plan build (0 on a reuse) */
    double upload_ms;        /* staging + enqueue of the uploads and the device gather */
    double total_ms;         /* the whole prepare, device work included */
    int32_t lin_path;        /* linearisation of the LM loop: 1 = small window, the point side inside the Schur
                                tiles and the camera side in the Schur launch (no separate linearisation launch);
                                0 = a linearisation launch before the Schur launch */
    int32_t plan_device;     /* 1: the window's plan passes ran on the device (MIBA_DEVICE_PLAN; 0 on a reuse) */
    int32_t tail;            /* 1: the band solve's launch also runs the point back-substitution and the LM
                                decision (bcr_path 5, small unsharded windows; MIBA_TAIL=0: separate launches) */
    int32_t bsfin;           /* 1: the point back-substitution and the LM decision run in one launch (larger
                                unsharded windows, k_backsub_final; opt-in, MIBA_BSFIN=1) — version 2 */
} ba_prepare_info;
/* the smallest struct_size ba_last_prepare accepts: the fields through total_ms (the round-3 layout) */
#define BA_PREPARE_INFO_MIN_SIZE ((int32_t)(offsetof(ba_prepare_info, total_ms) + sizeof(double)))
#define BA_PREPARE_INFO_INIT(s) (memset(&(s), 0, sizeof(s)), (s).struct_size = (int32_t)sizeof(s))
/* Writes min(info->struct_size, sizeof(ba_prepare_info)) bytes; BA_E_INVALID below BA_PREPARE_INFO_MIN_SIZE. */
int32_t ba_last_prepare(const ba_context* ctx, ba_prepare_info* info);

/* Landmark sharding (one process per GPU). Every rank passes the SAME window
 * cameras, intrinsics, prior and fixed_cam to ba_solve / ba_prepare, and its OWN block of
 * landmarks (points with all their observations). Per LM iteration the ranks all-reduce
 * (RCCL over xGMI) the camera-side partials, the packed envelope of the reduced camera
 * system and the step scalars; every rank then runs the identical deterministic solve of
 * the reduced system, so poses and intrinsics stay bitwise identical across ranks and each
 * rank updates its own points. Rank 0 calls ba_comm_unique_id() and ships the id to the
 * other ranks (any host channel); then every rank calls ba_comm_init() collectively.
 * Sharding pays only when the per-rank point work exceeds the all-reduce time (a few
 * tens of us per iteration over xGMI): small windows should stay on one GPU. */
#define BA_COMM_ID_BYTES 128
int32_t ba_comm_unique_id(uint8_t id[BA_COMM_ID_BYTES]);
int32_t ba_comm_init(ba_context* ctx, int32_t nranks, int32_t rank, const uint8_t id[BA_COMM_ID_BYTES]);

/* The same landmark sharding over a caller-supplied host collective instead of RCCL (e.g. MPI,
 * or torch.distributed gloo in the multi-rank tests, where several ranks share one GPU and RCCL
 * refuses duplicate devices). fn reduces `count` elements of the host buffer `buf` in place across
 * the ranks and returns 0 on success (dtype BA_DTYPE_*, op BA_OP_*); libmiba calls it on the
 * thread running ba_solve, at the same points of the LM iteration as the RCCL collectives, with
 * the device data staged through pinned memory. Local (not collective): every rank calls it once. */
#define BA_DTYPE_F64 0
#define BA_DTYPE_I32 1
#define BA_OP_SUM 0
#define BA_OP_MAX 1
#define BA_OP_MIN 2
typedef int32_t (*ba_allreduce_fn)(void* buf, int64_t count, int32_t dtype, int32_t op, void* user);
int32_t ba_comm_init_host(ba_context* ctx, int32_t nranks, int32_t rank, ba_allreduce_fn fn, void* user);

/* Per-iteration log of the last solve, the rows Ceres prints with minimizer_progress_to_stdout
 * (iteration 0 .. num_iterations): cost, cost_change, |gradient|_inf, |step|, tr_ratio, tr_radius,
 * accepted (1 = successful step, 0 = unsuccessful / invalid, -1 = the step that met a tolerance),
 * 0. Returns the number of rows available (at most max_rows are written; rows may be NULL). */
#define BA_LOG_WIDTH 8
int32_t ba_iteration_log(const ba_context* ctx, double* rows, int32_t max_rows);

/* Per-kernel device timing (requires ba_options.profile_kernels = 1).
 * bytes_per_launch is the ALGORITHMIC traffic model of DESIGN.md §Roofline
 * for the last prepared window (compulsory bytes, each input/output once). */
typedef struct ba_kernel_stat {
    char name[32];
    int32_t launches;
    int32_t reserved;
    double total_ms;
    double bytes_per_launch;
    double flops_per_launch;
} ba_kernel_stat;
int32_t ba_kernel_stats(const ba_context* ctx, ba_kernel_stat* out, int32_t max_n); /* returns count */
void ba_reset_kernel_stats(ba_context* ctx);

/* ---- verification hooks (used by the parity tests; not on the hot path) ----
 * Evaluate per-observation robustified residuals and local Jacobians on the
 * device at the given parameters. Output layout per admissible observation k
 * in the ORIGINAL observation order (inadmissible rows are zero):
 *   res[k*3+{0,1,2}]   : sqrt(rho') * (reproj u, reproj v, depth) residual
 *   jcam[k*18 + r*6+d] : d res_r / d delta_d, delta = [upsilon(3), omega(3)]
 *   jpt [k*9  + r*3+i] : d res_r / d X_i
 *   jint[k*8  + r*4+i] : d res_r / d (fx,fy,cx,cy)_i  (rows 0,1; depth row is 0)
 * cost receives 0.5 * sum_blocks rho(|f_b|^2) including the intrinsics prior.
 * Any output pointer may be NULL. */
int32_t ba_debug_linearize(ba_context* ctx, const ba_problem* prob, double* cost,
                           double* res, double* jcam, double* jpt, double* jint);

/* Build the damped, Jacobi-scaled reduced camera system exactly as the first
 * LM iteration would (radius = initial_trust_region_radius unless radius > 0):
 * S [n*n] row-major dense (full symmetric), rhs [n], scale [6*n_cams + 3*n_points + 4]
 * where n = 6*active_cams + 4; active cameras in increasing index order. */
int32_t ba_debug_reduced_system(ba_context* ctx, const ba_problem* prob, double radius,
                                int32_t* n_out, double* S, double* rhs);

/* Test hook: the production camera-side pass (k_cam_side + k_cam_finalize, iteration-0 form) at the
 * problem's parameters. camdata[nac*51]: per active camera U upper-packed (21) | C 6x4 (24) | g (6);
 * lin[16]: cost, gradient max-norm of cameras + intrinsics, Ukk packed (10, + IntrinsicsPrior), gk (4,
 * + prior); ac_cam[nac]: the camera index of each active camera. With NULL outputs only *nac is set. */
int32_t ba_debug_camera_sums(ba_context* ctx, const ba_problem* prob, int32_t* nac, double* camdata,
                             double* lin, int32_t* ac_cam);

/* Test hook: FNV-1a digests of the last prepared window's plan arrays as the kernels read them from HBM (the
 * observation orderings, point order, tiles, chunks, segments, envelope), one per array, into out[max_n].
 * Returns the number of arrays. The host plan and the device plan (MIBA_DEVICE_PLAN) give the same digests. */
int32_t ba_debug_plan_digest(ba_context* ctx, uint64_t* out, int32_t max_n);

#ifdef __cplusplus
}
#endif
#endif /* MIBA_BA_H */
