/*
 * ba_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + cpu_baseline leg).
 *
 * CPU float64 restatement of the reference hot path
 *     windowOptimize -> ceres::Solve   (/root/reference/src/OptimizationUtils.cpp:215-313)
 * Never linked into, loaded by, or called from the product (libmiba). Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 *
 * PARITY STATUS: the reference's arithmetic lives in Ceres Solver 2.0.0 and
 * Eigen 3.4.0 (reference conanfile.txt:2,4), neither vendored nor installed,
 * and the reference has no test / golden vector for this path.
 * This restatement is therefore "parity unpinned" against Ceres itself; it is
 * cross-checked against an independent minimiser (scipy least_squares) and
 * finite differences in tests/ (see DESIGN.md "Oracle").
 *
 * What is restated (each function cites the reference / third-party source):
 *   - ReprojectionConstraint::operator()  OptimizationUtils.cpp:25-49
 *   - DepthPrior::operator()              OptimizationUtils.cpp:72-94
 *   - IntrinsicsPrior::operator()         OptimizationUtils.cpp:117-125
 *   - weights 1/N, WEIGHT_UNPR/N, WEIGHT_INTRINSICS  :238,280,290; N = countConstraints :184-213
 *   - Huber(1e-3) per residual block, Ceres HuberLoss + Corrector       :223-226
 *   - Sophus LocalParameterizationSE3::Plus  T*exp(delta)   local_parameterization_se3.hpp:17-24,
 *       SE3::exp se3.hpp:725-746, SO3::expAndTheta so3.hpp:537-571, SO3 *= renorm so3.hpp:339-356
 *   - analytic local Jacobian == ambient AutoDiff Jacobian x Dx_this_mul_exp_x_at_0 (se3.hpp:113-182)
 *   - Ceres 2.0 TrustRegionMinimizer + LevenbergMarquardtStrategy + SPARSE_SCHUR
 *     (third-party, restated from the published Ceres 2.0 algorithm)
 */
#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/ba.h"

#define EXPORT __attribute__((visibility("default")))

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/* ------------------------------------------------------------------ */
/* defaults: ceresGlobalProblem (BundleAdjustmentConfig.h:47-67) + Ceres 2.0 */
EXPORT void oracle_default_options(ba_options* o) {
    memset(o, 0, sizeof(*o));
    o->hub_p_repr = 1e-3;
    o->hub_p_unpr = 1e-3;
    o->weight_intrinsics = 1e-6;
    o->weight_unpr = 10.0;
    o->max_num_iterations = 75;
    o->minimizer_progress_to_stdout = 1;
    o->eta = 1e-6;
    o->initial_trust_region_radius = 1e4;
    o->max_trust_region_radius = 1e16;
    o->min_trust_region_radius = 1e-32;
    o->min_relative_decrease = 1e-3;
    o->min_lm_diagonal = 1e-6;
    o->max_lm_diagonal = 1e32;
    o->max_num_consecutive_invalid_steps = 5;
    o->jacobi_scaling = 1;
    o->function_tolerance = 1e-6;
    o->gradient_tolerance = 1e-10;
    o->parameter_tolerance = 1e-8;
    o->device = -1;
    o->deterministic = 0;        /* the oracle is single-ordered anyway; mirrors ba_default_options */
    o->shard_min_obs = 262144;   /* libmiba execution knob, unused here */
}

/* ------------------------------------------------------------------ */
/* SE(3) / quaternion helpers (Eigen / Sophus semantics)               */

/* Eigen::QuaternionBase::toRotationMatrix, q = (w=pose[3], x=pose[0], y=pose[1], z=pose[2])
 * as built at OptimizationUtils.cpp:36-37 and used via q.matrix() at :41. */
static void quat_R(const double* pose, double R[9]) {
    const double x = pose[0], y = pose[1], z = pose[2], w = pose[3];
    const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
    const double twx = tx * w, twy = ty * w, twz = tz * w;
    const double txx = tx * x, txy = ty * x, txz = tz * x;
    const double tyy = ty * y, tyz = tz * y, tzz = tz * z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

/* Sophus::SE3d::exp (se3.hpp:725-746) + SO3::expAndTheta (so3.hpp:537-571),
 * then T * exp(delta) via SE3 operator*= (se3.hpp:317-320) and the SO3 quaternion
 * renormalisation (so3.hpp:339-356). delta = [upsilon(3), omega(3)]. */
static void se3_plus(const double* T, const double* d, double* out) {
    const double ox = d[3], oy = d[4], oz = d[5];
    const double theta_sq = ox * ox + oy * oy + oz * oz;
    const double theta = sqrt(theta_sq);
    const double half = 0.5 * theta;
    double imag, real;
    if (theta < 1e-10) { /* Sophus::Constants<double>::epsilon(), common.hpp:144 */
        const double t4 = theta_sq * theta_sq;
        imag = 0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * t4;
        real = 1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * t4;
    } else {
        imag = sin(half) / theta;
        real = cos(half);
    }
    /* q_d = (w=real, imag*omega) */
    double qd[4] = {imag * ox, imag * oy, imag * oz, real}; /* xyzw */
    double V[9];
    if (theta < 1e-10) {
        quat_R(qd, V);
    } else {
        const double Om[9] = {0, -oz, oy, oz, 0, -ox, -oy, ox, 0};
        double Om2[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                double s = 0;
                for (int k = 0; k < 3; ++k) s += Om[i * 3 + k] * Om[k * 3 + j];
                Om2[i * 3 + j] = s;
            }
        const double a = (1.0 - cos(theta)) / theta_sq;
        const double b = (theta - sin(theta)) / (theta_sq * theta);
        for (int i = 0; i < 9; ++i) V[i] = ((i % 4) == 0 ? 1.0 : 0.0) + a * Om[i] + b * Om2[i];
    }
    double td[3];
    for (int i = 0; i < 3; ++i) td[i] = V[i * 3 + 0] * d[0] + V[i * 3 + 1] * d[1] + V[i * 3 + 2] * d[2];
    /* translation += so3 * td  (Eigen _transformVector: v + w*uv + q.vec x uv, uv = 2 q.vec x v) */
    const double qx = T[0], qy = T[1], qz = T[2], qw = T[3];
    double uv[3] = {2 * (qy * td[2] - qz * td[1]), 2 * (qz * td[0] - qx * td[2]), 2 * (qx * td[1] - qy * td[0])};
    double rv[3] = {td[0] + qw * uv[0] + (qy * uv[2] - qz * uv[1]),
                    td[1] + qw * uv[1] + (qz * uv[0] - qx * uv[2]),
                    td[2] + qw * uv[2] + (qx * uv[1] - qy * uv[0])};
    out[4] = T[4] + rv[0];
    out[5] = T[5] + rv[1];
    out[6] = T[6] + rv[2];
    /* quaternion product q * q_d (Eigen, w-last storage) */
    const double bx = qd[0], by = qd[1], bz = qd[2], bw = qd[3];
    double nw = qw * bw - qx * bx - qy * by - qz * bz;
    double nx = qw * bx + qx * bw + qy * bz - qz * by;
    double ny = qw * by + qy * bw + qz * bx - qx * bz;
    double nz = qw * bz + qz * bw + qx * by - qy * bx;
    const double sq = nx * nx + ny * ny + nz * nz + nw * nw;
    if (sq != 1.0) {
        const double f = 2.0 / (1.0 + sq);
        nx *= f; ny *= f; nz *= f; nw *= f;
    }
    out[0] = nx; out[1] = ny; out[2] = nz; out[3] = nw;
}


/* ------------------------------------------------------------------ */
/* execution knobs of the restatement (not of the reference): OpenMP threads and the
 * storage of the reduced camera system. threads = 1 and profile = 0 (full lower
 * triangle, dense Cholesky) is the checker configuration; the CPU baseline leg runs
 * the profile (skyline) storage — the Ceres SPARSE_SCHUR stand-in, whose fill stays
 * inside the co-visibility envelope — at 1 and at all host threads.             */
static int g_threads = 1;
static int g_profile = 0;

EXPORT void oracle_config(int32_t threads, int32_t profile) {
    g_threads = threads < 1 ? 1 : threads;
#ifndef _OPENMP
    g_threads = 1;
#endif
    g_profile = profile ? 1 : 0;
}
EXPORT int32_t oracle_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

static inline int tid(void) {
#ifdef _OPENMP
    return omp_get_thread_num();
#else
    return 0;
#endif
}
/* contiguous chunk [lo, hi) of n items for thread t of T */
static inline void chunk(int n, int t, int T, int* lo, int* hi) {
    *lo = (int)((long long)n * t / T);
    *hi = (int)((long long)n * (t + 1) / T);
}

/* ------------------------------------------------------------------ */
/* problem bookkeeping                                                  */
typedef struct {
    const ba_problem* p;
    ba_options o;
    int n_adm;       /* N: admissible observations (countConstraints) */
    int* adm;        /* admissible obs -> original obs index */
    int* cam_ac;     /* camera -> active index or -1 */
    int nac, n;      /* active cams, reduced system size */
    int* pt_active;
    int n_act_pts;
    int* pt_ptr;     /* CSR over admissible obs by point */
    int* pt_obs;     /* admissible indices */
    int max_m;       /* max admissible observations of one point */
    double sw_r, sw_d, sw_k; /* sqrt weights */
    /* lower profile of the reduced system S (n x n): row i holds columns [fc[i], i]
     * at a[rp[i] + j - fc[i]]; the 4 intrinsics rows are last and full (arrowhead border) */
    int* fc;
    size_t* rp;
    size_t nnz;
} orc_t;

static void orc_free(orc_t* c) {
    free(c->adm); free(c->cam_ac); free(c->pt_active); free(c->pt_ptr); free(c->pt_obs);
    free(c->fc); free(c->rp);
}

static int orc_init(orc_t* c, const ba_problem* p, const ba_options* o) {
    memset(c, 0, sizeof(*c));
    c->p = p;
    c->o = *o;
    if (p->n_cams < 0 || p->n_points < 0 || p->n_obs < 0) return -1;
    c->adm = (int*)malloc(sizeof(int) * (p->n_obs + 1));
    c->cam_ac = (int*)malloc(sizeof(int) * (p->n_cams + 1));
    c->pt_active = (int*)calloc(p->n_points + 1, sizeof(int));
    c->pt_ptr = (int*)calloc(p->n_points + 2, sizeof(int));
    c->pt_obs = (int*)malloc(sizeof(int) * (p->n_obs + 1));
    int* cam_has = (int*)calloc(p->n_cams + 1, sizeof(int));
    /* countConstraints (:184-213) + skip at :265-268: depth <= 1e-15 is inadmissible */
    for (int k = 0; k < p->n_obs; ++k) {
        const int ci = p->obs_cam[k], pi = p->obs_pt[k];
        if (ci < 0 || ci >= p->n_cams || pi < 0 || pi >= p->n_points) { free(cam_has); return -1; }
        if (!(p->obs_depth[k] > 1e-15)) continue;
        c->adm[c->n_adm++] = k;
        cam_has[ci] = 1;
        c->pt_active[pi] = 1;
        c->pt_ptr[pi + 1]++;
    }
    /* unused parameter blocks are removed by the Ceres preprocessor; the gauge
     * block is constant (SetParameterBlockConstant, :299) */
    c->nac = 0;
    for (int i = 0; i < p->n_cams; ++i)
        c->cam_ac[i] = (cam_has[i] && i != p->fixed_cam) ? c->nac++ : -1;
    free(cam_has);
    c->n = 6 * c->nac + 4;
    for (int i = 0; i < p->n_points; ++i) {
        c->n_act_pts += c->pt_active[i];
        const int m = c->pt_ptr[i + 1];
        if (m > c->max_m) c->max_m = m;
        c->pt_ptr[i + 1] += c->pt_ptr[i];
    }
    int* fill = (int*)malloc(sizeof(int) * (p->n_points + 1));
    memcpy(fill, c->pt_ptr, sizeof(int) * (p->n_points + 1));
    for (int a = 0; a < c->n_adm; ++a) c->pt_obs[fill[p->obs_pt[c->adm[a]]]++] = a;
    free(fill);
    /* profile of S: first co-visible active camera of every active camera */
    int* fcam = (int*)malloc(sizeof(int) * (c->nac + 1));
    for (int a = 0; a < c->nac; ++a) fcam[a] = a;
    for (int pi = 0; pi < p->n_points; ++pi) {
        int lo = c->nac;
        for (int q = c->pt_ptr[pi]; q < c->pt_ptr[pi + 1]; ++q) {
            const int ac = c->cam_ac[p->obs_cam[c->adm[c->pt_obs[q]]]];
            if (ac >= 0 && ac < lo) lo = ac;
        }
        for (int q = c->pt_ptr[pi]; q < c->pt_ptr[pi + 1]; ++q) {
            const int ac = c->cam_ac[p->obs_cam[c->adm[c->pt_obs[q]]]];
            if (ac >= 0 && lo < fcam[ac]) fcam[ac] = lo;
        }
    }
    c->fc = (int*)malloc(sizeof(int) * (c->n + 1));
    c->rp = (size_t*)malloc(sizeof(size_t) * (c->n + 1));
    size_t off = 0;
    for (int r = 0; r < c->n; ++r) {
        c->fc[r] = (g_profile && r < 6 * c->nac) ? 6 * fcam[r / 6] : 0;
        c->rp[r] = off;
        off += (size_t)(r - c->fc[r] + 1);
    }
    c->rp[c->n] = off;
    c->nnz = off;
    free(fcam);
    const double N = (double)c->n_adm;
    c->sw_r = sqrt(1.0 / N);                 /* ReprojectionConstraint weight 1/N (:280) */
    c->sw_d = sqrt(o->weight_unpr / N);      /* DepthPrior weight WEIGHT_UNPR/N (:290) */
    c->sw_k = sqrt(o->weight_intrinsics);    /* IntrinsicsPrior weight (:238) */
    return 0;
}

/* Per-observation robustified residual and local Jacobians.
 * Returns the block cost 0.5*rho_r + 0.5*rho_d; 0 on success, -1 if non-finite. */
static int eval_obs(const orc_t* c, const double* pose, const double* X, const double* K,
                    double u_obs, double v_obs, double depth, double f[3], double* jc, double* jp,
                    double* jk, double* cost) {
    double R[9];
    quat_R(pose, R);
    const double d0 = X[0] - pose[4], d1 = X[1] - pose[5], d2 = X[2] - pose[6];
    /* p_C = R^T (p_W - t)  (:41) */
    const double x = R[0] * d0 + R[3] * d1 + R[6] * d2;
    const double y = R[1] * d0 + R[4] * d1 + R[7] * d2;
    const double z = R[2] * d0 + R[5] * d1 + R[8] * d2;
    const double fx = K[0], fy = K[1], cx = K[2], cy = K[3];
    /* (K p_C / z)(0:1)  (:42) */
    const double u = (fx * x + cx * z) / z;
    const double v = (fy * y + cy * z) / z;
    double r0 = c->sw_r * (u - u_obs); /* :45-46 */
    double r1 = c->sw_r * (v - v_obs);
    double r2 = c->sw_d * (depth - z); /* :91 */
    /* Huber per block (Ceres HuberLoss::Evaluate), corrector = sqrt(rho') since rho'' <= 0 */
    const double ar = c->o.hub_p_repr, br = ar * ar;
    const double ad = c->o.hub_p_unpr, bd = ad * ad;
    const double sr = r0 * r0 + r1 * r1, sd = r2 * r2;
    double rho0r, rho1r, rho0d, rho1d;
    if (sr > br) { const double q = sqrt(sr); rho0r = 2 * ar * q - br; rho1r = fmax(DBL_MIN, ar / q); }
    else { rho0r = sr; rho1r = 1.0; }
    if (sd > bd) { const double q = sqrt(sd); rho0d = 2 * ad * q - bd; rho1d = fmax(DBL_MIN, ad / q); }
    else { rho0d = sd; rho1d = 1.0; }
    *cost = 0.5 * rho0r + 0.5 * rho0d;
    if (!isfinite(*cost) || !isfinite(u) || !isfinite(v)) return -1;
    const double gr = sqrt(rho1r), gd = sqrt(rho1d);
    f[0] = gr * r0; f[1] = gr * r1; f[2] = gd * r2;
    if (!jc) return 0;
    const double iz = 1.0 / z;
    /* d(u,v)/d p_C, scaled by sqrt(w) * sqrt(rho') */
    const double su = gr * c->sw_r;
    const double a00 = su * fx * iz, a02 = -su * fx * x * iz * iz;
    const double a11 = su * fy * iz, a12 = -su * fy * y * iz * iz;
    const double dz = -gd * c->sw_d; /* d r2 / d z */
    /* rows: [du/dpC; dv/dpC; dr2/dpC] */
    const double A[9] = {a00, 0, a02, 0, a11, a12, 0, 0, dz};
    /* d p_C / d delta = [-I | [p_C]x],  d p_C / d X = R^T */
    const double P[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    for (int r = 0; r < 3; ++r) {
        for (int i = 0; i < 3; ++i) {
            jc[r * 6 + i] = -A[r * 3 + i];
            double s = 0;
            for (int k = 0; k < 3; ++k) s += A[r * 3 + k] * P[k * 3 + i];
            jc[r * 6 + 3 + i] = s;
            double t = 0;
            for (int k = 0; k < 3; ++k) t += A[r * 3 + k] * R[i * 3 + k]; /* (R^T)_{k i} = R_{i k} */
            jp[r * 3 + i] = t;
        }
    }
    /* intrinsics: du/dfx = x/z, du/dcx = 1; dv/dfy = y/z, dv/dcy = 1 */
    jk[0] = su * x * iz; jk[1] = 0; jk[2] = su; jk[3] = 0;
    jk[4] = 0; jk[5] = su * y * iz; jk[6] = 0; jk[7] = su;
    return 0;
}

/* Linearisation storage over admissible observations */
typedef struct {
    double* f;  /* [n_adm*3] */
    double* jc; /* [n_adm*18] */
    double* jp; /* [n_adm*9] */
    double* jk; /* [n_adm*8] */
    double fk[4]; /* intrinsics prior residual */
} lin_t;

static int lin_alloc(lin_t* L, int n) {
    L->f = (double*)malloc(sizeof(double) * 3 * (n + 1));
    L->jc = (double*)malloc(sizeof(double) * 18 * (n + 1));
    L->jp = (double*)malloc(sizeof(double) * 9 * (n + 1));
    L->jk = (double*)malloc(sizeof(double) * 8 * (n + 1));
    return (L->f && L->jc && L->jp && L->jk) ? 0 : -1;
}
static void lin_free(lin_t* L) { free(L->f); free(L->jc); free(L->jp); free(L->jk); }

/* Evaluate cost (and Jacobians if L != NULL). Returns 0 ok, -1 non-finite.
 * Per-thread partial costs over contiguous observation ranges, summed in thread order. */
static int evaluate(const orc_t* c, const double* cams, const double* pts, const double* K, lin_t* L,
                    double* cost_out) {
    const ba_problem* p = c->p;
    const int T = g_threads;
    double part[T];
    int badv[T];
#pragma omp parallel num_threads(T)
    {
        const int t = tid();
        int lo, hi;
        chunk(c->n_adm, t, T, &lo, &hi);
        double cost = 0, f[3];
        int bad = 0;
        for (int a = lo; a < hi && !bad; ++a) {
            const int k = c->adm[a];
            double cb;
            bad = eval_obs(c, cams + 7 * p->obs_cam[k], pts + 3 * p->obs_pt[k], K, p->obs_uv[2 * k],
                           p->obs_uv[2 * k + 1], p->obs_depth[k], L ? L->f + 3 * a : f,
                           L ? L->jc + 18 * a : NULL, L ? L->jp + 9 * a : NULL, L ? L->jk + 8 * a : NULL, &cb);
            cost += cb;
        }
        part[t] = cost;
        badv[t] = bad;
    }
    double cost = 0;
    for (int t = 0; t < T; ++t) {
        if (badv[t]) return -1;
        cost += part[t];
    }
    /* IntrinsicsPrior (:117-125), squared loss */
    double ck = 0;
    for (int i = 0; i < 4; ++i) {
        const double r = c->sw_k * (p->intr_prior[i] - K[i]);
        if (L) L->fk[i] = r;
        ck += r * r;
    }
    cost += 0.5 * ck;
    if (!isfinite(cost)) return -1;
    *cost_out = cost;
    return 0;
}

/* Parameter-vector layout used for the Jacobi scale / LM diagonal (local coords):
 * cams: 6*nac, points: 3*n_points (inactive points unused), intr: 4 */
static inline int off_pt(const orc_t* c, int pi) { return 6 * c->nac + 3 * pi; }
static inline int off_k(const orc_t* c) { return 6 * c->nac + 3 * c->p->n_points; }
static inline int nloc(const orc_t* c) { return 6 * c->nac + 3 * c->p->n_points + 4; }

/* Squared column norms of the (robustified) Jacobian (Ceres SparseMatrix::SquaredColumnNorm)
 * and the gradient g = J^T f (local coords, unscaled), point-major: each point's entries
 * are owned by one thread, the camera / intrinsics entries are per-thread partials summed
 * in thread order. Either output may be NULL. */
static void colnorm_grad(const orc_t* c, const lin_t* L, double* cn, double* g) {
    const ba_problem* p = c->p;
    const int T = g_threads, nf = 6 * c->nac + 4;
    double* pc = (double*)calloc((size_t)T * 2 * nf + 1, sizeof(double)); /* [t][cn | g] camera + intr */
    if (cn) memset(cn, 0, sizeof(double) * nloc(c));
    if (g) memset(g, 0, sizeof(double) * nloc(c));
#pragma omp parallel num_threads(T)
    {
        const int t = tid();
        double* mc = pc + (size_t)t * 2 * nf;
        double* mg = mc + nf;
        int lo, hi;
        chunk(p->n_points, t, T, &lo, &hi);
        for (int pi = lo; pi < hi; ++pi)
            for (int q = c->pt_ptr[pi]; q < c->pt_ptr[pi + 1]; ++q) {
                const int a = c->pt_obs[q];
                const int ac = c->cam_ac[p->obs_cam[c->adm[a]]];
                const double* jc = L->jc + 18 * a;
                const double* jp = L->jp + 9 * a;
                const double* jk = L->jk + 8 * a;
                const double* f = L->f + 3 * a;
                const int op = off_pt(c, pi);
                for (int r = 0; r < 3; ++r) {
                    if (ac >= 0)
                        for (int d = 0; d < 6; ++d) {
                            mc[6 * ac + d] += jc[r * 6 + d] * jc[r * 6 + d];
                            mg[6 * ac + d] += jc[r * 6 + d] * f[r];
                        }
                    for (int i = 0; i < 3; ++i) {
                        if (cn) cn[op + i] += jp[r * 3 + i] * jp[r * 3 + i];
                        if (g) g[op + i] += jp[r * 3 + i] * f[r];
                    }
                }
                for (int r = 0; r < 2; ++r)
                    for (int i = 0; i < 4; ++i) {
                        mc[6 * c->nac + i] += jk[r * 4 + i] * jk[r * 4 + i];
                        mg[6 * c->nac + i] += jk[r * 4 + i] * f[r];
                    }
            }
    }
    const int ok = off_k(c);
    for (int t = 0; t < T; ++t) {
        const double* mc = pc + (size_t)t * 2 * nf;
        for (int j = 0; j < nf; ++j) {
            const int dst = j < 6 * c->nac ? j : ok + (j - 6 * c->nac);
            if (cn) cn[dst] += mc[j];
            if (g) g[dst] += mc[nf + j];
        }
    }
    for (int i = 0; i < 4; ++i) {
        if (cn) cn[ok + i] += c->sw_k * c->sw_k; /* prior: J = -sqrt(w) I */
        if (g) g[ok + i] += -c->sw_k * L->fk[i];
    }
    free(pc);
}

/* 3x3 SPD inverse via Cholesky; returns -1 if not PD */
static int inv3_spd(const double V[9], double Vi[9]) {
    const double l00 = V[0];
    if (!(l00 > 0)) return -1;
    const double L00 = sqrt(l00);
    const double L10 = V[3] / L00, L20 = V[6] / L00;
    const double l11 = V[4] - L10 * L10;
    if (!(l11 > 0)) return -1;
    const double L11 = sqrt(l11);
    const double L21 = (V[7] - L20 * L10) / L11;
    const double l22 = V[8] - L20 * L20 - L21 * L21;
    if (!(l22 > 0)) return -1;
    const double L22 = sqrt(l22);
    /* inverse of L */
    const double i00 = 1 / L00, i11 = 1 / L11, i22 = 1 / L22;
    const double i10 = -L10 * i00 * i11;
    const double i21 = -L21 * i11 * i22;
    const double i20 = -(L20 * i00 + L21 * i10) * i22;
    const double Li[9] = {i00, 0, 0, i10, i11, 0, i20, i21, i22};
    /* Vi = Li^T Li */
    for (int r = 0; r < 3; ++r)
        for (int s = 0; s < 3; ++s) {
            double acc = 0;
            for (int k = 0; k < 3; ++k) acc += Li[k * 3 + r] * Li[k * 3 + s];
            Vi[r * 3 + s] = acc;
        }
    return 0;
}

/* element (r, cc), cc <= r, of the packed lower profile */
#define SP(a, r, cc) ((a)[c->rp[(r)] + (size_t)((cc) - c->fc[(r)])])

/* Schur elimination of the points in [pb, pe) into the packed lower profile Sa and rhs
 * (accumulated): the observations' camera / intrinsics (F-block) terms plus, per point,
 * -W V~^-1 W^T (Ceres SchurEliminator semantics: E-block = point, F-blocks = poses +
 * intrinsics). W / Y / rowb are per-thread scratch of c->max_m observations. Per point
 * it also stores Vinv (9), e (3) and Kt (12) for the back-substitution when non-NULL. */
static int eliminate_points(const orc_t* c, const lin_t* L, const double* scale, const double* D2, int pb, int pe,
                            double* Sa, double* rhs, double* Vinv_all, double* e_all, double* Kt_all, double* W,
                            double* Y, int* rowb) {
    const ba_problem* p = c->p;
    const int kb = 6 * c->nac; /* intrinsics rows */
    const double* sk = scale + off_k(c);
    double Vt[9], Vi[9], Kt[12];
    int bad = 0;
    for (int pi = pb; pi < pe; ++pi) {
        if (!c->pt_active[pi]) continue;
        const double* sp = scale + off_pt(c, pi);
        memset(Vt, 0, sizeof(Vt));
        memset(Kt, 0, sizeof(Kt));
        double e[3] = {0, 0, 0};
        int nw = 0;
        for (int q = c->pt_ptr[pi]; q < c->pt_ptr[pi + 1]; ++q) {
            const int a = c->pt_obs[q];
            const int k = c->adm[a];
            const int ac = c->cam_ac[p->obs_cam[k]];
            const double* f = L->f + 3 * a;
            double Jp[9], Jc[18], Jk[8];
            for (int r = 0; r < 3; ++r)
                for (int i = 0; i < 3; ++i) Jp[r * 3 + i] = L->jp[9 * a + r * 3 + i] * sp[i];
            for (int r = 0; r < 2; ++r)
                for (int i = 0; i < 4; ++i) Jk[r * 4 + i] = L->jk[8 * a + r * 4 + i] * sk[i];
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j)
                    Vt[i * 3 + j] += Jp[i] * Jp[j] + Jp[3 + i] * Jp[3 + j] + Jp[6 + i] * Jp[6 + j];
            for (int i = 0; i < 3; ++i) e[i] += Jp[i] * f[0] + Jp[3 + i] * f[1] + Jp[6 + i] * f[2];
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 3; ++j) Kt[i * 3 + j] += Jk[i] * Jp[j] + Jk[4 + i] * Jp[3 + j];
            /* camera-side (F-block) terms of this observation */
            for (int i = 0; i < 4; ++i) {
                for (int j = 0; j <= i; ++j) SP(Sa, kb + i, kb + j) += Jk[i] * Jk[j] + Jk[4 + i] * Jk[4 + j];
                rhs[kb + i] += Jk[i] * f[0] + Jk[4 + i] * f[1];
            }
            if (ac < 0) continue;
            const double* sc = scale + 6 * ac;
            for (int r = 0; r < 3; ++r)
                for (int d = 0; d < 6; ++d) Jc[r * 6 + d] = L->jc[18 * a + r * 6 + d] * sc[d];
            const int cb = 6 * ac;
            for (int i = 0; i < 6; ++i) {
                for (int j = 0; j <= i; ++j)
                    SP(Sa, cb + i, cb + j) += Jc[i] * Jc[j] + Jc[6 + i] * Jc[6 + j] + Jc[12 + i] * Jc[12 + j];
                for (int j = 0; j < 4; ++j) SP(Sa, kb + j, cb + i) += Jc[i] * Jk[j] + Jc[6 + i] * Jk[4 + j];
                rhs[cb + i] += Jc[i] * f[0] + Jc[6 + i] * f[1] + Jc[12 + i] * f[2];
            }
            /* W = Jc^T Jp (6x3) of this observation */
            for (int d = 0; d < 6; ++d)
                for (int i = 0; i < 3; ++i)
                    W[18 * nw + d * 3 + i] = Jc[d] * Jp[i] + Jc[6 + d] * Jp[3 + i] + Jc[12 + d] * Jp[6 + i];
            rowb[nw++] = cb;
        }
        /* LM damping of the E block */
        for (int i = 0; i < 3; ++i) Vt[i * 4] += D2[off_pt(c, pi) + i];
        if (inv3_spd(Vt, Vi)) { bad = 1; continue; }
        if (Vinv_all) memcpy(Vinv_all + 9 * pi, Vi, sizeof(Vi));
        if (e_all) memcpy(e_all + 3 * pi, e, sizeof(e));
        if (Kt_all) memcpy(Kt_all + 12 * pi, Kt, sizeof(Kt));
        /* Y = W Vi */
        for (int w = 0; w < nw; ++w)
            for (int d = 0; d < 6; ++d)
                for (int i = 0; i < 3; ++i)
                    Y[18 * w + d * 3 + i] = W[18 * w + d * 3 + 0] * Vi[0 * 3 + i] +
                                            W[18 * w + d * 3 + 1] * Vi[1 * 3 + i] +
                                            W[18 * w + d * 3 + 2] * Vi[2 * 3 + i];
        double YK[12]; /* Kt Vi */
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 3; ++j)
                YK[i * 3 + j] = Kt[i * 3 + 0] * Vi[j] + Kt[i * 3 + 1] * Vi[3 + j] + Kt[i * 3 + 2] * Vi[6 + j];
        for (int a = 0; a < nw; ++a) {
            /* lower part only: blocks (a, b) with rowb[b] < rowb[a], and the lower half of equal rows */
            for (int b = 0; b < nw; ++b) {
                if (rowb[b] > rowb[a]) continue;
                for (int d = 0; d < 6; ++d)
                    for (int d2 = 0; d2 < 6; ++d2) {
                        if (rowb[b] == rowb[a] && d2 > d) continue;
                        SP(Sa, rowb[a] + d, rowb[b] + d2) -= Y[18 * a + d * 3 + 0] * W[18 * b + d2 * 3 + 0] +
                                                             Y[18 * a + d * 3 + 1] * W[18 * b + d2 * 3 + 1] +
                                                             Y[18 * a + d * 3 + 2] * W[18 * b + d2 * 3 + 2];
                    }
            }
            for (int d = 0; d < 6; ++d) {
                for (int j = 0; j < 4; ++j)
                    SP(Sa, kb + j, rowb[a] + d) -= Y[18 * a + d * 3 + 0] * Kt[j * 3 + 0] +
                                                   Y[18 * a + d * 3 + 1] * Kt[j * 3 + 1] +
                                                   Y[18 * a + d * 3 + 2] * Kt[j * 3 + 2];
                rhs[rowb[a] + d] -= Y[18 * a + d * 3 + 0] * e[0] + Y[18 * a + d * 3 + 1] * e[1] +
                                    Y[18 * a + d * 3 + 2] * e[2];
            }
        }
        for (int i = 0; i < 4; ++i) {
            for (int j = 0; j <= i; ++j)
                SP(Sa, kb + i, kb + j) -=
                    YK[i * 3 + 0] * Kt[j * 3 + 0] + YK[i * 3 + 1] * Kt[j * 3 + 1] + YK[i * 3 + 2] * Kt[j * 3 + 2];
            rhs[kb + i] -= YK[i * 3 + 0] * e[0] + YK[i * 3 + 1] * e[1] + YK[i * 3 + 2] * e[2];
        }
    }
    return bad ? -1 : 0;
}

/* Build (part of) the Jacobi-scaled, LM-damped reduced camera system over the points
 * in [pb, pe): Sa (packed lower profile, c->nnz) and rhs (n) are overwritten. Threads
 * take contiguous point ranges into private copies, summed in thread order. The prior
 * and the damping of cameras / intrinsics are added when with_global != 0. */
static int build_reduced(const orc_t* c, const lin_t* L, const double* scale, const double* D2, int pb, int pe,
                         int with_global, double* Sa, double* rhs, double* Vinv_all, double* e_all, double* Kt_all) {
    const int T = g_threads, n = c->n;
    const size_t m = (size_t)c->max_m + 1, slab = c->nnz + (size_t)n;
    double* priv = (double*)calloc((size_t)T * slab, sizeof(double));
    double* scr = (double*)malloc(sizeof(double) * 36 * m * T);
    int* rowb = (int*)malloc(sizeof(int) * m * T);
    int badv[T];
#pragma omp parallel num_threads(T)
    {
        const int t = tid();
        int lo, hi;
        chunk(pe - pb, t, T, &lo, &hi);
        double* Sp = priv + (size_t)t * slab;
        badv[t] = eliminate_points(c, L, scale, D2, pb + lo, pb + hi, Sp, Sp + c->nnz, Vinv_all, e_all, Kt_all,
                                   scr + 36 * m * t, scr + 36 * m * t + 18 * m, rowb + m * t);
    }
    memcpy(Sa, priv, sizeof(double) * c->nnz);
    memcpy(rhs, priv + c->nnz, sizeof(double) * n);
    int bad = badv[0];
    for (int t = 1; t < T; ++t) {
        const double* Sp = priv + (size_t)t * slab;
        for (size_t i = 0; i < c->nnz; ++i) Sa[i] += Sp[i];
        for (int i = 0; i < n; ++i) rhs[i] += Sp[c->nnz + i];
        bad |= badv[t];
    }
    free(priv); free(scr); free(rowb);
    if (with_global) {
        const int kb = 6 * c->nac;
        const double* sk = scale + off_k(c);
        /* IntrinsicsPrior block: J = -sqrt(w) I (scaled), residual fk */
        for (int i = 0; i < 4; ++i) {
            SP(Sa, kb + i, kb + i) += c->sw_k * c->sw_k * sk[i] * sk[i];
            rhs[kb + i] += -c->sw_k * sk[i] * L->fk[i];
        }
        for (int ac = 0; ac < c->nac; ++ac)
            for (int d = 0; d < 6; ++d) SP(Sa, 6 * ac + d, 6 * ac + d) += D2[6 * ac + d];
        for (int i = 0; i < 4; ++i) SP(Sa, kb + i, kb + i) += D2[off_k(c) + i];
    }
    return bad ? -1 : 0;
}

/* Row-oriented profile (skyline) Cholesky S = L L^T in place, then L L^T x = b.
 * Fill stays inside the profile; with fc == 0 it is the dense Cholesky.
 * Returns -1 if S is not positive definite. */
static int chol_solve(const orc_t* c, double* a, double* b) {
    const int n = c->n;
    for (int i = 0; i < n; ++i) {
        const int fi = c->fc[i];
        double* ri = a + c->rp[i] - fi; /* ri[j] = L(i, j), j in [fi, i] */
        for (int j = fi; j <= i; ++j) {
            const int fj = c->fc[j];
            const double* rj = a + c->rp[j] - fj;
            double s = ri[j];
            for (int k = fi > fj ? fi : fj; k < j; ++k) s -= ri[k] * rj[k];
            if (j < i) {
                ri[j] = s / rj[j];
            } else {
                if (!(s > 0) || !isfinite(s)) return -1;
                ri[i] = sqrt(s);
            }
        }
    }
    for (int i = 0; i < n; ++i) { /* L z = b */
        const int fi = c->fc[i];
        const double* ri = a + c->rp[i] - fi;
        double s = b[i];
        for (int k = fi; k < i; ++k) s -= ri[k] * b[k];
        b[i] = s / ri[i];
    }
    for (int i = n - 1; i >= 0; --i) { /* L^T x = z */
        const int fi = c->fc[i];
        const double* ri = a + c->rp[i] - fi;
        b[i] /= ri[i];
        for (int k = fi; k < i; ++k) b[k] -= ri[k] * b[i];
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* Solver state                                                         */
typedef struct {
    double *cams, *pts, K[4];
} xstate_t;

static double x_norm2(const orc_t* c, const xstate_t* x) {
    double s = 0;
    for (int i = 0; i < c->p->n_cams; ++i)
        if (c->cam_ac[i] >= 0)
            for (int j = 0; j < 7; ++j) s += x->cams[7 * i + j] * x->cams[7 * i + j];
    for (int i = 0; i < c->p->n_points; ++i)
        if (c->pt_active[i])
            for (int j = 0; j < 3; ++j) s += x->pts[3 * i + j] * x->pts[3 * i + j];
    for (int j = 0; j < 4; ++j) s += x->K[j] * x->K[j];
    return s;
}

/* x_plus = Plus(x, delta) over active blocks (delta in local coords) */
static void plus(const orc_t* c, const xstate_t* x, const double* delta, xstate_t* xp) {
    memcpy(xp->cams, x->cams, sizeof(double) * 7 * c->p->n_cams);
    memcpy(xp->pts, x->pts, sizeof(double) * 3 * c->p->n_points);
    for (int i = 0; i < c->p->n_cams; ++i)
        if (c->cam_ac[i] >= 0) se3_plus(x->cams + 7 * i, delta + 6 * c->cam_ac[i], xp->cams + 7 * i);
    for (int i = 0; i < c->p->n_points; ++i)
        if (c->pt_active[i])
            for (int j = 0; j < 3; ++j) xp->pts[3 * i + j] = x->pts[3 * i + j] + delta[off_pt(c, i) + j];
    for (int j = 0; j < 4; ++j) xp->K[j] = x->K[j] + delta[off_k(c) + j];
}

/* ||x - Plus(x, -g)||_inf  (Ceres 2.0 gradient_max_norm, trust_region_minimizer.cc) */
static double grad_max_norm(const orc_t* c, const xstate_t* x, const double* g) {
    double m = 0;
    double ng[6], tp[7];
    for (int i = 0; i < c->p->n_cams; ++i) {
        const int ac = c->cam_ac[i];
        if (ac < 0) continue;
        for (int d = 0; d < 6; ++d) ng[d] = -g[6 * ac + d];
        se3_plus(x->cams + 7 * i, ng, tp);
        for (int j = 0; j < 7; ++j) m = fmax(m, fabs(x->cams[7 * i + j] - tp[j]));
    }
    for (int i = 0; i < c->p->n_points; ++i)
        if (c->pt_active[i])
            for (int j = 0; j < 3; ++j) {
                const double v = x->pts[3 * i + j];
                m = fmax(m, fabs(v - (v + -g[off_pt(c, i) + j])));
            }
    for (int j = 0; j < 4; ++j) m = fmax(m, fabs(x->K[j] - (x->K[j] + -g[off_k(c) + j])));
    return m;
}

/* Linear solve for one LM step (LevenbergMarquardtStrategy::ComputeStep + SchurComplementSolver).
 * Produces step (scaled local coords, = -y). Returns 0 ok, -1 linear solver failure. */
static int compute_step(const orc_t* c, const lin_t* L, const double* scale, const double* diag, double radius,
                        double* step) {
    const int n = c->n;
    const int nl = nloc(c);
    const ba_problem* p = c->p;
    double* D2 = (double*)malloc(sizeof(double) * nl);
    for (int i = 0; i < nl; ++i) D2[i] = diag[i] / radius; /* lm_diagonal = sqrt(diag / radius) */
    double* Sa = (double*)malloc(sizeof(double) * (c->nnz + 1));
    double* rhs = (double*)malloc(sizeof(double) * n);
    double* Vinv = (double*)malloc(sizeof(double) * 9 * (p->n_points + 1));
    double* e = (double*)malloc(sizeof(double) * 3 * (p->n_points + 1));
    double* Kt = (double*)malloc(sizeof(double) * 12 * (p->n_points + 1));
    int st = build_reduced(c, L, scale, D2, 0, p->n_points, 1, Sa, rhs, Vinv, e, Kt);
    if (!st) st = chol_solve(c, Sa, rhs);
    if (!st) {
        /* F-part of y */
        memset(step, 0, sizeof(double) * nl);
        for (int ac = 0; ac < c->nac; ++ac)
            for (int d = 0; d < 6; ++d) step[6 * ac + d] = rhs[6 * ac + d];
        for (int i = 0; i < 4; ++i) step[off_k(c) + i] = rhs[6 * c->nac + i];
        /* back-substitute points: y_p = Vinv (e - W^T y_c - Kt^T y_k) */
#pragma omp parallel for num_threads(g_threads) schedule(static)
        for (int pi = 0; pi < p->n_points; ++pi) {
            if (!c->pt_active[pi]) continue;
            const double* sp = scale + off_pt(c, pi);
            double t[3] = {e[3 * pi], e[3 * pi + 1], e[3 * pi + 2]};
            for (int q = c->pt_ptr[pi]; q < c->pt_ptr[pi + 1]; ++q) {
                const int a = c->pt_obs[q];
                const int ac = c->cam_ac[p->obs_cam[c->adm[a]]];
                if (ac < 0) continue;
                const double* sc = scale + 6 * ac;
                double Jc[18], Jp[9];
                for (int r = 0; r < 3; ++r) {
                    for (int d = 0; d < 6; ++d) Jc[r * 6 + d] = L->jc[18 * a + r * 6 + d] * sc[d];
                    for (int i = 0; i < 3; ++i) Jp[r * 3 + i] = L->jp[9 * a + r * 3 + i] * sp[i];
                }
                /* Jc y_c (3) then Jp^T (.) */
                double jy[3];
                for (int r = 0; r < 3; ++r) {
                    double s = 0;
                    for (int d = 0; d < 6; ++d) s += Jc[r * 6 + d] * rhs[6 * ac + d];
                    jy[r] = s;
                }
                for (int i = 0; i < 3; ++i) t[i] -= Jp[i] * jy[0] + Jp[3 + i] * jy[1] + Jp[6 + i] * jy[2];
            }
            for (int i = 0; i < 3; ++i)
                t[i] -= Kt[12 * pi + 0 * 3 + i] * rhs[6 * c->nac + 0] + Kt[12 * pi + 1 * 3 + i] * rhs[6 * c->nac + 1] +
                        Kt[12 * pi + 2 * 3 + i] * rhs[6 * c->nac + 2] + Kt[12 * pi + 3 * 3 + i] * rhs[6 * c->nac + 3];
            for (int i = 0; i < 3; ++i)
                step[off_pt(c, pi) + i] =
                    Vinv[9 * pi + i * 3 + 0] * t[0] + Vinv[9 * pi + i * 3 + 1] * t[1] + Vinv[9 * pi + i * 3 + 2] * t[2];
        }
        for (int i = 0; i < nl; ++i) {
            if (!isfinite(step[i])) { st = -1; break; }
            step[i] = -step[i];
        }
    }
    free(D2); free(Sa); free(rhs); free(Vinv); free(e); free(Kt);
    return st;
}

/* model_cost_change = -(J delta)^T (f + J delta / 2)  (ComputeTrustRegionStep);
 * per-thread partials over contiguous observation ranges, summed in thread order */
static double model_cost_change(const orc_t* c, const lin_t* L, const double* delta) {
    const ba_problem* p = c->p;
    const int T = g_threads;
    double part[T];
#pragma omp parallel num_threads(T)
    {
        const int t = tid();
        int lo, hi;
        chunk(c->n_adm, t, T, &lo, &hi);
        double m = 0;
        for (int a = lo; a < hi; ++a) {
            const int k = c->adm[a];
            const int ac = c->cam_ac[p->obs_cam[k]];
            const double* dp = delta + off_pt(c, p->obs_pt[k]);
            const double* dk = delta + off_k(c);
            for (int r = 0; r < 3; ++r) {
                double jd = 0;
                if (ac >= 0)
                    for (int d = 0; d < 6; ++d) jd += L->jc[18 * a + r * 6 + d] * delta[6 * ac + d];
                for (int i = 0; i < 3; ++i) jd += L->jp[9 * a + r * 3 + i] * dp[i];
                if (r < 2)
                    for (int i = 0; i < 4; ++i) jd += L->jk[8 * a + r * 4 + i] * dk[i];
                m += -jd * (L->f[3 * a + r] + jd / 2.0);
            }
        }
        part[t] = m;
    }
    double m = 0;
    for (int t = 0; t < T; ++t) m += part[t];
    for (int i = 0; i < 4; ++i) {
        const double jd = -c->sw_k * delta[off_k(c) + i];
        m += -jd * (L->fk[i] + jd / 2.0);
    }
    return m;
}

static void print_header(void) {
    printf("iter      cost      cost_change  |gradient|   |step|    tr_ratio  tr_radius  ls_iter  iter_time  total_time\n");
}
static void print_row(int it, double cost, double dc, double g, double st, double rho, double rad, double t_it,
                      double t_tot) {
    printf("% 4d % 3.6e % 3.2e % 3.2e % 3.2e % 3.2e % 3.2e % 4d % 3.2e % 3.2e\n", it, cost, dc, g, st, rho, rad, 0,
           t_it, t_tot);
}

/* Per-iteration trace row (same layout as libmiba's device iteration log, ba_iteration_log):
 * cost, cost_change, |gradient|_inf, |step|, tr_ratio, tr_radius, accepted (1 / 0 / -1 = the
 * terminating tolerance step), 0 */
#define TRACE_W 8
typedef struct {
    double* rows;
    int max_rows;
} trace_t;
static void trace_row(trace_t* tr, int it, double cost, double dc, double g, double st, double rho, double rad,
                      double acc) {
    if (!tr || !tr->rows || it >= tr->max_rows) return;
    double* r = tr->rows + (size_t)it * TRACE_W;
    r[0] = cost; r[1] = dc; r[2] = g; r[3] = st; r[4] = rho; r[5] = rad; r[6] = acc; r[7] = 0;
}

/* The Ceres 2.0 TrustRegionMinimizer::Minimize loop with LM strategy. */
static int solve_impl(ba_problem* p, const ba_options* opt, ba_summary* sum, trace_t* tr) {
    const double t0 = now_ms();
    memset(sum, 0, sizeof(*sum));
    sum->struct_size = (int32_t)sizeof(*sum);
    orc_t c;
    if (orc_init(&c, p, opt)) { orc_free(&c); return BA_E_INVALID; }
    sum->num_obs_admissible = c.n_adm;
    sum->num_active_cams = c.nac;
    sum->num_active_points = c.n_act_pts;
    sum->reduced_system_size = c.n;
    const int nl = nloc(&c);
    lin_t L;
    if (lin_alloc(&L, c.n_adm)) { orc_free(&c); return BA_E_NOMEM; }
    xstate_t x, xc;
    x.cams = p->cams; /* updated in place, like the reference's parameter blocks */
    x.pts = p->points;
    memcpy(x.K, p->intr, sizeof(x.K));
    xc.cams = (double*)malloc(sizeof(double) * 7 * (p->n_cams + 1));
    xc.pts = (double*)malloc(sizeof(double) * 3 * (p->n_points + 1));
    double* scale = (double*)malloc(sizeof(double) * nl);
    double* cn = (double*)malloc(sizeof(double) * nl);
    double* diag = (double*)malloc(sizeof(double) * nl);
    double* g = (double*)malloc(sizeof(double) * nl);
    double* step = (double*)malloc(sizeof(double) * nl);
    double* delta = (double*)malloc(sizeof(double) * nl);
    const int progress = opt->minimizer_progress_to_stdout;
    const double tl0 = now_ms();

    double x_cost, cand_cost;
    int ret = 0;
    /* IterationZero: EvaluateGradientAndJacobian */
    if (evaluate(&c, x.cams, x.pts, x.K, &L, &x_cost)) {
        sum->termination_type = BA_FAILURE;
        snprintf(sum->message, sizeof(sum->message), "Residual and Jacobian evaluation failed.");
        sum->initial_cost = NAN; sum->final_cost = NAN;
        goto done;
    }
    colnorm_grad(&c, &L, cn, g);
    for (int i = 0; i < nl; ++i) scale[i] = opt->jacobi_scaling ? 1.0 / (1.0 + sqrt(cn[i])) : 1.0;
    double gmax = grad_max_norm(&c, &x, g);
    sum->initial_cost = x_cost;
    double final_cost = x_cost; /* SetSummaryFinalCost: min over iteration costs */
    double radius = opt->initial_trust_region_radius;
    double decrease_factor = 2.0;
    int reuse_diag = 0;
    double xnorm = sqrt(x_norm2(&c, &x));
    int iter = 0, n_succ = 1, n_unsucc = 0, n_invalid = 0;
    int step_ok = 1; /* iteration 0 counts as successful */
    if (progress) { print_header(); print_row(0, x_cost, 0, gmax, 0, 0, radius, 0, 0); }
    trace_row(tr, 0, x_cost, 0, gmax, 0, 0, radius, 1);
    for (;;) {
        /* FinalizeIterationAndCheckIfMinimizerCanContinue */
        if (iter >= opt->max_num_iterations) {
            sum->termination_type = BA_NO_CONVERGENCE;
            snprintf(sum->message, sizeof(sum->message), "Maximum number of iterations reached. Number of iterations: %d.", iter);
            break;
        }
        if (step_ok && gmax <= opt->gradient_tolerance) {
            sum->termination_type = BA_CONVERGENCE;
            snprintf(sum->message, sizeof(sum->message), "Gradient tolerance reached. Gradient max norm: %e <= %e", gmax, opt->gradient_tolerance);
            break;
        }
        if (radius <= opt->min_trust_region_radius) {
            sum->termination_type = BA_CONVERGENCE;
            snprintf(sum->message, sizeof(sum->message), "Minimum trust region radius reached. Trust region radius: %e <= %e", radius, opt->min_trust_region_radius);
            break;
        }
        ++iter;
        /* ComputeTrustRegionStep */
        if (!reuse_diag)
            for (int i = 0; i < nl; ++i) {
                const double v = cn[i] * scale[i] * scale[i]; /* column norm of scaled J */
                diag[i] = fmin(fmax(v, opt->min_lm_diagonal), opt->max_lm_diagonal);
            }
        const int lsf = compute_step(&c, &L, scale, diag, radius, step);
        reuse_diag = 1;
        double mcc = 0;
        int valid = 0;
        if (!lsf) {
            for (int i = 0; i < nl; ++i) delta[i] = step[i] * scale[i];
            mcc = model_cost_change(&c, &L, delta);
            valid = mcc > 0.0;
        }
        if (!valid) {
            /* HandleInvalidStep */
            if (++n_invalid >= opt->max_num_consecutive_invalid_steps) {
                sum->termination_type = BA_FAILURE;
                snprintf(sum->message, sizeof(sum->message), "Number of consecutive invalid steps more than Solver::Options::max_num_consecutive_invalid_steps: %d", opt->max_num_consecutive_invalid_steps);
                ++n_unsucc;
                trace_row(tr, iter, x_cost, 0, gmax, 0, 0, radius, 0);
                break;
            }
            radius = radius / decrease_factor; /* LM StepIsInvalid == StepRejected */
            decrease_factor *= 2.0;
            reuse_diag = 1;
            step_ok = 0;
            ++n_unsucc;
            if (progress) print_row(iter, x_cost, 0, gmax, 0, 0, radius, 0, now_ms() - tl0);
            trace_row(tr, iter, x_cost, 0, gmax, 0, 0, radius, 0);
            continue;
        }
        n_invalid = 0;
        /* ComputeCandidatePointAndEvaluateCost */
        plus(&c, &x, delta, &xc);
        for (int j = 0; j < 4; ++j) xc.K[j] = x.K[j] + delta[off_k(&c) + j];
        if (evaluate(&c, xc.cams, xc.pts, xc.K, NULL, &cand_cost)) cand_cost = DBL_MAX;
        /* ParameterToleranceReached: |x - x_cand| in the ambient space */
        double sn2 = 0;
        for (int i = 0; i < p->n_cams; ++i)
            if (c.cam_ac[i] >= 0)
                for (int j = 0; j < 7; ++j) { const double d = x.cams[7 * i + j] - xc.cams[7 * i + j]; sn2 += d * d; }
        for (int i = 0; i < p->n_points; ++i)
            if (c.pt_active[i])
                for (int j = 0; j < 3; ++j) { const double d = x.pts[3 * i + j] - xc.pts[3 * i + j]; sn2 += d * d; }
        for (int j = 0; j < 4; ++j) { const double d = x.K[j] - xc.K[j]; sn2 += d * d; }
        const double step_norm = sqrt(sn2);
        const double cost_change = x_cost - cand_cost;
        if (step_norm <= opt->parameter_tolerance * (xnorm + opt->parameter_tolerance)) {
            sum->termination_type = BA_CONVERGENCE;
            snprintf(sum->message, sizeof(sum->message), "Parameter tolerance reached. Relative step_norm: %e <= %e.", step_norm / (xnorm + opt->parameter_tolerance), opt->parameter_tolerance);
            /* the iteration is not finalized (returns before FinalizeIteration) */
            trace_row(tr, iter, cand_cost, cost_change, gmax, step_norm, 0, radius, -1);
            break;
        }
        /* FunctionToleranceReached */
        if (fabs(cost_change) <= opt->function_tolerance * x_cost) {
            sum->termination_type = BA_CONVERGENCE;
            snprintf(sum->message, sizeof(sum->message), "Function tolerance reached. |cost_change|/cost: %e <= %e", fabs(cost_change) / x_cost, opt->function_tolerance);
            trace_row(tr, iter, cand_cost, cost_change, gmax, step_norm, 0, radius, -1);
            break;
        }
        /* IsStepSuccessful (monotonic: relative decrease vs model) */
        const double rho = (cand_cost >= DBL_MAX) ? -DBL_MAX : (x_cost - cand_cost) / mcc;
        if (rho > opt->min_relative_decrease) {
            /* HandleSuccessfulStep */
            memcpy(x.cams, xc.cams, sizeof(double) * 7 * p->n_cams);
            memcpy(x.pts, xc.pts, sizeof(double) * 3 * p->n_points);
            memcpy(x.K, xc.K, sizeof(x.K));
            xnorm = sqrt(x_norm2(&c, &x));
            double ncost;
            if (evaluate(&c, x.cams, x.pts, x.K, &L, &ncost)) {
                sum->termination_type = BA_FAILURE;
                snprintf(sum->message, sizeof(sum->message), "Residual and Jacobian evaluation failed.");
                break;
            }
            x_cost = ncost;
            colnorm_grad(&c, &L, cn, g);
            gmax = grad_max_norm(&c, &x, g);
            /* LevenbergMarquardtStrategy::StepAccepted */
            radius = radius / fmax(1.0 / 3.0, 1.0 - pow(2.0 * rho - 1.0, 3));
            radius = fmin(opt->max_trust_region_radius, radius);
            decrease_factor = 2.0;
            reuse_diag = 0;
            step_ok = 1;
            ++n_succ;
            final_cost = fmin(final_cost, x_cost);
            if (progress) print_row(iter, x_cost, cost_change, gmax, step_norm, rho, radius, 0, now_ms() - tl0);
            trace_row(tr, iter, x_cost, cost_change, gmax, step_norm, rho, radius, 1);
        } else {
            /* HandleUnsuccessfulStep: iteration cost reported = candidate cost */
            radius = radius / decrease_factor;
            decrease_factor *= 2.0;
            reuse_diag = 1;
            step_ok = 0;
            ++n_unsucc;
            final_cost = fmin(final_cost, cand_cost);
            if (progress) print_row(iter, cand_cost, cost_change, gmax, step_norm, rho, radius, 0, now_ms() - tl0);
            trace_row(tr, iter, cand_cost, cost_change, gmax, step_norm, rho, radius, 0);
        }
    }
    sum->final_cost = final_cost;
    sum->num_successful_steps = n_succ;
    sum->num_unsuccessful_steps = n_unsucc;
    sum->num_iterations = iter;
    memcpy(p->intr, x.K, sizeof(x.K));
done:
    sum->time_lm_ms = now_ms() - tl0;
    sum->time_total_ms = now_ms() - t0;
    sum->time_setup_ms = tl0 - t0;
    free(xc.cams); free(xc.pts); free(scale); free(cn); free(diag); free(g); free(step); free(delta);
    lin_free(&L);
    orc_free(&c);
    return ret;
}

EXPORT int oracle_solve(ba_problem* p, const ba_options* opt, ba_summary* sum) {
    return solve_impl(p, opt, sum, NULL);
}

/* oracle_solve plus the per-iteration trace (TRACE_W doubles per row, rows 0..num_iterations) */
EXPORT int oracle_solve_trace(ba_problem* p, const ba_options* opt, ba_summary* sum, double* rows,
                              int32_t max_rows) {
    trace_t tr = {rows, max_rows};
    if (rows && max_rows > 0) memset(rows, 0, sizeof(double) * TRACE_W * (size_t)max_rows);
    return solve_impl(p, opt, sum, &tr);
}

/* Per-observation residuals/Jacobians in the ORIGINAL obs order (same layout
 * as ba_debug_linearize). */
EXPORT int oracle_linearize(const ba_problem* p, const ba_options* opt, double* cost, double* res, double* jcam,
                            double* jpt, double* jint) {
    orc_t c;
    if (orc_init(&c, p, opt)) { orc_free(&c); return BA_E_INVALID; }
    lin_t L;
    if (lin_alloc(&L, c.n_adm)) { orc_free(&c); return BA_E_NOMEM; }
    double cst;
    const int st = evaluate(&c, p->cams, p->points, p->intr, &L, &cst);
    if (cost) *cost = st ? NAN : cst;
    if (res) memset(res, 0, sizeof(double) * 3 * p->n_obs);
    if (jcam) memset(jcam, 0, sizeof(double) * 18 * p->n_obs);
    if (jpt) memset(jpt, 0, sizeof(double) * 9 * p->n_obs);
    if (jint) memset(jint, 0, sizeof(double) * 8 * p->n_obs);
    for (int a = 0; a < c.n_adm; ++a) {
        const int k = c.adm[a];
        if (res) memcpy(res + 3 * k, L.f + 3 * a, sizeof(double) * 3);
        if (jcam) memcpy(jcam + 18 * k, L.jc + 18 * a, sizeof(double) * 18);
        if (jpt) memcpy(jpt + 9 * k, L.jp + 9 * a, sizeof(double) * 9);
        if (jint) memcpy(jint + 8 * k, L.jk + 8 * a, sizeof(double) * 8);
    }
    lin_free(&L);
    orc_free(&c);
    return st ? BA_E_INVALID : 0;
}

/* Reduced camera system of the first LM iteration (same contract as
 * ba_debug_reduced_system), restricted to the Schur/observation terms of points
 * in [pt_begin, pt_end); with_global adds the prior and camera/intrinsics damping.
 * Summing shards over a point partition reproduces the full system: this is the
 * landmark-sharded multi-device decomposition. */
EXPORT int oracle_reduced_system(const ba_problem* p, const ba_options* opt, double radius, int32_t pt_begin,
                                 int32_t pt_end, int32_t with_global, int32_t* n_out, double* S, double* rhs) {
    orc_t c;
    if (orc_init(&c, p, opt)) { orc_free(&c); return BA_E_INVALID; }
    if (n_out) *n_out = c.n;
    if (!S || !rhs) { orc_free(&c); return 0; }
    lin_t L;
    if (lin_alloc(&L, c.n_adm)) { orc_free(&c); return BA_E_NOMEM; }
    double cst;
    int st = evaluate(&c, p->cams, p->points, p->intr, &L, &cst);
    const int nl = nloc(&c);
    double* cn = (double*)malloc(sizeof(double) * nl);
    double* scale = (double*)malloc(sizeof(double) * nl);
    double* D2 = (double*)malloc(sizeof(double) * nl);
    double* Sa = (double*)malloc(sizeof(double) * (c.nnz + 1));
    colnorm_grad(&c, &L, cn, NULL);
    if (radius <= 0) radius = opt->initial_trust_region_radius;
    for (int i = 0; i < nl; ++i) {
        scale[i] = opt->jacobi_scaling ? 1.0 / (1.0 + sqrt(cn[i])) : 1.0;
        const double v = cn[i] * scale[i] * scale[i];
        D2[i] = fmin(fmax(v, opt->min_lm_diagonal), opt->max_lm_diagonal) / radius;
    }
    memset(S, 0, sizeof(double) * (size_t)c.n * c.n);
    if (!st) st = build_reduced(&c, &L, scale, D2, pt_begin, pt_end, with_global, Sa, rhs, NULL, NULL, NULL);
    if (!st) {
        const orc_t* cc = &c;
        for (int r = 0; r < cc->n; ++r)
            for (int j = cc->fc[r]; j <= r; ++j) {
                const double v = Sa[cc->rp[r] + (size_t)(j - cc->fc[r])];
                S[(size_t)r * cc->n + j] = v;
                S[(size_t)j * cc->n + r] = v;
            }
    }
    free(cn); free(scale); free(D2); free(Sa);
    lin_free(&L);
    orc_free(&c);
    return st ? BA_E_INVALID : 0;
}

/* exposed for unit tests of the manifold restatement */
EXPORT void oracle_se3_plus(const double* T, const double* delta, double* out) { se3_plus(T, delta, out); }
