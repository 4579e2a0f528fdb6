/*
 * ba_io.h — window-problem files for libmiba. Host-only; no GPU needed.
 *
 * 1. Window dump / replay (.miba). A binary SoA image of exactly the ba_problem that
 *    windowOptimize hands to the solver (reference src/OptimizationUtils.cpp:236-299, the
 *    input of ceres::Solve at :300), optionally followed by the ba_options it was solved with.
 *    Windows captured on a machine that runs the reference's full front-end (TUM sequence,
 *    SURF/ORB, tracking) can be replayed bit-for-bit on a GPU box that has none of it.
 *    Capture needs no code change: with MIBA_DUMP_DIR set in the environment, every
 *    ba_solve() / ba_prepare() first writes its window to $MIBA_DUMP_DIR/window_<pid>_<n>.miba.
 *
 *    Layout (little endian, every array 8-byte aligned):
 *      off   0  char     magic[8] = "MIBAWIN1"
 *            8  uint32   version = 1
 *           12  uint32   options_bytes   (0, or sizeof(ba_options) when options follow)
 *           16  int32    n_cams, n_points, n_obs, fixed_cam
 *           32  double   intr[4], intr_prior[4]
 *           96  uint64   checksum        (FNV-1a 64 over every byte after the header)
 *          104  uint64   reserved = 0
 *          112  double   cams[n_cams*7]  (Sophus order qx,qy,qz,qw,tx,ty,tz)
 *               double   points[n_points*3]
 *               double   obs_uv[n_obs*2]
 *               double   obs_depth[n_obs]
 *               int32    obs_cam[n_obs], obs_pt[n_obs]
 *               (pad to 8 bytes)
 *               ba_options (options_bytes bytes), if options_bytes > 0
 *
 * 2. BAL ("Bundle Adjustment in the Large", Agarwal et al. 2010) text problems, the usual
 *    on-disk format for C5-scale windows. Not part of the reference; the conversion to the
 *    reference's cost (one shared pinhole intrinsics block, depth prior per observation):
 *      - BAL camera: P = R(w) X + t, p = -P/P.z, pixel = f (1 + k1|p|^2 + k2|p|^4) p,
 *        image origin at the centre, y up. Our camera looks down +z with v down, so
 *        R_cw = diag(1,-1,-1) R, t_cw = diag(1,-1,-1) t, and T_w_c is their inverse.
 *      - Each observation is undistorted with its camera's (f, k1, k2) and re-expressed at
 *        the shared focal f_s = median of the cameras' f:  uv = f_s * (p_x, -p_y).
 *        intr = intr_prior = (f_s, f_s, 0, 0).
 *      - BAL has no depth: obs_depth = z of the point in the initial camera (0 — i.e. the
 *        observation is skipped like the reference's missing depth — when not in front).
 *        Set ba_options.weight_unpr = 0 to drop the depth prior for pure BAL problems.
 *      - fixed_cam = 0.
 *    ba_bal_write is the inverse (f = fx, k1 = k2 = 0, %.17g), so a window written to BAL
 *    and read back has the same reprojection residuals when fx == fy.
 *
 * Every function returns BA_OK (0) or BA_E_INVALID / BA_E_NOMEM; ba_last_error(NULL) explains.
 * Readers fill caller-owned buffers sized from the *_dims call (intr_prior is written through
 * the const pointer of ba_problem: it must point to writable memory).
 */
#ifndef MIBA_BA_IO_H
#define MIBA_BA_IO_H
#include "ba.h"
#ifdef __cplusplus
extern "C" {
#endif

#define BA_DUMP_VERSION 1

int32_t ba_problem_write(const char* path, const ba_problem* prob, const ba_options* opts /* may be NULL */);
int32_t ba_problem_read_dims(const char* path, int32_t* n_cams, int32_t* n_points, int32_t* n_obs);
/* opts_out may be NULL; if the file carries no options it receives ba_default_options(). */
int32_t ba_problem_read(const char* path, ba_problem* prob, ba_options* opts_out);

int32_t ba_bal_read_dims(const char* path, int32_t* n_cams, int32_t* n_points, int32_t* n_obs);
int32_t ba_bal_read(const char* path, ba_problem* prob);
int32_t ba_bal_write(const char* path, const ba_problem* prob);

#ifdef __cplusplus
}
#endif
#endif /* MIBA_BA_IO_H */
