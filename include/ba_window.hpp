// ba_window.hpp — header-only host adapter: the reference's windowOptimize()
// (/root/reference/src/OptimizationUtils.cpp:215-313) on top of the ba_solve() C-ABI.
//
// It reproduces, step for step, everything windowOptimize does around ceres::Solve:
//   :231-232  initialPose = T_w_c[kf_i], initialPoseInv = initialPose^-1
//   :248      every window pose is re-anchored: T <- initialPoseInv * T
//   :257-268  observations iterate global_points_map; depth <= 1e-15 is skipped BEFORE the
//             landmark is touched (an only-inadmissible landmark is neither moved nor optimised)
//   :271-276  first admissible sighting of a landmark moves it into the kf_i frame
//   :279-294  one reprojection + one depth residual per admissible observation
//   :299      kf_i is the gauge (constant)
//   :300      ceres::Solve  ->  solve(&problem, &summary)   (ba_solve / oracle)
//   :303-310  poses and the touched landmarks are mapped back with initialPose
// and intrinsics_optimized is updated in place (it persists across windows, main.cpp:114).
//
// Duck-typed on the reference's own types (no Sophus/Eigen/OpenCV include here):
//   keyframes[k].T_w_c.data()                 -> double*  [qx,qy,qz,qw,tx,ty,tz] (Sophus::SE3d)
//   keyframes[k].global_points_map            -> iterable of (localId, landmarkId)
//   keyframes[k].points3d_local[localId][2]   -> depth (Eigen::Vector3d)
//   keyframes[k].keypoints[localId].pt.x / .y -> float pixel (cv::KeyPoint)
//   map.at(landmarkId).point.data()           -> double* [3] (Eigen::Vector3d)
//   intrinsics[i], i < 4                      -> double (Eigen::Vector4d)
#ifndef MIBA_BA_WINDOW_HPP
#define MIBA_BA_WINDOW_HPP

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "ba.h"

namespace miba {

// ---- SE(3) on Sophus storage [qx,qy,qz,qw,tx,ty,tz] (se3.hpp / so3.hpp semantics)
inline void so3_rotate(const double* q, const double* v, double* out) {
    // Eigen _transformVector: v + w*uv + q.vec x uv, uv = 2 q.vec x v
    const double qx = q[0], qy = q[1], qz = q[2], qw = q[3];
    const double uv0 = 2 * (qy * v[2] - qz * v[1]);
    const double uv1 = 2 * (qz * v[0] - qx * v[2]);
    const double uv2 = 2 * (qx * v[1] - qy * v[0]);
    out[0] = v[0] + qw * uv0 + (qy * uv2 - qz * uv1);
    out[1] = v[1] + qw * uv1 + (qz * uv0 - qx * uv2);
    out[2] = v[2] + qw * uv2 + (qx * uv1 - qy * uv0);
}

// out = a * b  (SE3 operator*= with the SO3 renormalisation of so3.hpp:339-356)
inline void se3_mul(const double* a, const double* b, double* out) {
    double t[3];
    so3_rotate(a, b + 4, t);
    const double ax = a[0], ay = a[1], az = a[2], aw = a[3];
    const double bx = b[0], by = b[1], bz = b[2], bw = b[3];
    double w = aw * bw - ax * bx - ay * by - az * bz;
    double x = aw * bx + ax * bw + ay * bz - az * by;
    double y = aw * by + ay * bw + az * bx - ax * bz;
    double z = aw * bz + az * bw + ax * by - ay * bx;
    const double sq = x * x + y * y + z * z + w * w;
    if (sq != 1.0) {
        const double f = 2.0 / (1.0 + sq);
        x *= f; y *= f; z *= f; w *= f;
    }
    out[0] = x; out[1] = y; out[2] = z; out[3] = w;
    out[4] = a[4] + t[0]; out[5] = a[5] + t[1]; out[6] = a[6] + t[2];
}

// out = a^-1  (SE3::inverse: R^-1 = conjugate, t' = -(R^-1 t))
inline void se3_inv(const double* a, double* out) {
    const double qi[4] = {-a[0], -a[1], -a[2], a[3]};
    const double mt[3] = {-a[4], -a[5], -a[6]};
    double t[3];
    so3_rotate(qi, mt, t);
    out[0] = qi[0]; out[1] = qi[1]; out[2] = qi[2]; out[3] = qi[3];
    out[4] = t[0]; out[5] = t[1]; out[6] = t[2];
}

// out = T * p
inline void se3_act(const double* T, const double* p, double* out) {
    double r[3];
    so3_rotate(T, p, r);
    out[0] = r[0] + T[4]; out[1] = r[1] + T[5]; out[2] = r[2] + T[6];
}

// Flattened window (owns the SoA buffers a ba_problem points into).
struct WindowProblem {
    std::vector<double> cams, points, uv, depth;
    std::vector<int32_t> obs_cam, obs_pt;
    double intr[4], prior[4];
    std::vector<int> landmark_ids;  // point index -> LandmarkId
    ba_problem view() {
        ba_problem p{};
        p.n_cams = (int32_t)(cams.size() / 7);
        p.n_points = (int32_t)(points.size() / 3);
        p.n_obs = (int32_t)obs_cam.size();
        p.fixed_cam = 0;  // kf_i, SetParameterBlockConstant (:299)
        p.cams = cams.data();
        p.points = points.data();
        p.intr = intr;
        p.intr_prior = prior;
        p.obs_cam = obs_cam.data();
        p.obs_pt = obs_pt.data();
        p.obs_uv = uv.data();
        p.obs_depth = depth.data();
        return p;
    }
};

// windowOptimize with an injectable solver: solve(ba_problem*, ba_summary*) -> int32_t
// (e.g. [&](ba_problem* p, ba_summary* s) { return ba_solve(ctx, p, s); }).
// Returns true like the reference (:312); the solver status is returned through *status.
template <class KeyFrames, class Map3D, class Vec4In, class Vec4Out, class SolveFn>
bool windowOptimize(int kf_i, int kf_f, KeyFrames& keyframes, Map3D& map, const Vec4In& intrinsics_initial,
                    Vec4Out& intrinsics_optimized, SolveFn&& solve, ba_summary* summary_out = nullptr,
                    int32_t* status = nullptr) {
    double initialPose[7], initialPoseInv[7];
    {
        const double* T0 = keyframes[kf_i].T_w_c.data();
        for (int j = 0; j < 7; ++j) initialPose[j] = T0[j];
        se3_inv(initialPose, initialPoseInv);
    }
    WindowProblem w;
    for (int i = 0; i < 4; ++i) {
        w.intr[i] = intrinsics_optimized[i];
        w.prior[i] = intrinsics_initial[i];
    }
    std::unordered_map<int, int> pt_index;  // LandmarkId -> point index (already_observed_pts, :229)
    const int n_kf = kf_f - kf_i + 1;
    w.cams.resize(7 * (size_t)n_kf);
    for (int kf_n = kf_i; kf_n <= kf_f; ++kf_n) {
        auto& kf = keyframes[kf_n];
        double* T = kf.T_w_c.data();
        double Tn[7];
        se3_mul(initialPoseInv, T, Tn);  // :248
        for (int j = 0; j < 7; ++j) T[j] = Tn[j];
        const int c = kf_n - kf_i;
        for (int j = 0; j < 7; ++j) w.cams[7 * (size_t)c + j] = Tn[j];
        for (const auto& index_pair : kf.global_points_map) {  // :257
            const int landmarkId = index_pair.second;
            const int localId = index_pair.first;
            const double depth = kf.points3d_local[localId][2];  // :261
            const double px = kf.keypoints[localId].pt.x, py = kf.keypoints[localId].pt.y;  // :262
            if (depth <= 1e-15) continue;  // :265-268
            auto it = pt_index.find(landmarkId);
            int pi;
            if (it == pt_index.end()) {  // :271-276
                double* X = map.at(landmarkId).point.data();
                double Xn[3];
                se3_act(initialPoseInv, X, Xn);
                for (int j = 0; j < 3; ++j) X[j] = Xn[j];
                pi = (int)w.landmark_ids.size();
                pt_index.emplace(landmarkId, pi);
                w.landmark_ids.push_back(landmarkId);
                w.points.insert(w.points.end(), Xn, Xn + 3);
            } else {
                pi = it->second;
            }
            w.obs_cam.push_back(c);
            w.obs_pt.push_back(pi);
            w.uv.push_back(px);
            w.uv.push_back(py);
            w.depth.push_back(depth);
        }
    }
    ba_problem prob = w.view();
    ba_summary summary;
    BA_SUMMARY_INIT(summary);
    // :300 — solved even when no observation is admissible: the IntrinsicsPrior block (:236-241) is always
    // added, so Ceres still pulls intrinsics_optimized toward intrinsics_initial (poses have no residual)
    const int32_t rc = solve(&prob, &summary);
    if (status) *status = rc;
    if (summary_out) *summary_out = summary;
    if (rc == BA_OK) {
        for (int i = 0; i < 4; ++i) intrinsics_optimized[i] = w.intr[i];
        for (size_t k = 0; k < w.landmark_ids.size(); ++k) {
            double* X = map.at(w.landmark_ids[k]).point.data();
            for (int j = 0; j < 3; ++j) X[j] = w.points[3 * k + j];
        }
        for (int kf_n = kf_i; kf_n <= kf_f; ++kf_n) {
            double* T = keyframes[kf_n].T_w_c.data();
            for (int j = 0; j < 7; ++j) T[j] = w.cams[7 * (size_t)(kf_n - kf_i) + j];
        }
    }
    // :303-310 map back (also after a failed solve, the re-anchoring is undone)
    for (int kf_n = kf_i; kf_n <= kf_f; ++kf_n) {
        double* T = keyframes[kf_n].T_w_c.data();
        double Tn[7];
        se3_mul(initialPose, T, Tn);
        for (int j = 0; j < 7; ++j) T[j] = Tn[j];
    }
    for (int id : w.landmark_ids) {
        double* X = map.at(id).point.data();
        double Xn[3];
        se3_act(initialPose, X, Xn);
        for (int j = 0; j < 3; ++j) X[j] = Xn[j];
    }
    return true;
}

// The driver's window schedule (main.cpp:132-133, 163-183) as a pure function: which
// [kf_i, kf_f] window (if any) to optimise after a tracking step.
//   window_size > 0: periodic windows every frame_frequency keyframes (+ leftover at the end);
//   window_size < 0: one global window when tracking finished; 0: never.
struct WindowDecision {
    bool run;
    int kf_i, kf_f;
    bool finishes;  // sets is_optimization_finished
};
inline WindowDecision window_schedule(int frame_frequency, int window_size, size_t n_keyframes, bool tracking_finished,
                                      bool optimization_finished, bool tracked_this_frame) {
    WindowDecision d{false, 0, 0, false};
    if (optimization_finished) return d;
    const long n = (long)n_keyframes;
    if (window_size > 0) {
        if (tracked_this_frame && n % frame_frequency == 0 && n >= window_size) {  // :163-168
            d = {true, (int)(n - window_size), (int)(n - 1), false};
        } else if (tracking_finished && n % frame_frequency != 0) {  // :170-176 (leftovers)
            const long first = n - window_size;  // the reference's size_t arithmetic would wrap here
            d = {true, (int)(first < 0 ? 0 : first), (int)(n - 1), true};
        }
    } else if (window_size < 0 && tracking_finished) {  // :179-183
        d = {true, 0, (int)(n - 1), true};
    }
    return d;
}

}  // namespace miba

#endif  // MIBA_BA_WINDOW_HPP
