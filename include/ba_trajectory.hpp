// ba_trajectory.hpp — header-only host code for the TUM trajectory output of the pipeline
// that surrounds windowOptimize, duck-typed like ba_window.hpp:
//   nearest_interp_1d         src/nearest_interp_1d.cpp:11-78
//   get_first_pose            getFirstPose,  src/OptimizationUtils.cpp:323-370
//   pose_offset               poseOffset,    src/OptimizationUtils.cpp:372-379
//   write_keyframe_poses      write_keyframe_poses_to_file, src/OptimizationUtils.cpp:160-172
// called by the reference driver after the last window (src/main.cpp:191-195).
//
// Poses use the Sophus::SE3d storage order [qx,qy,qz,qw,tx,ty,tz] (keyframes[k].T_w_c.data()).
// keyframes[k].timestamp is the keyframe's timestamp string (CommonTypes.h KeyFrame).
#ifndef MIBA_BA_TRAJECTORY_HPP
#define MIBA_BA_TRAJECTORY_HPP

#include <cmath>
#include <fstream>
#include <ostream>
#include <string>
#include <vector>

#include "ba_window.hpp"

namespace miba {

// Nearest-neighbour interpolation: for every xi the FIRST index k minimising |xi - xd[k]|
// (strict '<' while scanning), yi = yd[k].
inline void nearest_interp_1d(const std::vector<double>& xd, const std::vector<double>& yd,
                              const std::vector<double>& xi, std::vector<double>& yi, std::vector<int>& idx) {
    yi.clear();
    idx.clear();
    for (double x : xi) {
        int best = 0;
        double d = std::fabs(x - xd[0]);
        for (size_t j = 1; j < xd.size(); ++j) {
            const double dj = std::fabs(x - xd[j]);
            if (dj < d) { d = dj; best = (int)j; }
        }
        idx.push_back(best);
        yi.push_back(yd[best]);
    }
}

// Ground-truth pose nearest in time to first_timestamp. The file has 3 header lines, then
// "timestamp tx ty tz qx qy qz qw" records; the quaternion is normalised as Sophus::SO3 does.
// out = [qx,qy,qz,qw,tx,ty,tz]. Returns false if the file has no record.
inline bool get_first_pose(const std::string& first_timestamp, const std::string& ground_truth_path, double out[7]) {
    std::ifstream in(ground_truth_path);
    std::string line;
    for (int i = 0; i < 3; ++i) std::getline(in, line);  // header
    std::vector<double> ts, rec;
    double t, tx, ty, tz, qx, qy, qz, qw;
    while (in >> t >> tx >> ty >> tz >> qx >> qy >> qz >> qw) {
        ts.push_back(t);
        rec.insert(rec.end(), {tx, ty, tz, qx, qy, qz, qw});
    }
    if (ts.empty()) return false;
    std::vector<double> yi;
    std::vector<int> idx;
    nearest_interp_1d(ts, ts, std::vector<double>{std::stod(first_timestamp)}, yi, idx);
    const double* r = rec.data() + 7 * (size_t)idx[0];
    const double n = std::sqrt(r[6] * r[6] + r[3] * r[3] + r[4] * r[4] + r[5] * r[5]);
    out[0] = r[3] / n; out[1] = r[4] / n; out[2] = r[5] / n; out[3] = r[6] / n;
    out[4] = r[0]; out[5] = r[1]; out[6] = r[2];
    return true;
}

// Make initial_pose the first keyframe's pose: T <- (initial * T_0^-1) * T for every keyframe.
template <class KeyFrames>
void pose_offset(KeyFrames& keyframes, const double initial_pose[7]) {
    if (keyframes.size() == 0) return;
    double inv0[7], delta[7];
    se3_inv(keyframes[0].T_w_c.data(), inv0);
    se3_mul(initial_pose, inv0, delta);
    for (auto& kf : keyframes) {
        double* T = kf.T_w_c.data();
        double Tn[7];
        se3_mul(delta, T, Tn);
        for (int j = 0; j < 7; ++j) T[j] = Tn[j];
    }
}

// One line per keyframe: "timestamp tx ty tz qx qy qz qw" with the stream's default
// floating-point formatting (6 significant digits, like the reference's ofstream).
template <class KeyFrames>
void write_keyframe_poses(std::ostream& out, const KeyFrames& keyframes) {
    for (const auto& kf : keyframes) {
        const double* T = kf.T_w_c.data();
        out << kf.timestamp << " " << T[4] << " " << T[5] << " " << T[6] << " " << T[0] << " " << T[1] << " " << T[2]
            << " " << T[3] << "\n";
    }
}

template <class KeyFrames>
bool write_keyframe_poses_to_file(const std::string& path, const KeyFrames& keyframes) {
    std::ofstream out(path);
    if (!out) return false;
    write_keyframe_poses(out, keyframes);
    return (bool)out;
}

}  // namespace miba

#endif  // MIBA_BA_TRAJECTORY_HPP
