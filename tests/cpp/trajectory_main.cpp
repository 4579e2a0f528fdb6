// Test harness for include/ba_trajectory.hpp: reads keyframes ("timestamp qx qy qz qw tx ty tz"
// per line) from argv[2], the ground-truth file argv[1]; runs get_first_pose(keyframes[0].timestamp),
// pose_offset, write_keyframe_poses to stdout (the reference driver's main.cpp:191-195 sequence).
#include <cstdio>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "ba_trajectory.hpp"

struct Pose {
    double v[7];
    double* data() { return v; }
    const double* data() const { return v; }
};
struct KF {
    Pose T_w_c;
    std::string timestamp;
};

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    std::ifstream in(argv[2]);
    std::vector<KF> kfs;
    KF k;
    while (in >> k.timestamp >> k.T_w_c.v[0] >> k.T_w_c.v[1] >> k.T_w_c.v[2] >> k.T_w_c.v[3] >> k.T_w_c.v[4] >>
           k.T_w_c.v[5] >> k.T_w_c.v[6])
        kfs.push_back(k);
    double first[7];
    if (kfs.empty() || !miba::get_first_pose(kfs[0].timestamp, argv[1], first)) return 3;
    miba::pose_offset(kfs, first);
    miba::write_keyframe_poses(std::cout, kfs);
    return 0;
}
