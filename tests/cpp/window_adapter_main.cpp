// Test driver for include/ba_window.hpp: builds a synthetic keyframe sequence with
// reference-shaped types (mirrors of KeyFrame / Landmark / Map3D, CommonTypes.h:15-43),
// dumps it, runs miba::windowOptimize on one window with the chosen solver and dumps
// the result. tests/test_window_adapter.py replays the dump through the Python mirror.
//   usage: window_adapter_main <in_dump> <out_dump> <seed> <kf_i> <kf_f> [oracle|gpu]
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "ba_window.hpp"

extern "C" int oracle_solve(ba_problem*, const ba_options*, ba_summary*);
extern "C" void oracle_default_options(ba_options*);

struct Pt { float x, y; };
struct KeyPoint { Pt pt; };
struct Vec3 {
    double v[3];
    double& operator[](int i) { return v[i]; }
    double operator[](int i) const { return v[i]; }
    double* data() { return v; }
};
struct SE3 { double d[7]; double* data() { return d; } };
struct KeyFrame {
    std::string timestamp;
    SE3 T_w_c;
    std::vector<KeyPoint> keypoints;
    std::vector<Vec3> points3d_local;
    std::unordered_map<int, int> global_points_map;
};
struct Landmark { Vec3 point; };
using Map3D = std::unordered_map<int, Landmark>;

static void dump(const char* path, std::vector<KeyFrame>& kfs, Map3D& map, const double* K0, const double* K, int kf_i,
                 int kf_f, const ba_summary* s) {
    FILE* f = std::fopen(path, "w");
    std::fprintf(f, "K %zu\n", kfs.size());
    for (auto& kf : kfs) {
        for (int j = 0; j < 7; ++j) std::fprintf(f, "%.17g ", kf.T_w_c.d[j]);
        std::fprintf(f, "%zu\n", kf.keypoints.size());
        for (size_t i = 0; i < kf.keypoints.size(); ++i)
            std::fprintf(f, "%.9g %.9g %.17g %.17g %.17g\n", kf.keypoints[i].pt.x, kf.keypoints[i].pt.y,
                         kf.points3d_local[i][0], kf.points3d_local[i][1], kf.points3d_local[i][2]);
        std::fprintf(f, "%zu\n", kf.global_points_map.size());
        for (auto& pr : kf.global_points_map) std::fprintf(f, "%d %d\n", pr.first, pr.second);
    }
    std::fprintf(f, "L %zu\n", map.size());
    for (auto& pr : map)
        std::fprintf(f, "%d %.17g %.17g %.17g\n", pr.first, pr.second.point.v[0], pr.second.point.v[1], pr.second.point.v[2]);
    std::fprintf(f, "I");
    for (int i = 0; i < 4; ++i) std::fprintf(f, " %.17g", K0[i]);
    for (int i = 0; i < 4; ++i) std::fprintf(f, " %.17g", K[i]);
    std::fprintf(f, "\nW %d %d\n", kf_i, kf_f);
    if (s) std::fprintf(f, "S %.17g %.17g %d %d\n", s->initial_cost, s->final_cost, s->num_iterations, s->termination_type);
    std::fclose(f);
}

int main(int argc, char** argv) {
    if (argc < 6) { std::fprintf(stderr, "usage\n"); return 2; }
    const int seed = std::atoi(argv[3]), kf_i = std::atoi(argv[4]), kf_f = std::atoi(argv[5]);
    const bool gpu = argc > 6 && std::strcmp(argv[6], "gpu") == 0;
    std::mt19937_64 rng(seed);
    std::normal_distribution<double> N01(0.0, 1.0);
    std::uniform_real_distribution<double> U01(0.0, 1.0);
    const int n_kf = 12, per_kf = 40;
    const double Kt[4] = {527.0, 523.5, 320.5, 238.7};
    double K0[4] = {525.0, 525.0, 319.5, 239.5};
    double K[4] = {525.3, 524.6, 319.9, 239.2};  // intrinsics_optimized carried over from a previous window
    // true trajectory: world pose of camera n (first pose NOT identity)
    std::vector<std::vector<double>> Ttrue(n_kf), Test(n_kf);
    for (int n = 0; n < n_kf; ++n) {
        const double yaw = 0.2 + 0.02 * n, half = 0.5 * yaw;
        Ttrue[n] = {0.0, std::sin(half), 0.0, std::cos(half), 1.0 + 0.03 * n, -0.5 + 0.01 * n, 0.3};
        Test[n] = Ttrue[n];
        if (n > 0) {
            for (int j = 4; j < 7; ++j) Test[n][j] += 0.01 * N01(rng);
            double dq[7] = {0.004 * N01(rng), 0.004 * N01(rng), 0.004 * N01(rng), 1.0, 0, 0, 0};
            const double nn = std::sqrt(1 + dq[0] * dq[0] + dq[1] * dq[1] + dq[2] * dq[2]);
            for (int j = 0; j < 4; ++j) dq[j] /= nn;
            double out[7];
            miba::se3_mul(Test[n].data(), dq, out);
            Test[n].assign(out, out + 7);
        }
    }
    std::vector<KeyFrame> kfs(n_kf);
    Map3D map;
    int next_id = 0;
    for (int n = 0; n < n_kf; ++n) {
        std::memcpy(kfs[n].T_w_c.d, Test[n].data(), sizeof(double) * 7);
        kfs[n].timestamp = std::to_string(1305031102.0 + 0.1 * n);
    }
    // landmarks born at keyframe b, seen by b..b+len-1
    for (int b = 0; b < n_kf; ++b)
        for (int q = 0; q < per_kf; ++q) {
            const int len = 2 + (int)(U01(rng) * 3);
            const double u = 60 + U01(rng) * 520, v = 50 + U01(rng) * 380, z = 0.8 + U01(rng) * 3.0;
            const double pc[3] = {(u - Kt[2]) / Kt[0] * z, (v - Kt[3]) / Kt[1] * z, z};
            double Xw[3];
            miba::se3_act(Ttrue[b].data(), pc, Xw);
            const int id = next_id++;
            Landmark lm;
            for (int j = 0; j < 3; ++j) lm.point.v[j] = Xw[j] + 0.02 * N01(rng);
            map.emplace(id, lm);
            for (int n = b; n < std::min(n_kf, b + len); ++n) {
                double Tinv[7], p[3];
                miba::se3_inv(Ttrue[n].data(), Tinv);
                miba::se3_act(Tinv, Xw, p);
                KeyPoint kp;
                kp.pt.x = (float)(Kt[0] * p[0] / p[2] + Kt[2] + 0.5 * N01(rng));
                kp.pt.y = (float)(Kt[1] * p[1] / p[2] + Kt[3] + 0.5 * N01(rng));
                Vec3 loc;
                double d = p[2] * (1 + 0.01 * N01(rng));
                if (U01(rng) < 0.03) d = 0.0;  // missing depth (VirtualSensor MINF / 0)
                loc.v[0] = (kp.pt.x - K0[2]) / K0[0] * d;
                loc.v[1] = (kp.pt.y - K0[3]) / K0[1] * d;
                loc.v[2] = d;
                const int local = (int)kfs[n].keypoints.size();
                kfs[n].keypoints.push_back(kp);
                kfs[n].points3d_local.push_back(loc);
                kfs[n].global_points_map.emplace(local, id);
            }
        }
    dump(argv[1], kfs, map, K0, K, kf_i, kf_f, nullptr);
    ba_options opts;
    oracle_default_options(&opts);
    opts.minimizer_progress_to_stdout = 0;
    ba_summary summ{};
    int32_t status = 0;
    if (gpu) {
#ifdef MIBA_WITH_GPU
        opts.device = 0;
        ba_context* ctx = ba_create(&opts);
        if (!ctx) { std::fprintf(stderr, "ba_create: %s\n", ba_last_error(nullptr)); return 3; }
        miba::windowOptimize(kf_i, kf_f, kfs, map, K0, K, [&](ba_problem* p, ba_summary* s) { return ba_solve(ctx, p, s); },
                             &summ, &status);
        ba_destroy(ctx);
#else
        std::fprintf(stderr, "built without MIBA_WITH_GPU\n");
        return 3;
#endif
    } else {
        miba::windowOptimize(kf_i, kf_f, kfs, map, K0, K,
                             [&](ba_problem* p, ba_summary* s) { return (int32_t)oracle_solve(p, &opts, s); }, &summ,
                             &status);
    }
    dump(argv[2], kfs, map, K0, K, kf_i, kf_f, &summ);
    return status == 0 ? 0 : 4;
}
