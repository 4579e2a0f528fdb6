// ba_plan.h — host-side structure of one window (libmiba, internal; host-only C++, no HIP types).
//
// ba_prepare()'s host work, the part of windowOptimize (OptimizationUtils.cpp:231-299) that a fresh
// Ceres problem rebuilds on every call: admissibility and the N count (countConstraints :184-213, the
// skip at :265-268), the active parameter blocks (Ceres drops blocks without residuals; the gauge block
// kf_i is constant, :299), and the orderings the kernels stream — observations grouped by point (each
// point's list by active camera), points grouped into Schur tiles by first camera, observations grouped
// by camera — plus the envelope of the reduced camera system.
//
// The passes over observations and points run on a small pool of host threads (MIBA_HOST_THREADS, else
// min(16, OMP_NUM_THREADS, the affinity mask)); every result is independent of the thread count (each
// ordering is a total order: parallel fills are followed by sorts on a unique key, or are two-pass
// counting scatters), so the plan is identical to a serial build.
#pragma once
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace miba {

// Runs fn(task) for task in [0, n) on the pool (the calling thread takes part); returns after all ran.
void host_parallel(int n, const std::function<void(int)>& fn);
int host_threads();

struct PlanInput {
    int nc = 0, np = 0, no = 0, fixed_cam = -1;
    const int32_t* obs_cam = nullptr;
    const int32_t* obs_pt = nullptr;
    const double* obs_depth = nullptr;
    const double* obs_uv = nullptr;  // nullptr: no obs32 check (Plan::obs32 stays false)
};

struct PlanParams {
    int tile_win = 12;      // cameras per Schur tile window
    int chunk_pts = 32;     // points per Schur chunk
    int chunk_obs = 256;    // observations per Schur chunk (a point with more is an overflow point)
    int tile_slots = 0;     // resident Schur tile workgroups (0: unknown) -> points per tile
    int tile_pts_env = 0;   // MIBA_TILE_PTS override (0: none)
    int bs_pts = 128, bs_obs = 1024;  // back-substitution chunks
    int subseg = 1024;      // observations per camera sub-segment
};

struct Plan {
    // ---- stage 1 (plan_count): validation, admissibility, counts
    std::string err;                 // non-empty: the problem is malformed
    std::vector<int> cam_cnt, pt_cnt;
    std::vector<unsigned char> adm;  // observation k admissible (depth > 1e-15)
    int n_adm = 0;
    bool obs32 = false;              // every admissible pixel and depth is exactly an f32 (DevProblem::obs32)
    // ---- stage 2 (plan_order): given the active cameras (cam_seen, all shards)
    std::vector<int> cam_ac;         // camera -> active index or -1 (fixed / unobserved)
    std::vector<int> ac_cam;         // active camera -> camera
    int nac = 0;
    std::vector<int> pmin, pmax;     // per point: first / last active camera of its observations
    std::vector<int> pt_idx;         // active point order: tiled (by first camera) | overflow | gauge-only
    std::vector<int> pt_ptr;         // [n_ap + 1] point-major observation ranges
    std::vector<int> po_orig;        // point-major admissible obs -> original observation index
    int n_tiled = 0;
    std::vector<int> tile_chunk, tile_base, tile_span, chunk_ap;  // Schur tiles / chunks
    std::vector<int> ovf_obs;        // point-major obs of overflow points on an active camera
    std::vector<int> bs_chunk;       // back-substitution chunk boundaries (active points)
    std::vector<int> co_orig;        // camera-major admissible obs -> original index (per camera in index order)
    std::vector<int> po_dest, co_dest;  // [no] original index -> point-major / camera-major slot (-1: not admissible)
    std::vector<int> seg_ptr, seg_cam, seg_ac;  // camera sub-segments
    std::vector<int> ac_seg;         // [2 * nac]: sub-segment range of each active camera
    std::vector<int> fc;             // first co-visible active camera of each active camera (this shard)
    // ---- stage 3 (plan_envelope): given fc (union over the shards)
    int n = 0, npad = 0, nb = 0, cam_band = 0, band_w = 0;
    std::vector<int> fcol, rptr, rows;
    std::vector<int> env_tile;       // (block row, block col) pairs, flattened
    int n_ap() const { return (int)pt_idx.size(); }
};

// stage 1: index validation + admissibility + per-camera / per-point admissible counts
void plan_count(const PlanInput& in, Plan& pl);
// stage 2: cam_seen[nc] = the camera has an admissible observation on some shard
void plan_order(const PlanInput& in, const std::vector<int>& cam_seen, const PlanParams& pp, Plan& pl);
// stage 3: envelope and band of S from fc (already min-reduced over the shards)
void plan_envelope(Plan& pl);

}  // namespace miba
