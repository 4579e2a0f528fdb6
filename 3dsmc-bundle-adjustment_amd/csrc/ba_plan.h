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
    int obs_tasks = 0;               // ranges of the observation passes (the same split in plan_order)
    std::vector<int> task_cam;       // [obs_tasks * nc] admissible observations per (range, camera)
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
    // ---- device plan (plan_from_device): pt_idx, po_*, co_*, ovf_obs and cam_ac live in HBM only
    bool dev = false;
    int dev_nap = 0, dev_novf = 0;
    int n_ap() const { return dev ? dev_nap : (int)pt_idx.size(); }
    int n_ovf() const { return dev ? dev_novf : (int)ovf_obs.size(); }
};

// The device plan's read-back summary (ba_dplan.hip): a header, then cam_cnt [nc] | fc [nc] | pt_ptr [np + 1] (the
// point-major ranges of the active points, zeros past them) | per active point in the point order: first active
// camera << 16 | last active camera (16 bits each) [np].
enum {
    DP_BAD = 0,    // first out-of-range observation index (INT_MAX: none)
    DP_NOTF32,     // (unused: the host checks obs32 while it stages the pixels)
    DP_NADM,       // admissible observations
    DP_NAC,        // active cameras
    DP_NAP,        // active points (observed by an admissible observation)
    DP_NTILED,     // tiled points (class 0)
    DP_NOVF,       // point-major slots of overflow points on an active camera (ovf_obs)
    DP_TOOLONG,    // a point has more than DP_LONG_MAX admissible observations (the host plan takes over)
    DP_NLONG,      // points of more than 16 observations (sorted by one workgroup each)
    DP_HDR = 16
};
inline size_t dplan_sum_ints(int nc, int np) { return (size_t)DP_HDR + 2 * (size_t)nc + 2 * (size_t)np + 1; }

// the host plan's stage 2 from the device plan's summary (counts, fc, the point order's columns): active cameras,
// pt_ptr, Schur tiles, back-substitution chunks, camera sub-segments. n_adm / obs32 / err are the caller's.
void plan_from_device(const int* sum, int nc, int np, int fixed_cam, const PlanParams& pp, Plan& pl);

// stage 1: index validation + admissibility + per-camera / per-point admissible counts
void plan_count(const PlanInput& in, Plan& pl);
// stage 2: cam_seen[nc] = the camera has an admissible observation on some shard
void plan_order(const PlanInput& in, const std::vector<int>& cam_seen, const PlanParams& pp, Plan& pl);
// stage 3: envelope and band of S from fc (already min-reduced over the shards)
void plan_envelope(Plan& pl);

}  // namespace miba
