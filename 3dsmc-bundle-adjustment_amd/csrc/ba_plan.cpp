// ba_plan.cpp — host-side structure of one window (see ba_plan.h), on a small pool of host threads.
#include "ba_plan.h"

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <mutex>
#include <thread>

namespace miba {

// ---------------------------------------------------------------- thread pool
namespace {

int pick_threads() {
    if (const char* e = std::getenv("MIBA_HOST_THREADS")) {
        const int v = std::atoi(e);
        if (v >= 1) return std::min(v, 256);
    }
    int n = 16;  // one GPU's CPU share on the MI355X boxes
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = std::min(n, std::max(1, CPU_COUNT(&cs)));
    if (const char* e = std::getenv("OMP_NUM_THREADS")) {
        const int v = std::atoi(e);
        if (v >= 1) n = std::min(n, v);
    }
    return std::max(n, 1);
}

class Pool {
   public:
    explicit Pool(int n) : nthreads_(n) {
        for (int i = 1; i < n; ++i) workers_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    int size() const { return nthreads_; }
    void run(int n, const std::function<void(int)>& fn) {
        std::lock_guard<std::mutex> call(call_m_);  // one parallel region at a time (contexts on several threads)
        if (n <= 0) return;
        if (n == 1 || workers_.empty()) {
            for (int t = 0; t < n; ++t) fn(t);
            return;
        }
        {
            std::lock_guard<std::mutex> g(m_);
            job_ = &fn;
            n_ = n;
            next_.store(0, std::memory_order_relaxed);
            busy_ = (int)workers_.size();
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> g(m_);
        done_cv_.wait(g, [this] { return busy_ == 0; });
        job_ = nullptr;
    }

   private:
    void work() {
        for (;;) {
            const int t = next_.fetch_add(1, std::memory_order_relaxed);
            if (t >= n_) break;
            (*job_)(t);
        }
    }
    void loop() {
        unsigned seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
            }
            work();
            {
                std::lock_guard<std::mutex> g(m_);
                if (--busy_ == 0) done_cv_.notify_one();
            }
        }
    }
    int nthreads_;
    std::vector<std::thread> workers_;
    std::mutex m_, call_m_;
    std::condition_variable cv_, done_cv_;
    const std::function<void(int)>* job_ = nullptr;
    int n_ = 0, busy_ = 0;
    unsigned gen_ = 0;
    bool stop_ = false;
    std::atomic<int> next_{0};
};

Pool& pool() {
    static Pool p(pick_threads());
    return p;
}

// [0, n) in `parts` near-equal ranges; range t = [lo(t), lo(t + 1))
struct Split {
    long long n;
    int parts;
    long long lo(int t) const { return n * t / parts; }
};
// tasks for a pass over n items: enough to balance, at least `grain` items each
inline int n_tasks(long long n, long long grain) {
    const long long want = std::max<long long>(1, std::min<long long>(4LL * host_threads(), n / grain));
    return (int)want;
}


// tiles over the tiled points (sequence i < n0 in the point order: first / last active camera, observation count):
// window [base, base + span), span <= tile_win, <= tile_pts points; chunks of <= chunk_pts points and <= chunk_obs
// observations. tile_pts spreads the points over one wave of resident workgroups (no second, partly empty wave of
// tiles), grown until the tile count fits the resident slots.
template <class Fmin, class Fmax, class Fcnt>
void build_tiles(int n0, Fmin pmin, Fmax pmax, Fcnt cnt, const PlanParams& pp, Plan& pl) {
    auto count = [&](int tile_pts) {  // the tile boundaries alone (the trial sizes of the growth loop)
        int n = 0;
        for (int i = 0; i < n0; ++n) {
            const int base = pmin(i);
            int j = i;
            while (j < n0 && j - i < tile_pts && pmax(j) - base < pp.tile_win) ++j;
            i = j;
        }
        return n;
    };
    auto build = [&](int tile_pts) {
        pl.tile_chunk.assign(1, 0); pl.tile_base.clear(); pl.tile_span.clear(); pl.chunk_ap.assign(1, 0);
        int i = 0;
        while (i < n0) {
            const int base = pmin(i);
            int j = i, hi = base;
            while (j < n0 && j - i < tile_pts && pmax(j) - base < pp.tile_win) { hi = std::max(hi, pmax(j)); ++j; }
            int c0 = i;
            while (c0 < j) {
                int c1 = c0, nob = 0;
                while (c1 < j && c1 - c0 < pp.chunk_pts && nob + cnt(c1) <= pp.chunk_obs) { nob += cnt(c1); ++c1; }
                pl.chunk_ap.push_back(c1);
                c0 = c1;
            }
            pl.tile_chunk.push_back((int)pl.chunk_ap.size() - 1);
            pl.tile_base.push_back(base);
            pl.tile_span.push_back(hi - base + 1);
            i = j;
        }
    };
    const int slots = pp.tile_slots - 1;  // one resident slot for the intrinsics-term workgroup
    int tile_pts = 128;
    // small windows (<= 64 chunks of points: the TUM windows) take half-chunk tiles — twice the tiles, each a
    // shorter chain, in a launch that is far from filling the chip (C1 -1 to -2 % per LM iteration)
    const int min_pts = n0 <= 64 * pp.chunk_pts ? std::max(1, pp.chunk_pts / 2) : pp.chunk_pts;
    if (slots > 0) tile_pts = std::max(min_pts, (n0 + slots - 1) / slots);
    if (pp.tile_pts_env > 0) tile_pts = pp.tile_pts_env;
    for (int grow = 0; pp.tile_pts_env <= 0 && slots > 0 && grow < 16 && count(tile_pts) > slots; ++grow)
        tile_pts += std::max(1, tile_pts / 8);
    build(tile_pts);
}

// back-substitution chunks over all active points: <= bs_pts points and <= bs_obs observations
void build_bs_chunks(int n_ap, const PlanParams& pp, Plan& pl) {
    pl.bs_chunk.assign(1, 0);
    for (int a = 0; a < n_ap;) {
        int b = a + 1;
        while (b < n_ap && b - a < pp.bs_pts && pl.pt_ptr[b + 1] - pl.pt_ptr[a] <= pp.bs_obs) ++b;
        pl.bs_chunk.push_back(b);
        a = b;
    }
}

// sub-segments of <= subseg observations (one workgroup each), equal-sized within a camera; ac_seg[ac] = the
// sub-segment range of active camera ac (empty when this shard has no observation of it)
void build_segments(int nc, const std::vector<int>& cstart, const PlanParams& pp, Plan& pl) {
    const int nac = pl.nac;
    pl.seg_ptr.assign(1, 0); pl.seg_cam.clear(); pl.seg_ac.clear();
    pl.ac_seg.assign(2 * (size_t)std::max(nac, 1), 0);
    for (int i = 0; i < nc; ++i)
        if (pl.cam_cnt[i] > 0) {
            const int first = (int)pl.seg_cam.size();
            const int cnt = pl.cam_cnt[i], nseg = (cnt + pp.subseg - 1) / pp.subseg;
            const int ac = pl.cam_ac[i];
            for (int k = 1; k <= nseg; ++k) {
                pl.seg_cam.push_back(i);
                pl.seg_ac.push_back(ac);
                pl.seg_ptr.push_back(cstart[i] + (int)(((long long)cnt * k) / nseg));
            }
            if (ac >= 0) {
                pl.ac_seg[2 * ac] = first;
                pl.ac_seg[2 * ac + 1] = (int)pl.seg_cam.size();
            }
        }
}

// active cameras (Ceres removes unused blocks; the gauge block is constant, :299)
void build_active_cameras(int nc, const std::vector<int>& cam_seen, int fixed_cam, Plan& pl) {
    pl.cam_ac.assign(nc, -1);
    pl.ac_cam.clear();
    for (int i = 0; i < nc; ++i)
        if (cam_seen[i] && i != fixed_cam) { pl.cam_ac[i] = (int)pl.ac_cam.size(); pl.ac_cam.push_back(i); }
    pl.nac = (int)pl.ac_cam.size();
}

}  // namespace

int host_threads() { return pool().size(); }
void host_parallel(int n, const std::function<void(int)>& fn) { pool().run(n, fn); }

// MIBA_PLAN_TIMES=1: per-phase wall times of the plan on stderr (diagnostic)
struct PhaseTimer {
    bool on;
    double t;
    const char* stage;
    explicit PhaseTimer(const char* s) : on(std::getenv("MIBA_PLAN_TIMES") != nullptr), t(now()), stage(s) {}
    static double now() {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
    void mark(const char* what) {
        if (!on) return;
        const double n = now();
        std::fprintf(stderr, "plan %s/%s %.3f ms\n", stage, what, n - t);
        t = n;
    }
};

// ---------------------------------------------------------------- stage 1
void plan_count(const PlanInput& in, Plan& pl) {
    const int nc = in.nc, np = in.np, no = in.no;
    PhaseTimer tm("count");
    pl.err.clear();
    pl.cam_cnt.assign(nc, 0);
    pl.pt_cnt.assign(np, 0);
    pl.adm.assign(no, 0);
    pl.n_adm = 0;
    const int T = n_tasks(no, 32768);
    const Split sp{no, T};
    // per-range camera counts, kept for plan_order's camera-major scatter over the same ranges
    pl.obs_tasks = T;
    pl.task_cam.assign((size_t)T * nc, 0);
    std::vector<int> nadm(T, 0);
    std::vector<long long> bad(T, -1);  // first out-of-range observation of each range
    std::vector<unsigned char> f32ok(T, 1);
    int* ptc = pl.pt_cnt.data();
    // an f64 value that survives the round trip through f32 unchanged (NaN does not)
    auto f32_exact = [](double v) { return (double)(float)v == v; };
    host_parallel(T, [&](int t) {
        int* c = pl.task_cam.data() + (size_t)t * nc;
        int na = 0;
        bool f32 = in.obs_uv != nullptr;
        for (long long k = sp.lo(t); k < sp.lo(t + 1); ++k) {
            const int ci = in.obs_cam[k], pi = in.obs_pt[k];
            if (ci < 0 || ci >= nc || pi < 0 || pi >= np) { bad[t] = k; break; }
            if (!(in.obs_depth[k] > 1e-15)) continue;  // countConstraints / the skip at :265-268
            pl.adm[k] = 1;
            ++na;
            ++c[ci];
            __atomic_fetch_add(ptc + pi, 1, __ATOMIC_RELAXED);
            if (f32) f32 = f32_exact(in.obs_uv[2 * k]) && f32_exact(in.obs_uv[2 * k + 1]) && f32_exact(in.obs_depth[k]);
        }
        nadm[t] = na;
        f32ok[t] = f32;
    });
    for (int t = 0; t < T; ++t)
        if (bad[t] >= 0) { pl.err = "observation index out of range"; return; }
    pl.obs32 = in.obs_uv != nullptr;
    for (int t = 0; t < T; ++t) {
        pl.n_adm += nadm[t];
        pl.obs32 = pl.obs32 && f32ok[t];
        for (int i = 0; i < nc; ++i) pl.cam_cnt[i] += pl.task_cam[(size_t)t * nc + i];
    }
    tm.mark("all");
}

// ---------------------------------------------------------------- stage 2
void plan_order(const PlanInput& in, const std::vector<int>& cam_seen, const PlanParams& pp, Plan& pl) {
    const int nc = in.nc, np = in.np, no = in.no;
    const int n_adm = pl.n_adm;
    PhaseTimer tm("order");
    pl.dev = false;
    build_active_cameras(nc, cam_seen, in.fixed_cam, pl);
    const int nac = pl.nac;
    const int* cam_ac = pl.cam_ac.data();
    // CSR of admissible obs by original point index, each list ordered by (active camera, obs index): the order
    // of a stable sort by active camera of the obs in index order
    std::vector<int> pptr(np + 1, 0);
    for (int i = 0; i < np; ++i) pptr[i + 1] = pptr[i] + pl.pt_cnt[i];
    std::vector<int> plist(n_adm);
    // one pass over the observations fills both: the point lists (atomic slots, sorted below) and the camera-major
    // order (one segment per camera with admissible obs, gauge included; each camera's in index order), a counting
    // scatter whose per-range offsets come from plan_count's per-range camera counts over the same ranges
    std::vector<int> cstart(nc + 1, 0);
    for (int i = 0; i < nc; ++i) cstart[i + 1] = cstart[i] + pl.cam_cnt[i];
    pl.co_orig.resize(n_adm);
    pl.co_dest.resize(no);
    pl.po_dest.resize(no);  // the admissible entries in the point-major pass below
    {
        std::vector<int> cur(pptr.begin(), pptr.end() - 1);
        int* cp = cur.data();
        const int T = pl.obs_tasks;
        const Split sp{no, T};
        std::vector<int> off(pl.task_cam);
        {
            std::vector<int> run(cstart.begin(), cstart.end() - 1);
            for (int t = 0; t < T; ++t)
                for (int i = 0; i < nc; ++i) {
                    int& o = off[(size_t)t * nc + i];
                    const int v = o;
                    o = run[i];
                    run[i] += v;
                }
        }
        host_parallel(T, [&](int t) {
            int* c = off.data() + (size_t)t * nc;
            for (long long k = sp.lo(t); k < sp.lo(t + 1); ++k)
                if (pl.adm[k]) {
                    plist[__atomic_fetch_add(cp + in.obs_pt[k], 1, __ATOMIC_RELAXED)] = (int)k;
                    const int q = c[in.obs_cam[k]]++;
                    pl.co_orig[q] = (int)k;
                    pl.co_dest[k] = q;
                } else {
                    pl.co_dest[k] = -1;
                    pl.po_dest[k] = -1;
                }
        });
    }
    tm.mark("point_camera_lists");
    pl.pmin.assign(np, INT_MAX);
    pl.pmax.assign(np, -1);
    std::vector<signed char> pclass(np, -1);  // 0 tiled, 1 overflow (Schur via atomics), 2 gauge-only
    // envelope of S: fc[a] = first co-visible active camera of active camera a (the min over the first cameras of
    // the points it observes), gathered from each point's sorted list
    pl.fc.resize(nac);
    for (int a = 0; a < nac; ++a) pl.fc[a] = a;
    {
        const int T = n_tasks(np, 8192);
        const Split sp{np, T};
        std::vector<int> floc((size_t)T * std::max(nac, 1), INT_MAX);
        host_parallel(T, [&](int t) {
            std::vector<long long> key;
            int* f = floc.data() + (size_t)t * std::max(nac, 1);
            for (long long i = sp.lo(t); i < sp.lo(t + 1); ++i) {
                const int b = pptr[i], e = pptr[i + 1];
                if (e == b) continue;
                int* L = plist.data() + b;
                const int m = e - b;
                // key = (active camera + 1, obs index): unique, so the order does not depend on the fill order
                key.resize(m);
                for (int q = 0; q < m; ++q)
                    key[q] = ((long long)(cam_ac[in.obs_cam[L[q]]] + 1) << 32) | (unsigned)L[q];
                if (m <= 24) {
                    for (int q = 1; q < m; ++q) {
                        const long long v = key[q];
                        int r = q - 1;
                        while (r >= 0 && key[r] > v) { key[r + 1] = key[r]; --r; }
                        key[r + 1] = v;
                    }
                } else {
                    std::sort(key.begin(), key.end());
                }
                bool dup = false;
                int prev = -2, lo = INT_MAX, hi = -1;
                for (int q = 0; q < m; ++q) {
                    L[q] = (int)(unsigned)(key[q] & 0xffffffffLL);
                    const int a = (int)(key[q] >> 32) - 1;
                    if (a < 0) continue;
                    lo = std::min(lo, a);
                    hi = std::max(hi, a);
                    if (a == prev) dup = true;
                    prev = a;
                }
                pl.pmin[i] = lo;
                pl.pmax[i] = hi;
                if (hi < 0) pclass[i] = 2;
                else if (dup || hi - lo + 1 > pp.tile_win || m > pp.chunk_obs) pclass[i] = 1;
                else pclass[i] = 0;
                for (int q = 0; q < m; ++q) {
                    const int a = (int)(key[q] >> 32) - 1;
                    if (a >= 0) f[a] = std::min(f[a], lo);
                }
            }
        });
        for (int t = 0; t < T; ++t)
            for (int a = 0; a < nac; ++a) pl.fc[a] = std::min(pl.fc[a], floc[(size_t)t * nac + a]);
    }
    tm.mark("point_sort_class_fc");
    // points by class; tiled and overflow points by first camera, ties in point order (a stable counting sort)
    std::vector<int> cls[3];
    {
        std::vector<int> cnt0(nac + 1, 0), cnt1(nac + 1, 0);
        int n2 = 0;
        for (int i = 0; i < np; ++i) {
            if (pclass[i] == 0) ++cnt0[pl.pmin[i] + 1];
            else if (pclass[i] == 1) ++cnt1[pl.pmin[i] + 1];
            else if (pclass[i] == 2) ++n2;
        }
        for (int a = 0; a < nac; ++a) { cnt0[a + 1] += cnt0[a]; cnt1[a + 1] += cnt1[a]; }
        cls[0].resize(cnt0[nac]);
        cls[1].resize(cnt1[nac]);
        cls[2].reserve(n2);
        for (int i = 0; i < np; ++i) {
            if (pclass[i] == 0) cls[0][cnt0[pl.pmin[i]]++] = i;
            else if (pclass[i] == 1) cls[1][cnt1[pl.pmin[i]]++] = i;
            else if (pclass[i] == 2) cls[2].push_back(i);
        }
    }
    {
        const std::vector<int>& T0 = cls[0];
        build_tiles((int)T0.size(), [&](int i) { return pl.pmin[T0[i]]; }, [&](int i) { return pl.pmax[T0[i]]; },
                    [&](int i) { return pl.pt_cnt[T0[i]]; }, pp, pl);
    }
    tm.mark("class_sort_tiles");
    // active point order: tiled (tile order), overflow, gauge-only; point-major obs in that order
    pl.pt_idx.clear();
    pl.pt_idx.reserve(cls[0].size() + cls[1].size() + cls[2].size());
    for (int k = 0; k < 3; ++k) pl.pt_idx.insert(pl.pt_idx.end(), cls[k].begin(), cls[k].end());
    const int n_ap = (int)pl.pt_idx.size();
    pl.n_tiled = (int)cls[0].size();
    pl.pt_ptr.assign(n_ap + 1, 0);
    for (int a = 0; a < n_ap; ++a) pl.pt_ptr[a + 1] = pl.pt_ptr[a] + pl.pt_cnt[pl.pt_idx[a]];
    pl.po_orig.resize(n_adm);
    {
        const int T = n_tasks(n_ap, 8192);
        const Split sp{n_ap, T};
        host_parallel(T, [&](int t) {
            for (long long a = sp.lo(t); a < sp.lo(t + 1); ++a) {
                const int i = pl.pt_idx[a];
                for (int j = pptr[i], q = pl.pt_ptr[a]; j < pptr[i + 1]; ++j, ++q) {
                    pl.po_orig[q] = plist[j];
                    pl.po_dest[plist[j]] = q;
                }
            }
        });
    }
    tm.mark("point_major");
    pl.ovf_obs.clear();
    for (int q = pl.pt_ptr[pl.n_tiled]; q < pl.pt_ptr[n_ap]; ++q)
        if (cam_ac[in.obs_cam[pl.po_orig[q]]] >= 0) pl.ovf_obs.push_back(q);
    build_bs_chunks(n_ap, pp, pl);
    tm.mark("ovf_bs");
    build_segments(nc, cstart, pp, pl);
    tm.mark("segments");
}

// ---------------------------------------------------------------- stage 2 from the device plan
void plan_from_device(const int* sum, int nc, int np, int fixed_cam, const PlanParams& pp, Plan& pl) {
    PhaseTimer tm("device");
    pl.dev = true;
    pl.cam_cnt.assign(sum + DP_HDR, sum + DP_HDR + nc);
    pl.pt_cnt.clear(); pl.adm.clear(); pl.pmin.clear(); pl.pmax.clear(); pl.task_cam.clear();
    pl.pt_idx.clear(); pl.po_orig.clear(); pl.po_dest.clear(); pl.co_orig.clear(); pl.co_dest.clear();
    pl.ovf_obs.clear();
    std::vector<int> cam_seen(nc);
    for (int i = 0; i < nc; ++i) cam_seen[i] = pl.cam_cnt[i] > 0;
    build_active_cameras(nc, cam_seen, fixed_cam, pl);
    const int nac = pl.nac;
    const int* fc = sum + DP_HDR + nc;
    const int* ptp = fc + nc;
    const int* pmm = ptp + np + 1;
    pl.fc.assign(fc, fc + nac);
    const int n_ap = pl.dev_nap = sum[DP_NAP];
    pl.n_tiled = sum[DP_NTILED];
    pl.dev_novf = sum[DP_NOVF];
    pl.pt_ptr.assign(ptp, ptp + n_ap + 1);
    build_tiles(pl.n_tiled, [&](int i) { return (int)((unsigned)pmm[i] >> 16); },
                [&](int i) { return (int)((unsigned)pmm[i] & 0xffffu); }, [&](int i) { return ptp[i + 1] - ptp[i]; },
                pp, pl);
    build_bs_chunks(n_ap, pp, pl);
    std::vector<int> cstart(nc + 1, 0);
    for (int i = 0; i < nc; ++i) cstart[i + 1] = cstart[i] + pl.cam_cnt[i];
    build_segments(nc, cstart, pp, pl);
    tm.mark("tiles_chunks_segments");
}

// ---------------------------------------------------------------- stage 3
void plan_envelope(Plan& pl) {
    const int nac = pl.nac;
    pl.n = 6 * nac + 4;
    pl.npad = (pl.n + 15) / 16 * 16;
    const int nb = pl.nb = pl.npad / 16;
    pl.fcol.assign(nb, INT_MAX);
    for (int r = 0; r < pl.npad; ++r) {
        const int first = (r < 6 * nac) ? 6 * pl.fc[r / 6] : 0;
        pl.fcol[r / 16] = std::min(pl.fcol[r / 16], first / 16);
    }
    pl.cam_band = 0;
    for (int a = 0; a < nac; ++a) pl.cam_band = std::max(pl.cam_band, a - pl.fc[a]);
    // band width (in 16-tiles) of the camera part; the last block row is the dense border
    pl.band_w = 0;
    for (int i = 0; i + 1 < nb; ++i) pl.band_w = std::max(pl.band_w, i - pl.fcol[i]);
    pl.rptr.assign(nb + 1, 0);
    pl.rows.clear();
    for (int k = 0; k < nb; ++k) {
        for (int i = k + 1; i < nb; ++i)
            if (pl.fcol[i] <= k) pl.rows.push_back(i);
        pl.rptr[k + 1] = (int)pl.rows.size();
    }
    pl.env_tile.clear();
    for (int i = 0; i < nb; ++i)
        for (int j = pl.fcol[i]; j <= i; ++j) {
            pl.env_tile.push_back(i);
            pl.env_tile.push_back(j);
        }
}

}  // namespace miba
