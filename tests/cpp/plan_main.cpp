// plan_main.cpp — host-plan harness (built by tests/test_host_plan.py, with and without sanitizers).
//
// Links only csrc/ba_plan.cpp (the host plan of ba_prepare: admissibility and counts, the point-major CSR, the
// Schur tiles / chunks, the back-substitution chunks, the camera-major order and sub-segments, the envelope of S)
// and builds the plan of generated windows shaped like BASELINE's configs — banded co-visibility, shuffled
// observation order, duplicate keypoint links, inadmissible depths, non-f32 pixels — several times each. It prints
// one line per plan field: its length and an FNV-1a hash of its contents. The test runs it at MIBA_HOST_THREADS=1
// and =16 and requires identical output (ba_plan.h: the plan does not depend on the thread count), and runs it
// under ThreadSanitizer and under AddressSanitizer + UndefinedBehaviorSanitizer.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ba_plan.h"

using miba::Plan;
using miba::PlanInput;
using miba::PlanParams;

static uint64_t g_rng = 0;
static uint64_t next_u64() {  // splitmix64
    uint64_t z = (g_rng += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static double urand() { return (double)(next_u64() >> 11) * (1.0 / 9007199254740992.0); }
static int irand(int n) { return (int)(next_u64() % (uint64_t)n); }

struct Window {
    int nc = 0, np = 0, fixed_cam = 0;
    std::vector<int32_t> oc, op;
    std::vector<double> uv, depth;
};

// nc cameras, np points, each point seen by k in [kmin, kmax] cameras of a contiguous band around its birth
// camera (band <= span); options: shuffled order, a fraction of duplicate links, of inadmissible depths, of
// non-f32 pixels, of points spanning a wide band (overflow points)
static Window make_window(int nc, int np, int kmin, int kmax, int span, bool shuffle, double dup, double bad,
                          double nonf32, double wide, uint64_t seed) {
    g_rng = seed * 0x2545F4914F6CDD1Dull + 17;
    Window w;
    w.nc = nc;
    w.np = np;
    for (int i = 0; i < np; ++i) {
        const int k = kmin + irand(kmax - kmin + 1);
        const bool is_wide = urand() < wide;
        const int sp = is_wide ? std::min(nc, 3 * span) : std::min(nc, span);
        const int birth = irand(std::max(1, nc - sp + 1));
        for (int j = 0; j < k; ++j) {
            const int cam = birth + (sp > 1 ? (j * sp) / k : 0);
            w.oc.push_back(cam);
            w.op.push_back(i);
            float u = (float)(640.0 * urand()), v = (float)(480.0 * urand());
            w.uv.push_back(u);
            w.uv.push_back(v);
            w.depth.push_back((float)(0.8 + 3.2 * urand()));
        }
    }
    const size_t n0 = w.oc.size();
    for (size_t k = 0; k < n0; ++k)
        if (urand() < dup) {  // the same keypoint linked twice (Map3D duplicate links)
            w.oc.push_back(w.oc[k]);
            w.op.push_back(w.op[k]);
            w.uv.push_back(w.uv[2 * k]);
            w.uv.push_back(w.uv[2 * k + 1]);
            w.depth.push_back(w.depth[k]);
        }
    const size_t no = w.oc.size();
    for (size_t k = 0; k < no; ++k) {
        if (urand() < bad) w.depth[k] = (k & 1) ? 0.0 : -1.0;  // inadmissible (depth <= 1e-15)
        if (urand() < nonf32) w.uv[2 * k] += 1e-7;               // not an exact f32
    }
    if (shuffle)
        for (size_t k = no; k > 1; --k) {
            const size_t j = next_u64() % k;
            std::swap(w.oc[k - 1], w.oc[j]);
            std::swap(w.op[k - 1], w.op[j]);
            std::swap(w.uv[2 * (k - 1)], w.uv[2 * j]);
            std::swap(w.uv[2 * (k - 1) + 1], w.uv[2 * j + 1]);
            std::swap(w.depth[k - 1], w.depth[j]);
        }
    return w;
}

template <class T>
static void emit(const char* name, const std::vector<T>& v) {
    uint64_t h = 1469598103934665603ull;
    const unsigned char* b = reinterpret_cast<const unsigned char*>(v.data());
    for (size_t k = 0; k < v.size() * sizeof(T); ++k) h = (h ^ b[k]) * 1099511628211ull;
    std::printf("  %-10s n=%zu h=%016llx\n", name, v.size(), (unsigned long long)h);
}

static void run(const char* label, const Window& w, int subseg, int tile_slots) {
    PlanInput in;
    in.nc = w.nc;
    in.np = w.np;
    in.no = (int)w.oc.size();
    in.fixed_cam = w.fixed_cam;
    in.obs_cam = w.oc.data();
    in.obs_pt = w.op.data();
    in.obs_depth = w.depth.data();
    in.obs_uv = w.uv.data();
    Plan pl;
    miba::plan_count(in, pl);
    std::printf("%s: err='%s' n_adm=%d obs32=%d\n", label, pl.err.c_str(), pl.n_adm, (int)pl.obs32);
    if (!pl.err.empty()) return;
    std::vector<int> cam_seen(w.nc);
    for (int i = 0; i < w.nc; ++i) cam_seen[i] = pl.cam_cnt[i] > 0;
    PlanParams pp;
    pp.tile_slots = tile_slots;
    pp.subseg = subseg;
    miba::plan_order(in, cam_seen, pp, pl);
    miba::plan_envelope(pl);
    std::printf("  nac=%d n_ap=%d n_tiled=%d n=%d npad=%d nb=%d cam_band=%d band_w=%d\n", pl.nac, pl.n_ap(),
                pl.n_tiled, pl.n, pl.npad, pl.nb, pl.cam_band, pl.band_w);
    emit("cam_cnt", pl.cam_cnt); emit("pt_cnt", pl.pt_cnt); emit("adm", pl.adm);
    emit("cam_ac", pl.cam_ac); emit("ac_cam", pl.ac_cam); emit("pmin", pl.pmin); emit("pmax", pl.pmax);
    emit("pt_idx", pl.pt_idx); emit("pt_ptr", pl.pt_ptr); emit("po_orig", pl.po_orig);
    emit("tile_chunk", pl.tile_chunk); emit("tile_base", pl.tile_base); emit("tile_span", pl.tile_span);
    emit("chunk_ap", pl.chunk_ap); emit("ovf_obs", pl.ovf_obs); emit("bs_chunk", pl.bs_chunk);
    emit("co_orig", pl.co_orig); emit("seg_ptr", pl.seg_ptr); emit("seg_cam", pl.seg_cam);
    emit("seg_ac", pl.seg_ac); emit("ac_seg", pl.ac_seg); emit("fc", pl.fc); emit("fcol", pl.fcol);
    emit("rptr", pl.rptr); emit("rows", pl.rows); emit("env_tile", pl.env_tile);
    emit("po_dest", pl.po_dest); emit("co_dest", pl.co_dest);
    // the device scatter's slots (k_prep_gather): each admissible observation's slot in both orders, -1 otherwise
    bool inv = (int)pl.po_dest.size() == in.no && (int)pl.co_dest.size() == in.no;
    for (int q = 0; inv && q < pl.n_adm; ++q)
        inv = pl.po_dest[pl.po_orig[q]] == q && pl.co_dest[pl.co_orig[q]] == q;
    for (int k = 0; inv && k < in.no; ++k)
        inv = pl.adm[k] ? (pl.po_dest[k] >= 0 && pl.co_dest[k] >= 0) : (pl.po_dest[k] == -1 && pl.co_dest[k] == -1);
    std::printf("  dest_inverse=%d\n", (int)inv);
}

int main(int argc, char** argv) {
    const bool big = argc > 1 && std::strcmp(argv[1], "big") == 0;
    const int reps = 3;  // the same plan again on the same pool: racy fills would show as differing lines
    std::printf("host_threads=%d\n", miba::host_threads());
    for (int r = 0; r < reps; ++r) {
        std::printf("--- rep %d\n", r);
        // C2-shaped: 20 cams / 5k points / 10 obs per point, banded
        run("c2", make_window(20, 5000, 10, 10, 10, false, 0.0, 0.0, 0.0, 0.0, 2), 1024, 512);
        // shuffled, duplicate links, inadmissible depths, overflow points
        run("c2_shuffled_dup_bad", make_window(20, 5000, 2, 14, 10, true, 0.03, 0.05, 0.0, 0.02, 3), 1024, 512);
        // non-f32 pixels (the f64 layout), gauge camera 3
        {
            Window w = make_window(40, 8000, 3, 9, 8, true, 0.0, 0.02, 0.01, 0.0, 4);
            w.fixed_cam = 3;
            run("c3_nonf32_gauge3", w, 1024, 512);
        }
        // cameras without observations, points without admissible observations
        {
            Window w = make_window(30, 3000, 1, 4, 5, true, 0.0, 0.3, 0.0, 0.0, 6);
            w.nc = 36;
            w.np = 3100;
            run("holes", w, 256, 64);
        }
        // malformed: an out-of-range index
        {
            Window w = make_window(10, 100, 2, 4, 4, false, 0.0, 0.0, 0.0, 0.0, 7);
            w.op[57] = w.np;
            run("bad_index", w, 1024, 512);
        }
        if (big)  // C4-shaped: 200 cams / 100k points / 1M obs (large-window sub-segments)
            run("c4", make_window(200, 100000, 10, 10, 10, true, 0.0, 0.01, 0.0, 0.0, 5), 1700, 512);
    }
    std::printf("plan_main: ok\n");
    return 0;
}
