// ba_solver.cpp — libmiba host side: the C-ABI of include/ba.h.
//
// ba_solve() replaces `ceres::Solve(globalProblem.options, &problem, &summary)`
// at /root/reference/src/OptimizationUtils.cpp:300 for the problem assembled at
// :236-299. The trust-region control flow below restates Ceres 2.0's
// TrustRegionMinimizer::Minimize with LevenbergMarquardtStrategy;
// every numeric pass over observations / points / the reduced camera system runs
// on the GPU (ba_kernels.hip). Per iteration the host reads back 8 scalars.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cstdint>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ba.h"
#include "ba_host.h"
#include "ba_kernels.h"
#include "ba_dplan.h"
#include "ba_plan.h"

using namespace miba;

namespace {

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes, 256);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

enum BufId {
    B_CAMS0, B_CAMS1, B_PTS0, B_PTS1, B_K0, B_K1, B_PRIOR,
    B_PO_CAM, B_PO_AC, B_PO_UV, B_PO_DEP, B_PO_AP, B_PO_PT,
    B_CO_PT, B_CO_UV, B_CO_DEP, B_RAW_CAM, B_RAW_PT, B_RAW_UV, B_RAW_DEP, B_PLAN,
    B_CAMDATA, B_SEGINTR, B_LIN, B_SCALE, B_CNP, B_PDATA, B_S, B_RHS, B_DELTA, B_PART, B_SCAL, B_FLAG,
    B_BCR, B_CAMDATA_LOC, B_ENV_LOC, B_RED, B_PREP, B_CAMPART, B_STATE, B_LOG, B_CAMS_INIT, B_PTS_INIT, B_K_INIT,
    B_DBG0, B_DBG1, B_DBG2, B_DBG3, B_DET_TBUF, B_PO_REC, B_CO_REC,
    B_RAW_ADM, B_DP_SCRATCH, B_DP_PO_DEST, B_DP_CO_DEST, B_DP_CAM_AC, B_DP_PT_IDX, B_DP_OVF, B_DP_SUM, B_TAIL_Y,
    B_COUNT
};

}  // namespace

struct ba_context {
    ba_options opts;
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    unsigned* hprog = nullptr;  // host-mapped LM progress word (LmParams::progress)
    unsigned* dprog = nullptr;  // its device address
    double* hres = nullptr;     // pinned staging of the solved cameras + intrinsics (async device-to-host copies)
    size_t hres_cap = 0;        // its capacity in doubles
    DevBuf buf[B_COUNT];
    std::string err;
    // host-side structure of the last prepared problem (ba_plan.h; plan.po_orig: point-major admissible obs ->
    // original obs index)
    Plan plan;
    std::vector<int> pt_idx, ac_cam;
    char* stage = nullptr;  // pinned staging of ba_prepare's uploads: [raw observations | plan index arrays]
    size_t stage_cap = 0;
    char* pstage = nullptr;  // pinned staging of the parameter uploads (cameras | points | intrinsics | prior)
    size_t pstage_cap = 0;
    hipStream_t copy_stream = nullptr;  // the device plan's pixel DMA, beside the plan passes on `stream`
    hipEvent_t ev_idx = nullptr, ev_uv = nullptr;  // indices / depths DMA'd; pixels DMA'd
    bool uv_pending = false;  // the pixel DMA of the last prepare has not been waited for on `stream`
    int* rsum = nullptr;     // the device plan's summary (ba_plan.h), in mapped host memory the last pass writes
    int* rsum_dev = nullptr; // its device address
    size_t rsum_cap = 0;     // in ints
    std::vector<std::pair<size_t, size_t>> plan_parts;  // (offset, ints) of each array in B_PLAN (digest)
    // plan cache (ba_options.rebuild_plan = 0): the structure key of the last full prepare; while plan_ok the
    // staging buffer's raw region holds that window's observations (the reuse check compares against it) and
    // `raw` the device gather inputs (B_RAW_* + the plan's orderings in B_PLAN)
    struct PlanKey {
        int nc = -1, np = -1, no = -1, fixed_cam = 0, det = 0, obs32 = 0;
        unsigned long long env = 0;
        bool operator==(const PlanKey& o) const {
            return nc == o.nc && np == o.np && no == o.no && fixed_cam == o.fixed_cam && det == o.det &&
                   env == o.env;
        }
    } key;
    bool plan_ok = false;
    PrepRaw raw{};
    ba_prepare_info pinfo{};
    DevProblem P{};
    DevWork W{};
    BaConsts C{};
    int nblk_pt = 0;
    bool prepared = false;
    int n_tiles = 0, n_ovf_obs = 0, n_tiled_pts = 0;
    int n_adm_all = 0;  // admissible observations over all landmark shards
    int sw_full = 0;    // DevWork::sw as the last full prepare chose it (a timeout re-run clears W.sw)
    int tail_full = 0;  // DevWork::tail likewise
    int bsfin_full = 0;  // DevWork::bsfin likewise
    bool tail_possible = false;  // the window's LM loop can take the band tail launch (set before bcr_setup)
    int prep_nc = -1, prep_np = -1, prep_no = -1;
    int last_iter = -1;        // iterations of the last solve (ba_iteration_log rows - 1)
    // shard_min_obs: a window below the threshold is gathered onto every rank and solved there alone; the
    // communicator is parked meanwhile (restored by the next prepare), the rank's points are the slice
    // [gather_off, gather_off + its n_points) of the gathered window
    Comm comm_parked;
    int gather_off = 0;
    int dev_np = 0;  // points on the device (the gathered window's when gathered)
    struct Gathered {
        std::vector<double> cams, pts, uv, dep;
        std::vector<int> oc, op;
        double intr[4], prior[4];
    } gw;
    bool bcr_fallback = false;  // a resident BCR kernel timed out: per-level launches from then on
    unsigned long long bcr_launches = 0;  // split-kernel launches since the BCR workspace was initialised
    int bcr_retries = 0;        // iterations re-run with the per-level launches after a hand-off timeout
    // per-kernel profiling
    Prof prof;
    bool prof_events = false;
    int k_launches[K_COUNT] = {0};
    double k_ms[K_COUNT] = {0};
    double k_bytes[K_COUNT] = {0};
    double k_flops[K_COUNT] = {0};
    Prof* pf() { return opts.profile_kernels ? &prof : nullptr; }
};

static void flush_prof(ba_context* ctx) {
    Prof& P = ctx->prof;
    for (int i = 0; i < P.n; ++i) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, P.ev[2 * i], P.ev[2 * i + 1]) == hipSuccess) {
            ctx->k_ms[P.id[i]] += ms;
            ctx->k_launches[P.id[i]] += 1;
        }
    }
    P.n = 0;
}

static thread_local std::string g_err;

void miba_set_error(const std::string& msg) { g_err = msg; }

#define HIPCHECK(ctx, x)                                                                  \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            (ctx)->err = std::string("HIP error: ") + hipGetErrorString(e_) + " at " #x; \
            return BA_E_DEVICE;                                                           \
        }                                                                                 \
    } while (0)

template <class T>
static hipError_t upload(ba_context* ctx, int id, const T* src, size_t n) {
    hipError_t e = ctx->buf[id].ensure(sizeof(T) * std::max<size_t>(n, 1));
    if (e != hipSuccess) return e;
    if (n) e = hipMemcpyAsync(ctx->buf[id].p, src, sizeof(T) * n, hipMemcpyHostToDevice, ctx->stream);
    return e;
}

// Host-side all-reduce of a small array across the landmark shards (prepare time).
template <class T>
static int host_allreduce(ba_context* ctx, T* v, size_t n, CommOp op) {
    if (!ctx->W.comm.on() || n == 0) return BA_OK;
    if (ctx->buf[B_PREP].ensure(sizeof(T) * n) != hipSuccess) { ctx->err = "prepare scratch allocation failed"; return BA_E_NOMEM; }
    T* d = ctx->buf[B_PREP].as<T>();
    hipStream_t s = ctx->stream;
    const CommType t = sizeof(T) == 8 ? COMM_F64 : COMM_I32;
    if (hipMemcpyAsync(d, v, sizeof(T) * n, hipMemcpyHostToDevice, s) != hipSuccess ||
        comm_allreduce(ctx->W.comm, d, d, n, t, op, s) != hipSuccess ||
        hipMemcpyAsync(v, d, sizeof(T) * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        ctx->err = std::string("landmark-shard all-reduce failed: ") + comm_last_error();
        return BA_E_COMM;
    }
    return BA_OK;
}
static int host_allreduce_i32(ba_context* ctx, int* v, size_t n, CommOp op) { return host_allreduce(ctx, v, n, op); }

extern "C" {

int32_t ba_api_version(void) { return BA_API_VERSION; }

const char* ba_build_info(void) {
    return "libmiba " __DATE__ " gfx950 f64; kernels: cam_side/point_prep/obs_pairs(atomic)/chol(env,mfma_f64_16x16x4)/"
           "backsub_eval";
}

void ba_default_options(ba_options* o) {
    std::memset(o, 0, sizeof(*o));
    o->hub_p_repr = 1e-3;         // BundleAdjustmentConfig.h:47
    o->hub_p_unpr = 1e-3;         // :50
    o->weight_intrinsics = 1e-6;  // :48
    o->weight_unpr = 10.0;        // :49
    o->max_num_iterations = 75;   // :64
    o->minimizer_progress_to_stdout = 1;  // :63
    o->eta = 1e-6;                // :65
    o->initial_trust_region_radius = 1e4;  // Ceres 2.0 defaults below
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
    o->deterministic = 0;
    o->shard_min_obs = 262144;
    o->small_window = 0;          // ignored (the single-workgroup small-window kernel was removed)
}

ba_context* ba_create(const ba_options* opts) {
    ba_context* ctx = new ba_context();
    if (opts) ctx->opts = *opts; else ba_default_options(&ctx->opts);
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) {
        g_err = std::string("no HIP device available: ") + hipGetErrorString(e);
        delete ctx;
        return nullptr;
    }
    if (ctx->opts.device >= 0) {
        if (ctx->opts.device >= ndev) {
            g_err = "device ordinal out of range";
            delete ctx;
            return nullptr;
        }
        ctx->device = ctx->opts.device;
        e = hipSetDevice(ctx->device);
    } else {
        e = hipGetDevice(&ctx->device);
    }
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    for (int i = 0; i < 5 && e == hipSuccess; ++i) e = hipEventCreate(&ctx->ev[i]);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_idx, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ctx->ev_uv, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc((void**)&ctx->hprog, PROG_BYTES, hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) e = hipHostGetDevicePointer((void**)&ctx->dprog, ctx->hprog, 0);
    if (ctx->opts.profile_kernels) {
        for (int i = 0; i < 2 * Prof::MAXP && e == hipSuccess; ++i) e = hipEventCreate(&ctx->prof.ev[i]);
        ctx->prof_events = (e == hipSuccess);
        ctx->prof.on = 1;
        ctx->prof.mask = (unsigned)ctx->opts.profile_mask;
    }
    if (e != hipSuccess) {
        g_err = std::string("HIP init failed: ") + hipGetErrorString(e);
        delete ctx;
        return nullptr;
    }
    return ctx;
}

void ba_destroy(ba_context* ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    if (ctx->stream) hipStreamSynchronize(ctx->stream);
    // a prepare that returned early (e.g. BA_E_INVALID) may have left value copies queued on the copy stream:
    // they read the staging buffer and write device buffers released below
    if (ctx->copy_stream) hipStreamSynchronize(ctx->copy_stream);
    comm_destroy(ctx->W.comm);
    comm_destroy(ctx->comm_parked);
    for (auto& b : ctx->buf) b.release();
    for (auto& e : ctx->ev)
        if (e) hipEventDestroy(e);
    if (ctx->prof_events)
        for (int i = 0; i < 2 * Prof::MAXP; ++i) hipEventDestroy(ctx->prof.ev[i]);
    if (ctx->hprog) hipHostFree(ctx->hprog);
    if (ctx->hres) hipHostFree(ctx->hres);
    if (ctx->stage) hipHostFree(ctx->stage);
    if (ctx->pstage) hipHostFree(ctx->pstage);
    if (ctx->rsum) hipHostFree(ctx->rsum);
    if (ctx->copy_stream) {
        hipStreamSynchronize(ctx->copy_stream);
        hipStreamDestroy(ctx->copy_stream);
    }
    if (ctx->ev_idx) hipEventDestroy(ctx->ev_idx);
    if (ctx->ev_uv) hipEventDestroy(ctx->ev_uv);
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* ba_last_error(const ba_context* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int32_t ba_comm_unique_id(uint8_t id[BA_COMM_ID_BYTES]) {
    if (!id) { g_err = "null id buffer"; return BA_E_INVALID; }
    if (comm_unique_id(id, BA_COMM_ID_BYTES) != 0) {
        g_err = comm_last_error();
        return BA_E_COMM;
    }
    return BA_OK;
}

int32_t ba_comm_init(ba_context* ctx, int32_t nranks, int32_t rank, const uint8_t id[BA_COMM_ID_BYTES]) {
    if (!ctx || !id) return BA_E_INVALID;
    if (hipSetDevice(ctx->device) != hipSuccess) { ctx->err = "hipSetDevice failed"; return BA_E_DEVICE; }
    comm_destroy(ctx->comm_parked);
    if (comm_init(ctx->W.comm, nranks, rank, id) != 0) {
        ctx->err = comm_last_error();
        return nranks < 1 || rank < 0 || rank >= nranks ? BA_E_INVALID : BA_E_COMM;
    }
    ctx->prepared = false;  // the next solve re-prepares with the shard-global structure
    return BA_OK;
}

int32_t ba_comm_init_host(ba_context* ctx, int32_t nranks, int32_t rank, ba_allreduce_fn fn, void* user) {
    if (!ctx) return BA_E_INVALID;
    comm_destroy(ctx->comm_parked);
    if (comm_init_host(ctx->W.comm, nranks, rank, fn, user) != 0) {
        ctx->err = comm_last_error();
        return BA_E_INVALID;
    }
    ctx->prepared = false;  // the next solve re-prepares with the shard-global structure
    return BA_OK;
}

int32_t ba_iteration_log(const ba_context* ctx, double* rows, int32_t max_rows) {
    if (!ctx || ctx->last_iter < 0 || !ctx->W.log) return 0;
    const int n = ctx->last_iter + 1;
    if (rows && max_rows > 0) {
        const int m = std::min(n, (int)max_rows);
        if (hipSetDevice(ctx->device) != hipSuccess ||
            hipMemcpy(rows, ctx->W.log, sizeof(double) * LOG_W * m, hipMemcpyDeviceToHost) != hipSuccess)
            return 0;
        for (int i = 0; i < m; ++i) rows[(size_t)i * LOG_W + 7] = 0.0;
    }
    return n;
}

int32_t ba_set_options(ba_context* ctx, const ba_options* opts) {
    if (!ctx || !opts) return BA_E_INVALID;
    if (opts->device >= 0 && opts->device != ctx->device) {
        ctx->err = "ba_set_options cannot move a context to another device";
        return BA_E_INVALID;
    }
    const int dev = ctx->device;
    ctx->opts = *opts;
    ctx->opts.device = dev;
    if (ctx->opts.profile_kernels && !ctx->prof_events) {
        hipError_t e = hipSuccess;
        for (int i = 0; i < 2 * Prof::MAXP && e == hipSuccess; ++i) e = hipEventCreate(&ctx->prof.ev[i]);
        if (e != hipSuccess) { ctx->err = "event creation failed"; return BA_E_DEVICE; }
        ctx->prof_events = true;
    }
    ctx->prof.on = ctx->opts.profile_kernels ? 1 : 0;
    ctx->prof.mask = (unsigned)ctx->opts.profile_mask;
    return BA_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Problem preparation: admissibility (countConstraints :184-213, skip :265-268),
// active parameter blocks, point-major / camera-major orderings, envelope of S.
static int prepare_core(ba_context* ctx, const ba_problem* p, bool force_det);

// Landmark shards of a window too small to pay for the per-iteration exchange (admissible observations
// over all shards < ba_options.shard_min_obs): gather every shard onto every rank (SUM all-reduces of
// zero-padded slices, once per ba_prepare) and solve the whole window on each rank without collectives,
// in deterministic mode so that all ranks compute bitwise the same cameras; each rank keeps its slice.
// Returns 1 when the window was prepared gathered, 0 when it stays sharded, < 0 on error.
static int prepare_gathered(ba_context* ctx, const ba_problem* p) {
    Comm& comm = ctx->W.comm;
    const int R = comm.nranks, me = comm.rank;
    // agreement first (every rank reaches the same branch): local validity and admissible count
    int v[2] = {0, 0};
    bool ok = p && p->n_cams >= 0 && p->n_points >= 0 && p->n_obs >= 0 && p->intr && p->intr_prior &&
              (!p->n_cams || p->cams) && (!p->n_points || p->points) &&
              (!p->n_obs || (p->obs_cam && p->obs_pt && p->obs_uv && p->obs_depth));
    for (int k = 0; ok && k < p->n_obs; ++k) {
        if (p->obs_cam[k] < 0 || p->obs_cam[k] >= p->n_cams || p->obs_pt[k] < 0 || p->obs_pt[k] >= p->n_points) ok = false;
        else if (p->obs_depth[k] > 1e-15) ++v[1];
    }
    v[0] = ok ? 0 : 1;
    if (int rc = host_allreduce_i32(ctx, v, 2, COMM_SUM)) return rc;
    if (v[0] != 0 || v[1] >= ctx->opts.shard_min_obs) return 0;  // invalid (prepare_core reports it) or large
    std::vector<int> cnt(2 * (size_t)R, 0);
    cnt[2 * me] = p->n_points;
    cnt[2 * me + 1] = p->n_obs;
    if (int rc = host_allreduce_i32(ctx, cnt.data(), cnt.size(), COMM_SUM)) return rc;
    int np = 0, no = 0, poff = 0, ooff = 0;
    for (int r = 0; r < R; ++r) {
        if (r == me) { poff = np; ooff = no; }
        np += cnt[2 * r];
        no += cnt[2 * r + 1];
    }
    auto& g = ctx->gw;
    g.cams.assign(p->cams, p->cams + 7 * (size_t)p->n_cams);  // replicated on every rank
    std::memcpy(g.intr, p->intr, sizeof(g.intr));
    std::memcpy(g.prior, p->intr_prior, sizeof(g.prior));
    g.pts.assign(3 * (size_t)np, 0.0);
    g.uv.assign(2 * (size_t)no, 0.0);
    g.dep.assign(no, 0.0);
    g.oc.assign(no, 0);
    g.op.assign(no, 0);
    std::copy(p->points, p->points + 3 * (size_t)p->n_points, g.pts.begin() + 3 * (size_t)poff);
    std::copy(p->obs_uv, p->obs_uv + 2 * (size_t)p->n_obs, g.uv.begin() + 2 * (size_t)ooff);
    std::copy(p->obs_depth, p->obs_depth + p->n_obs, g.dep.begin() + ooff);
    std::copy(p->obs_cam, p->obs_cam + p->n_obs, g.oc.begin() + ooff);
    for (int k = 0; k < p->n_obs; ++k) g.op[ooff + k] = p->obs_pt[k] + poff;
    int rc = host_allreduce(ctx, g.pts.data(), g.pts.size(), COMM_SUM);
    if (!rc) rc = host_allreduce(ctx, g.uv.data(), g.uv.size(), COMM_SUM);
    if (!rc) rc = host_allreduce(ctx, g.dep.data(), g.dep.size(), COMM_SUM);
    if (!rc) rc = host_allreduce_i32(ctx, g.oc.data(), g.oc.size(), COMM_SUM);
    if (!rc) rc = host_allreduce_i32(ctx, g.op.data(), g.op.size(), COMM_SUM);
    if (rc) return rc;
    ba_problem full{};
    full.n_cams = p->n_cams;
    full.n_points = np;
    full.n_obs = no;
    full.fixed_cam = p->fixed_cam;
    full.cams = g.cams.data();
    full.points = g.pts.data();
    full.intr = g.intr;
    full.intr_prior = g.prior;
    full.obs_cam = g.oc.data();
    full.obs_pt = g.op.data();
    full.obs_uv = g.uv.data();
    full.obs_depth = g.dep.data();
    ctx->comm_parked = comm;  // no collective while this window is solved
    comm = Comm{};
    rc = prepare_core(ctx, &full, true);
    if (rc) return rc;
    ctx->gather_off = poff;
    ctx->dev_np = np;
    ctx->prep_nc = p->n_cams; ctx->prep_np = p->n_points; ctx->prep_no = p->n_obs;  // the caller's shard
    return 1;
}

// Landmark shards replicate the window's cameras, intrinsics, prior and gauge: every rank must pass the same
// values (each would otherwise solve a different window and still report success). FNV-1a over their bytes,
// MIN and MAX all-reduced: a mismatch anywhere gives every rank the same BA_E_INVALID.
static int shard_replicas_agree(ba_context* ctx, const ba_problem* p) {
    unsigned long long h = 1469598103934665603ull;
    auto mix = [&](const void* d, size_t n) {
        const unsigned char* b = static_cast<const unsigned char*>(d);
        for (size_t k = 0; k < n; ++k) h = (h ^ b[k]) * 1099511628211ull;
    };
    const bool ok = p && p->n_cams >= 0 && (!p->n_cams || p->cams) && p->intr && p->intr_prior;
    if (ok) {
        mix(&p->n_cams, sizeof(p->n_cams));
        mix(&p->fixed_cam, sizeof(p->fixed_cam));
        mix(p->cams, sizeof(double) * 7 * (size_t)p->n_cams);
        mix(p->intr, sizeof(double) * 4);
        mix(p->intr_prior, sizeof(double) * 4);
    }
    int lo[2] = {(int)(unsigned)h, (int)(unsigned)(h >> 32)}, hi[2] = {lo[0], lo[1]};
    int rc = host_allreduce_i32(ctx, lo, 2, COMM_MIN);
    if (rc == BA_OK) rc = host_allreduce_i32(ctx, hi, 2, COMM_MAX);
    if (rc != BA_OK) return rc;
    if (lo[0] != hi[0] || lo[1] != hi[1]) {
        ctx->err = "landmark shards disagree on the window cameras / intrinsics / prior / fixed_cam (every rank must "
                   "pass the same replicated values)";
        return BA_E_INVALID;
    }
    return BA_OK;
}

static int prepare(ba_context* ctx, const ba_problem* p) {
    if (ctx->comm_parked.on()) {  // the last window ran gathered: the communicator is back for this one
        ctx->W.comm = ctx->comm_parked;
        ctx->comm_parked = Comm{};
    }
    ctx->gather_off = 0;
    ctx->dev_np = p && p->n_points > 0 ? p->n_points : 0;
    if (ctx->W.comm.on())
        if (int rc = shard_replicas_agree(ctx, p)) return rc;
    if (ctx->W.comm.on() && ctx->opts.shard_min_obs > 0) {
        const int rc = prepare_gathered(ctx, p);
        if (rc != 0) return rc < 0 ? rc : BA_OK;
    }
    return prepare_core(ctx, p, false);
}

static size_t bcr_bytes(int nblk) {
    return sizeof(double) * ((BCR_BLOCK_DOUBLES + 64 * 64) * nblk + 16) + sizeof(unsigned) * (16 + 6 * nblk);
}

// k_bcr_split's hand-off state: the flags (epoch 0) and the flag-free buffers, which start empty (BCR_Y_EMPTY):
// y (Racc | Y, epoch parity), the published panels (Cf | X slots, two epochs) and the published X rows of the
// pull hand-off (bcr_reset_pull_slots: zeros instead when another BCR path runs)
static int bcr_init_handoffs(ba_context* ctx) {
    const BcrWork& Bw = ctx->W.bcr;
    const size_t b64 = (size_t)64 * 64 * Bw.nblk, b8 = (size_t)64 * 8 * Bw.nblk;
    hipStream_t s = ctx->stream;
    HIPCHECK(ctx, hipMemsetAsync(Bw.flags, 0, sizeof(unsigned) * (16 + 6 * Bw.nblk), s));
    HIPCHECK(ctx, hipMemsetD32Async((hipDeviceptr_t)Bw.Racc, BCR_Y_EMPTY_D32, 4 * b8, s));
    HIPCHECK(ctx, hipMemsetD32Async((hipDeviceptr_t)Bw.Cf, BCR_Y_EMPTY_D32, 2 * (b64 + (size_t)64 * BCR_XW * Bw.nblk), s));
    HIPCHECK(ctx, bcr_reset_pull_slots(Bw, Bw.persist >= 2, s));
    ctx->bcr_launches = 0;
    return BA_OK;
}

// Pinned host staging of ba_prepare's uploads (grown on demand, kept by the context): the raw window is copied
// in by the host threads and DMA'd while the plan is built; the plan's index arrays follow in one DMA. Growing
// keeps the first `keep` bytes (the raw region, which the plan cache compares the next window against).
static int stage_ensure(ba_context* ctx, size_t bytes, size_t keep) {
    if (ctx->stage_cap >= bytes) return BA_OK;
    const size_t want = std::max<size_t>(bytes + bytes / 8, 1 << 20);
    char* nb = nullptr;
    HIPCHECK(ctx, hipHostMalloc((void**)&nb, want, hipHostMallocDefault));
    if (ctx->stage) {
        if (keep) std::memcpy(nb, ctx->stage, std::min(keep, ctx->stage_cap));
        HIPCHECK(ctx, hipHostFree(ctx->stage));
    }
    ctx->stage = nb;
    ctx->stage_cap = want;
    return BA_OK;
}

// parallel memcpy (the host pool) of several arrays into the staging buffer
struct StageCopy { void* dst; const void* src; size_t bytes; };
static void stage_copy(const std::vector<StageCopy>& v) {
    size_t total = 0;
    for (const StageCopy& c : v) total += c.bytes;
    const int T = (int)std::max<size_t>(1, std::min<size_t>(4 * (size_t)host_threads(), total >> 18));
    host_parallel(T, [&](int t) {
        for (const StageCopy& c : v) {
            const size_t lo = c.bytes * t / T, hi = c.bytes * (t + 1) / T;
            if (hi > lo) std::memcpy(static_cast<char*>(c.dst) + lo, static_cast<const char*>(c.src) + lo, hi - lo);
        }
    });
}

// The pixels into the staging buffer (host pool), checking on the way that every admissible pixel and depth is
// exactly an f32 (the obs32 layout, DevProblem::obs32; plan_count's check for the device plan). Returns true when
// one is not.
static bool stage_values_f32check(double* dst_uv, double* dst_dep, const double* uv, const double* dep, size_t no) {
    const int T = (int)std::max<size_t>(1, std::min<size_t>(4 * (size_t)host_threads(), no >> 12));
    std::vector<unsigned char> bad(T, 0);
    auto f32_exact = [](double v) { return (double)(float)v == v; };
    host_parallel(T, [&](int t) {
        const size_t lo = no * t / T, hi = no * (t + 1) / T;
        std::memcpy(dst_uv + 2 * lo, uv + 2 * lo, 16 * (hi - lo));
        std::memcpy(dst_dep + lo, dep + lo, 8 * (hi - lo));
        bool ok = true;
        for (size_t k = lo; k < hi; ++k)
            if (dep[k] > 1e-15) ok = ok && f32_exact(uv[2 * k]) && f32_exact(uv[2 * k + 1]) && f32_exact(dep[k]);
        bad[t] = ok ? 0 : 1;
    });
    for (int t = 0; t < T; ++t)
        if (bad[t]) return true;
    return false;
}

// The staging layout of the raw observations: obs_uv | obs_depth | obs_cam | obs_pt.
// (+ the admissibility bytes the device plan reads instead of the depths)
struct RawStage {
    double* uv; double* dep; int* cam; int* pt; unsigned char* adm;
    RawStage(char* sg, size_t no)
        : uv(reinterpret_cast<double*>(sg)), dep(uv + 2 * no), cam(reinterpret_cast<int*>(dep + no)), pt(cam + no),
          adm(reinterpret_cast<unsigned char*>(pt + no)) {}
};
static size_t raw_stage_bytes(size_t no) { return no * (16 + 8 + 4 + 4 + 1); }

// The device plan's inputs into the staging buffer (host pool): the indices and one admissibility byte per
// observation (depth > 1e-15, countConstraints / the skip at OptimizationUtils.cpp:265-268).
static void stage_indices_adm(const RawStage& rs, const ba_problem* p, size_t no) {
    const int T = (int)std::max<size_t>(1, std::min<size_t>(4 * (size_t)host_threads(), no >> 15));
    host_parallel(T, [&](int t) {
        const size_t lo = no * t / T, hi = no * (t + 1) / T;
        std::memcpy(rs.cam + lo, p->obs_cam + lo, 4 * (hi - lo));
        std::memcpy(rs.pt + lo, p->obs_pt + lo, 4 * (hi - lo));
        for (size_t k = lo; k < hi; ++k) rs.adm[k] = p->obs_depth[k] > 1e-15 ? 1 : 0;
    });
}

// The window's parameters (cameras, points, intrinsics, prior) -> pinned staging -> HBM slot 0, then copied on the
// device into the candidate and initial slots (k_reset starts every solve from the initial ones).
static int upload_params(ba_context* ctx, const ba_problem* p, hipStream_t s) {
    const size_t nc = p->n_cams, np = p->n_points;
    const size_t bytes = 56 * nc + 24 * np + 64;
    if (ctx->pstage_cap < bytes) {
        if (ctx->pstage) HIPCHECK(ctx, hipHostFree(ctx->pstage));
        ctx->pstage = nullptr;
        ctx->pstage_cap = 0;
        const size_t want = std::max<size_t>(bytes + bytes / 8, 1 << 16);
        HIPCHECK(ctx, hipHostMalloc((void**)&ctx->pstage, want, hipHostMallocDefault));
        ctx->pstage_cap = want;
    }
    double* hc = reinterpret_cast<double*>(ctx->pstage);
    double* hp = hc + 7 * nc;
    double* hk = hp + 3 * np;
    std::vector<StageCopy> cp = {{hk, p->intr, 32}, {hk + 4, p->intr_prior, 32}};
    if (nc) cp.push_back({hc, p->cams, 56 * nc});
    if (np) cp.push_back({hp, p->points, 24 * np});
    stage_copy(cp);
    const int slots[3][3] = {{B_CAMS0, B_CAMS1, B_CAMS_INIT}, {B_PTS0, B_PTS1, B_PTS_INIT}, {B_K0, B_K1, B_K_INIT}};
    const size_t len[3] = {56 * nc, 24 * np, 32};
    const double* src[3] = {hc, hp, hk};
    for (int a = 0; a < 3; ++a) {
        for (int b = 0; b < 3; ++b) HIPCHECK(ctx, ctx->buf[slots[a][b]].ensure(std::max<size_t>(len[a], 8)));
        if (!len[a]) continue;
        HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[slots[a][0]].p, src[a], len[a], hipMemcpyHostToDevice, s));
        for (int b = 1; b < 3; ++b)
            HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[slots[a][b]].p, ctx->buf[slots[a][0]].p, len[a], hipMemcpyDeviceToDevice, s));
    }
    HIPCHECK(ctx, ctx->buf[B_PRIOR].ensure(32));
    HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[B_PRIOR].p, hk + 4, 32, hipMemcpyHostToDevice, s));
    return BA_OK;
}

// The band tail's flag-free partial slots (PART_TAIL, ba_kernels.h) start empty: the BCR_Y_EMPTY pattern in every
// double (its two 32-bit halves are equal, so one 32-bit fill)
static hipError_t empty_tail_slots(double* part, int stride, hipStream_t s) {
    static_assert((BCR_Y_EMPTY >> 32) == (BCR_Y_EMPTY & 0xffffffffull), "a 32-bit fill writes the pattern");
    return hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(part + (size_t)PART_TAIL * stride), (int)BCR_Y_EMPTY_D32,
                             2 * 5 * (size_t)stride, s);
}

// The MIBA_* settings ba_prepare reads (layout / solver choices): part of the plan cache key.
static unsigned long long env_key() {
    static const char* const names[] = {"MIBA_OBS32", "MIBA_TILE_PTS", "MIBA_SUBSEG", "MIBA_SOLVER", "MIBA_DENSE_CHOL",
                                        "MIBA_BCR", "MIBA_XCD_MAP", "MIBA_FUSED", "MIBA_SW", "MIBA_FPL",
                                        "MIBA_BCR_DENSE1", "MIBA_PP_LANES", "MIBA_DEVICE_PLAN", "MIBA_TAIL",
                                        "MIBA_BCR_BAND", "MIBA_BCR_XMAP"};
    unsigned long long h = 1469598103934665603ull;
    for (const char* n : names) {
        const char* v = std::getenv(n);
        const std::string t = std::string(n) + (v ? std::string("=") + v : std::string("\x01"));
        for (unsigned char c : t) h = (h ^ c) * 1099511628211ull;
    }
    return h;
}

// The block cyclic reduction's workspace: zeroed (the upper tiles of UL / UR are never written and must read as
// zero), the resident path probed (bcr_persist_ok; MIBA_BCR overrides), the hand-off state initialised. Every
// full prepare probes again, also after a hand-off timeout moved the last window to the per-level launches
// (ba_prepare_info.bcr_path reports the path).
// ba_prepare_info.bcr_path of the reduced-solve path (include/ba.h)
static int bcr_path_id(const BcrWork& Bw) { return Bw.band ? 5 : Bw.dense1 ? 4 : Bw.persist; }

static int bcr_setup(ba_context* ctx) {
    BcrWork& Bw = ctx->W.bcr;
    HIPCHECK(ctx, hipMemsetAsync(ctx->buf[B_BCR].p, 0, ctx->buf[B_BCR].cap, ctx->stream));
    Bw.persist = bcr_persist_ok(Bw.nblk);
    Bw.dense1 = bcr_dense1_ok(Bw.nblk, ctx->P.kb);
    Bw.band = bcr_band_ok(ctx->P.nac, ctx->P.cam_band, ctx->P.kb, ctx->tail_possible);
    if (const char* e = std::getenv("MIBA_BCR")) {
        if (!std::strcmp(e, "launch")) Bw.persist = 0;
        else if (!std::strcmp(e, "persist") && Bw.persist >= 2) Bw.persist = 1;
        else if (!std::strcmp(e, "split") && Bw.persist == 3) Bw.persist = 2;  // "split3" or unset: default
    }
    Bw.xmap = bcr_xmap_ok(Bw.nblk, Bw.persist);
    ctx->bcr_fallback = false;
    return bcr_init_handoffs(ctx);
}

// The cost constants of the window (weights, Huber scales, LM diagonal bounds) from the context's options and N.
// Every prepare sets them, the plan-cache reuse path included: ba_set_options may change a weight or a Huber
// scale between two solves of one window structure.
static void set_consts(ba_context* ctx) {
    const ba_options& o = ctx->opts;
    BaConsts& C = ctx->C;
    // all shards' admissible observations (N = 0: no observation block exists, so the 1/N weights are unused
    // and the window reduces to the IntrinsicsPrior block, :236-241)
    const double N = (double)std::max(ctx->n_adm_all, 1);
    C.sw_r = std::sqrt(1.0 / N);             // ReprojectionConstraint weight 1/N (:280)
    C.sw_d = std::sqrt(o.weight_unpr / N);   // DepthPrior WEIGHT_UNPR/N (:290)
    C.sw_k = std::sqrt(o.weight_intrinsics); // IntrinsicsPrior (:238)
    C.a_r = o.hub_p_repr; C.b_r = o.hub_p_repr * o.hub_p_repr;
    C.a_d = o.hub_p_unpr; C.b_d = o.hub_p_unpr * o.hub_p_unpr;
    C.min_diag = o.min_lm_diagonal; C.max_diag = o.max_lm_diagonal;
}

// Plan cache: the window has the structure of the last full prepare (sizes, gauge, deterministic option and layout
// settings in the key; obs_cam, obs_pt and the admissibility mask compared here, on the host threads, against the
// staged copy of that window) -> only the parameters, and the observation values that changed, are uploaded.
// An admissible value that is no longer an exact f32 on an obs32 plan also forces a rebuild.
// Returns 1 when the plan was reused, 0 when the window needs a full prepare, < 0 on error.
static int prepare_reuse(ba_context* ctx, const ba_problem* p, double tp0) {
    const int no = p->n_obs;
    RawStage rs(ctx->stage, (size_t)no);
    const bool o32 = ctx->key.obs32 != 0;
    const int T = (int)std::max<long long>(1, std::min<long long>(4LL * host_threads(), (long long)no >> 15));
    std::vector<unsigned char> changed(T, 0), vals(T, 0);
    auto f32_exact = [](double v) { return (double)(float)v == v; };
    host_parallel(T, [&](int t) {
        const size_t lo = (size_t)no * t / T, hi = (size_t)no * (t + 1) / T, n = hi - lo;
        if (!n) return;
        if (std::memcmp(rs.cam + lo, p->obs_cam + lo, 4 * n) || std::memcmp(rs.pt + lo, p->obs_pt + lo, 4 * n)) {
            changed[t] = 1;
            return;
        }
        if (std::memcmp(rs.dep + lo, p->obs_depth + lo, 8 * n)) {
            for (size_t k = lo; k < hi; ++k) {
                const double nd = p->obs_depth[k];
                const bool adm = nd > 1e-15;
                if (adm != (rs.dep[k] > 1e-15) || (adm && o32 && !f32_exact(nd))) { changed[t] = 1; return; }
            }
            std::memcpy(rs.dep + lo, p->obs_depth + lo, 8 * n);
            vals[t] = 1;
        }
        if (std::memcmp(rs.uv + 2 * lo, p->obs_uv + 2 * lo, 16 * n)) {
            if (o32)
                for (size_t k = lo; k < hi; ++k)
                    if (p->obs_depth[k] > 1e-15 && !(f32_exact(p->obs_uv[2 * k]) && f32_exact(p->obs_uv[2 * k + 1]))) {
                        changed[t] = 1;
                        return;
                    }
            std::memcpy(rs.uv + 2 * lo, p->obs_uv + 2 * lo, 16 * n);
            vals[t] = 1;
        }
    });
    ctx->pinfo.compare_ms = now_ms() - tp0;
    for (int t = 0; t < T; ++t)
        if (changed[t]) return 0;
    const double tu = now_ms();
    hipStream_t s = ctx->stream;
    bool any_vals = false;
    for (int t = 0; t < T; ++t) any_vals = any_vals || vals[t];
    if (any_vals) {  // new pixel / depth values on the same structure: re-gather the observation layouts
        HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[B_RAW_UV].p, rs.uv, 16 * (size_t)no, hipMemcpyHostToDevice, s));
        HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[B_RAW_DEP].p, rs.dep, 8 * (size_t)no, hipMemcpyHostToDevice, s));
        HIPCHECK(ctx, launch_prep_gather(ctx->P, ctx->raw, s));
    }
    if (int rc = upload_params(ctx, p, s)) return rc;
    // the same device state as after a full prepare: S, rhs and the partial slots cleared
    const DevProblem& P = ctx->P;
    HIPCHECK(ctx, hipMemsetAsync(ctx->buf[B_S].p, 0, sizeof(double) * (size_t)P.npad * P.npad, s));
    HIPCHECK(ctx, hipMemsetAsync(ctx->buf[B_RHS].p, 0, sizeof(double) * P.npad, s));
    HIPCHECK(ctx, hipMemsetAsync(ctx->buf[B_PART].p, 0, sizeof(double) * PART_NSLOTS * P.part_stride, s));
    HIPCHECK(ctx, empty_tail_slots(ctx->buf[B_PART].as<double>(), P.part_stride, s));
    if (P.solver == 2 && ctx->bcr_fallback)
        if (int rc = bcr_setup(ctx)) return rc;
    // a hand-off timeout cleared the small-window launch for the rest of that solve: the next one takes the path
    // the full prepare chose again (no sticky fallback)
    ctx->W.sw = ctx->sw_full;
    ctx->W.tail = ctx->tail_full;
    ctx->W.bsfin = ctx->bsfin_full;
    set_consts(ctx);
    ctx->pinfo.plan_reused = 1;
    ctx->pinfo.obs_uploaded = any_vals ? 1 : 0;
    ctx->pinfo.upload_ms = now_ms() - tu;
    ctx->pinfo.bcr_path = P.solver == 2 ? bcr_path_id(ctx->W.bcr) : -1;
    ctx->pinfo.lin_path = ctx->W.sw;
    ctx->pinfo.tail = ctx->W.tail;
    ctx->pinfo.bsfin = ctx->W.bsfin;
    ctx->prepared = true;
    ctx->prep_nc = p->n_cams; ctx->prep_np = p->n_points; ctx->prep_no = p->n_obs;
    return 1;
}

// The plan's tiling / chunking parameters (n_adm: this shard's admissible observations).
static PlanParams plan_params(int n_adm) {
    PlanParams pp;
    pp.tile_win = TILE_WIN;
    pp.chunk_pts = CHUNK_PTS;
    pp.chunk_obs = CHUNK_OBS;
    pp.tile_slots = schur_tile_slots();
    if (const char* e = std::getenv("MIBA_TILE_PTS")) pp.tile_pts_env = std::max(1, std::atoi(e));
    pp.bs_pts = BS_PTS;
    pp.bs_obs = BS_OBS;
    // sub-segment size: ~6.5 observations per thread on large windows (C4 rocprof, fused linearisation:
    // 34.2 us at 1700 vs 36.1 at 1024, 42.7 at 512, 34.7 at 2500); MIBA_SUBSEG overrides (tuning)
    // and 256 on windows of a few thousand observations (C1's camera side in its Schur launch: shorter per-thread
    // chains, with the half-chunk tiles -2.4 % per LM iteration; neutral at C3's 8k, which keeps 1024)
    pp.subseg = n_adm >= 200000 ? SUBSEG_OBS_LARGE : n_adm < 4096 ? SUBSEG_OBS_SMALL : SUBSEG_OBS;
    if (const char* e = std::getenv("MIBA_SUBSEG")) pp.subseg = std::max(64, std::atoi(e));
    return pp;
}

// MIBA_DEVICE_PLAN: 0 = the host plan; 1 = the device plan whenever the window fits it; unset = the device plan on
// windows of >= DPLAN_MIN_OBS observations (prepare, host vs device plan: C1, 1.6k observations, 0.15 vs 0.21 ms;
// C3, 8k, 0.26 vs 0.23-0.37; C2, 50k, 0.87 vs 0.31-0.34; C4, 1M, 2.8 vs 1.3-1.5)
static constexpr int DPLAN_MIN_OBS = 16384;
// windows from which a helper thread builds the host side of the plan while the values are staged (below, the
// thread costs more than the overlap saves)
static constexpr int DPLAN_HELPER_OBS = 262144;
static bool want_dplan(int nc, int np, int no) {
    const char* e = std::getenv("MIBA_DEVICE_PLAN");
    if (e && e[0] == '0') return false;
    if (!dplan_fits(no, np, nc)) return false;
    return (e && e[0] == '1') || no >= DPLAN_MIN_OBS;
}

// The device plan's prepare: the indices and admissibility bytes staged and DMA'd first; the plan's passes
// enqueued behind them (the last one writes the summary into mapped host memory, no DMA engine involved); the
// depths, pixels (obs32 checked on the way) and parameters staged meanwhile and DMA'd on the copy stream; then one
// wait for the passes. ok = false: a point list longer than the device sort takes, or a scan that did not settle
// (the host plan builds the window instead; the staged upload stands).
static int run_dplan(ba_context* ctx, const ba_problem* p, int nc, int np, int no, bool& notf32, bool& ok,
                     bool& built) {
    hipStream_t s = ctx->stream;
    built = false;
    const bool times = std::getenv("MIBA_PLAN_TIMES") != nullptr;  // diagnostic: host phases of the device plan
    double tm = now_ms();
    auto mark = [&](const char* what) {
        if (!times) return;
        const double t = now_ms();
        std::fprintf(stderr, "dplan %s %.3f ms\n", what, t - tm);
        tm = t;
    };
    if (ctx->uv_pending) {  // a prepare that failed after its value DMA: the staging buffer is still read
        HIPCHECK(ctx, hipEventSynchronize(ctx->ev_uv));
        ctx->uv_pending = false;
    }
    if (int rc = stage_ensure(ctx, raw_stage_bytes((size_t)no), 0)) return rc;
    RawStage rs(ctx->stage, (size_t)no);
    HIPCHECK(ctx, ctx->buf[B_RAW_UV].ensure(16 * (size_t)no));
    HIPCHECK(ctx, ctx->buf[B_RAW_DEP].ensure(8 * (size_t)no));
    HIPCHECK(ctx, ctx->buf[B_RAW_CAM].ensure(4 * (size_t)no));
    HIPCHECK(ctx, ctx->buf[B_RAW_PT].ensure(4 * (size_t)no));
    HIPCHECK(ctx, ctx->buf[B_RAW_ADM].ensure((size_t)no));
    mark("buffers");
    stage_indices_adm(rs, p, (size_t)no);
    mark("stage_indices");
    HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[B_RAW_CAM].p, rs.cam, 4 * (size_t)no, hipMemcpyHostToDevice, s));
    HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[B_RAW_PT].p, rs.pt, 4 * (size_t)no, hipMemcpyHostToDevice, s));
    HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[B_RAW_ADM].p, rs.adm, (size_t)no, hipMemcpyHostToDevice, s));
    HIPCHECK(ctx, hipEventRecord(ctx->ev_idx, s));
    const size_t nsum = dplan_sum_ints(nc, np);
    HIPCHECK(ctx, ctx->buf[B_DP_SCRATCH].ensure(4 * dplan_scratch_ints(no, np, nc)));
    HIPCHECK(ctx, ctx->buf[B_DP_PO_DEST].ensure(4 * (size_t)no));
    HIPCHECK(ctx, ctx->buf[B_DP_CO_DEST].ensure(4 * (size_t)no));
    HIPCHECK(ctx, ctx->buf[B_DP_CAM_AC].ensure(4 * (size_t)nc));
    HIPCHECK(ctx, ctx->buf[B_DP_PT_IDX].ensure(4 * (size_t)np));
    HIPCHECK(ctx, ctx->buf[B_DP_OVF].ensure(4 * (size_t)no));
    HIPCHECK(ctx, ctx->buf[B_DP_SUM].ensure(4 * nsum));
    if (ctx->rsum_cap < nsum) {
        if (ctx->rsum) HIPCHECK(ctx, hipHostFree(ctx->rsum));
        ctx->rsum = nullptr;
        ctx->rsum_dev = nullptr;
        ctx->rsum_cap = 0;
        const size_t want = nsum + nsum / 8 + 64;
        HIPCHECK(ctx, hipHostMalloc((void**)&ctx->rsum, 4 * want, hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHECK(ctx, hipHostGetDevicePointer((void**)&ctx->rsum_dev, ctx->rsum, 0));
        ctx->rsum_cap = want;
    }
    DPlanArgs a{};
    a.cam = ctx->buf[B_RAW_CAM].as<int>();
    a.pt = ctx->buf[B_RAW_PT].as<int>();
    a.adm = ctx->buf[B_RAW_ADM].as<unsigned char>();
    a.no = no; a.np = np; a.nc = nc; a.fixed_cam = p->fixed_cam;
    a.tile_win = TILE_WIN; a.chunk_obs = CHUNK_OBS;
    a.po_dest = ctx->buf[B_DP_PO_DEST].as<int>();
    a.co_dest = ctx->buf[B_DP_CO_DEST].as<int>();
    a.cam_ac = ctx->buf[B_DP_CAM_AC].as<int>();
    a.pt_idx = ctx->buf[B_DP_PT_IDX].as<int>();
    a.ovf_obs = ctx->buf[B_DP_OVF].as<int>();
    a.sum = ctx->buf[B_DP_SUM].as<int>();
    a.sum_host = ctx->rsum_dev;
    a.scratch = ctx->buf[B_DP_SCRATCH].as<int>();
    HIPCHECK(ctx, dplan_enqueue(a, s));
    mark("enqueue");
    // a helper thread waits for the passes and builds the host side of the plan (tiles, chunks, segments) from the
    // summary while this thread stages the values and parameters
    hipError_t helper_err = hipSuccess;
    auto build_host_side = [&]() {
        helper_err = hipStreamSynchronize(s);
        const int* sm = ctx->rsum;
        if (helper_err == hipSuccess && sm[DP_TOOLONG] == 0 && sm[DP_BAD] == INT_MAX) {
            plan_from_device(sm, nc, np, p->fixed_cam, plan_params(sm[DP_NADM]), ctx->plan);
            built = true;
        }
    };
    std::thread helper;
    if (no >= DPLAN_HELPER_OBS) helper = std::thread(build_host_side);
    struct Join {
        std::thread& t;
        ~Join() { if (t.joinable()) t.join(); }
    } join{helper};
    // host work while the passes run: the values (behind the index DMA on the copy stream) and the parameters
    hipStream_t cs = ctx->copy_stream;
    HIPCHECK(ctx, hipStreamWaitEvent(cs, ctx->ev_idx, 0));
    // the values in pieces, each DMA'd while the next is staged (the copies and the DMA share the host's memory
    // bandwidth: same-box A/B, prepare ms at 1 / 2 / 4 / 8 pieces: C4 1.28-1.59 / 1.29-1.37 / 1.26-1.28 /
    // 1.36-1.42, C5 7.44 / 5.10 / 5.78 / 6.33); MIBA_VALUE_CHUNKS overrides
    int nchunk = no >= (1 << 19) ? 2 : 1;
    if (const char* e = std::getenv("MIBA_VALUE_CHUNKS")) nchunk = std::max(1, std::min(64, std::atoi(e)));
    notf32 = false;
    for (int c = 0; c < nchunk; ++c) {
        const size_t lo = (size_t)no * c / nchunk, n = (size_t)no * (c + 1) / nchunk - lo;
        if (!n) continue;
        notf32 = stage_values_f32check(rs.uv + 2 * lo, rs.dep + lo, p->obs_uv + 2 * lo, p->obs_depth + lo, n) || notf32;
        HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[B_RAW_DEP].as<double>() + lo, rs.dep + lo, 8 * n, hipMemcpyHostToDevice,
                                     cs));
        HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[B_RAW_UV].as<double>() + 2 * lo, rs.uv + 2 * lo, 16 * n,
                                     hipMemcpyHostToDevice, cs));
    }
    mark("stage_values");
    if (int rc = upload_params(ctx, p, cs)) return rc;
    HIPCHECK(ctx, hipEventRecord(ctx->ev_uv, cs));
    ctx->uv_pending = true;
    mark("params");
    if (helper.joinable()) helper.join();
    else build_host_side();
    HIPCHECK(ctx, helper_err);
    mark("helper");
    ok = ctx->rsum[DP_TOOLONG] == 0;
    return BA_OK;
}

static int prepare_core(ba_context* ctx, const ba_problem* p, bool force_det) {
    const ba_options& o = ctx->opts;
    const bool shard = ctx->W.comm.on();
    const double tp0 = now_ms();
    ctx->pinfo = ba_prepare_info{};
    ctx->pinfo.host_threads = host_threads();
    ctx->pinfo.bcr_path = -1;
    // validation: with landmark shards every rank must reach the same verdict before any further collective (a
    // rank that bailed out alone would leave the others waiting), so until the verdict all-reduce a rank-local
    // failure (an invalid problem, 1; a staging / allocation error, 2) goes into verdict[0] instead of a return
    int verdict[3] = {0, 0, 0};  // [0] error code (max), [1] n_cams (min), [2] -n_cams (min)
    std::string local_err;
    if (!p || p->n_cams < 0 || p->n_points < 0 || p->n_obs < 0) { local_err = "invalid problem sizes"; verdict[0] = 1; }
    else if ((p->n_cams && !p->cams) || (p->n_points && !p->points) || !p->intr || !p->intr_prior ||
             (p->n_obs && (!p->obs_cam || !p->obs_pt || !p->obs_uv || !p->obs_depth))) {
        local_err = "null problem buffer";
        verdict[0] = 1;
    }
    const int nc = verdict[0] ? 0 : p->n_cams, np = verdict[0] ? 0 : p->n_points, no = verdict[0] ? 0 : p->n_obs;
    // plan cache: a window with the last full prepare's structure reuses its plan (unsharded contexts)
    ba_context::PlanKey key{};
    key.nc = nc; key.np = np; key.no = no;
    key.fixed_cam = verdict[0] ? -1 : p->fixed_cam;
    key.det = (o.deterministic || force_det) ? 1 : 0;
    key.env = env_key();
    if (!verdict[0] && !shard && !force_det && !o.rebuild_plan && ctx->plan_ok && key == ctx->key) {
        const int r = prepare_reuse(ctx, p, tp0);
        if (r != 0) {
            ctx->pinfo.total_ms = now_ms() - tp0;
            return r < 0 ? r : BA_OK;
        }
    }
    ctx->plan_ok = false;
    ctx->prepared = false;
    hipStream_t s = ctx->stream;
    // the raw observations -> pinned staging -> HBM, in flight while the host builds the plan (landmark shards:
    // after the local count, its errors into the verdict)
    const size_t raw_bytes = raw_stage_bytes((size_t)no);
    // the device plan (unsharded windows that fit it)
    bool dplan = !shard && !verdict[0] && want_dplan(nc, np, no);
    bool notf32 = false;
    auto stage_raw = [&]() -> int {
        if (no <= 0) return BA_OK;
        if (ctx->uv_pending) {  // a prepare that failed after its pixel DMA: the staging buffer is still read
            HIPCHECK(ctx, hipEventSynchronize(ctx->ev_uv));
            ctx->uv_pending = false;
        }
        if (int rc = stage_ensure(ctx, raw_bytes, 0)) return rc;
        RawStage rs(ctx->stage, (size_t)no);
        HIPCHECK(ctx, ctx->buf[B_RAW_UV].ensure(16 * (size_t)no));
        HIPCHECK(ctx, ctx->buf[B_RAW_DEP].ensure(8 * (size_t)no));
        HIPCHECK(ctx, ctx->buf[B_RAW_CAM].ensure(4 * (size_t)no));
        HIPCHECK(ctx, ctx->buf[B_RAW_PT].ensure(4 * (size_t)no));
        {
            stage_copy({{rs.uv, p->obs_uv, 16 * (size_t)no}, {rs.dep, p->obs_depth, 8 * (size_t)no},
                        {rs.cam, p->obs_cam, 4 * (size_t)no}, {rs.pt, p->obs_pt, 4 * (size_t)no}});
            HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[B_RAW_UV].p, rs.uv, 16 * (size_t)no, hipMemcpyHostToDevice, s));
            HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[B_RAW_DEP].p, rs.dep, 8 * (size_t)no, hipMemcpyHostToDevice, s));
            HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[B_RAW_CAM].p, rs.cam, 4 * (size_t)no, hipMemcpyHostToDevice, s));
            HIPCHECK(ctx, hipMemcpyAsync(ctx->buf[B_RAW_PT].p, rs.pt, 4 * (size_t)no, hipMemcpyHostToDevice, s));
        }
        return BA_OK;
    };
    // the device plan stages and uploads the window itself (run_dplan, below)
    if (!shard && !verdict[0] && !dplan)
        if (int rc = stage_raw()) return rc;
    const double tp_raw = now_ms();
    Plan& pl = ctx->plan;
    PlanInput in;
    in.nc = nc; in.np = np; in.no = no;
    in.fixed_cam = verdict[0] ? -1 : p->fixed_cam;
    if (!verdict[0]) { in.obs_cam = p->obs_cam; in.obs_pt = p->obs_pt; in.obs_depth = p->obs_depth; }
    // obs32 records when every admissible pixel / depth is an f32 (the reference's are); MIBA_OBS32=0: f64 arrays
    if (!verdict[0]) {
        const char* e = std::getenv("MIBA_OBS32");
        if (!(e && e[0] == '0')) in.obs_uv = p->obs_uv;
    }
    // the device plan: its passes run behind the index / depth upload, the parameters are staged meanwhile, one
    // read-back (the window's values are valid: a malformed window fails below, before any of them is used)
    bool params_up = false, dplan_built = false;
    if (dplan) {
        if (int rc = run_dplan(ctx, p, nc, np, no, notf32, dplan, dplan_built)) return rc;
        params_up = true;
    }
    ctx->pinfo.plan_device = dplan ? 1 : 0;
    if (dplan) {
        const int* sm = ctx->rsum;
        pl.err = sm[DP_BAD] != INT_MAX ? "observation index out of range" : "";
        pl.n_adm = sm[DP_NADM];
        pl.obs32 = in.obs_uv != nullptr && !notf32;
        pl.cam_cnt.assign(sm + DP_HDR, sm + DP_HDR + nc);
    } else {
        plan_count(in, pl);
    }
    if (!verdict[0] && !pl.err.empty()) { local_err = pl.err; verdict[0] = 1; }
    int local_rc = BA_OK;
    if (shard) {
        if (!verdict[0] && (local_rc = stage_raw()) != BA_OK) { local_err = ctx->err; verdict[0] = 2; }
        verdict[1] = nc;
        verdict[2] = -nc;
        int rc = host_allreduce_i32(ctx, verdict, 1, COMM_MAX);
        if (rc == BA_OK) rc = host_allreduce_i32(ctx, verdict + 1, 2, COMM_MIN);
        if (rc != BA_OK) return rc;
        if (!verdict[0] && verdict[1] != -verdict[2]) { local_err = "landmark shards disagree on n_cams"; verdict[0] = 1; }
        if (verdict[0]) {
            ctx->err = local_err.empty() ? (verdict[0] >= 2 ? "another landmark shard failed to stage its observations"
                                                             : "another landmark shard rejected its problem")
                                         : local_err;
            return local_rc != BA_OK ? local_rc : (verdict[0] >= 2 ? BA_E_DEVICE : BA_E_INVALID);
        }
    } else if (verdict[0]) {
        ctx->err = local_err;
        return BA_E_INVALID;
    }
    const int n_adm = pl.n_adm;
    // active cameras (Ceres removes unused blocks; the gauge block is constant, :299): a camera
    // is active when any shard observes it; N (the 1/N weights, :280/:290) counts every shard
    std::vector<int> cam_seen(nc);
    for (int i = 0; i < nc; ++i) cam_seen[i] = pl.cam_cnt[i] > 0;
    int n_adm_all = n_adm;
    if (shard) {
        int rc = host_allreduce_i32(ctx, cam_seen.data(), nc, COMM_MAX);
        if (rc == BA_OK) rc = host_allreduce_i32(ctx, &n_adm_all, 1, COMM_SUM);
        if (rc != BA_OK) return rc;
    }
    const PlanParams pp = plan_params(n_adm);
    if (dplan) {
        if (!dplan_built) plan_from_device(ctx->rsum, nc, np, in.fixed_cam, pp, pl);
    } else {
        plan_order(in, cam_seen, pp, pl);
    }
    const int nac = pl.nac;
    if (shard) {  // envelope / band of the summed S: union over the shards
        const int rc = host_allreduce_i32(ctx, pl.fc.data(), nac, COMM_MIN);
        if (rc != BA_OK) return rc;
    }
    plan_envelope(pl);
    // the uploads and the device structure: every collective of the prepare is behind us, so a landmark shard that
    // fails here (allocation, staging, launch) says so in one more agreement all-reduce instead of leaving the
    // other ranks to wait in the first LM iteration's collectives
    auto finish = [&]() -> int {
        const double tp_plan = now_ms();
        const bool ftimes = std::getenv("MIBA_PLAN_TIMES") != nullptr;  // diagnostic: host phases of the finish
        double ftm = tp_plan;
        auto fmark = [&](const char* what) {
            if (!ftimes) return;
            const double t = now_ms();
            std::fprintf(stderr, "finish %s %.3f ms\n", what, t - ftm);
            ftm = t;
        };
        const int n_ap = pl.n_ap(), n_tiled = pl.n_tiled;
        const int n = pl.n, npad = pl.npad, nb = pl.nb, band_w = pl.band_w, cam_band = pl.cam_band;
        const int n_bs_chunks = (int)pl.bs_chunk.size() - 1;
        const int n_seg = (int)pl.seg_cam.size();
        const int n_env = (int)pl.env_tile.size() / 2;
        const bool det = (o.deterministic || force_det) && !pl.tile_base.empty();
        std::vector<int> trange;  // deterministic mode: each active camera's Schur tile range
        if (det) {
            trange.assign(2 * (size_t)std::max(nac, 1), 0);
            const int nt = (int)pl.tile_base.size();
            for (int a = 0, lo = 0, hi = 0; a < nac; ++a) {
                while (lo < nt && pl.tile_base[lo] < a - (TILE_WIN - 1)) ++lo;
                while (hi < nt && pl.tile_base[hi] <= a) ++hi;
                trange[2 * a] = lo;
                trange[2 * a + 1] = std::max(lo, hi);
            }
        }
        // ---- uploads: the plan's index arrays in one staged DMA (each array 256-byte aligned in B_PLAN)
        // (device plan: po_dest, co_dest, pt_idx and ovf_obs are copied on the device into their slots)
        struct Part { const int* src; size_t n; size_t off; const int* dev; };
        auto dv = [&](int id) -> const int* { return pl.dev ? ctx->buf[id].as<int>() : nullptr; };
        std::vector<Part> parts = {
            {pl.po_dest.data(), (size_t)no, 0, dv(B_DP_PO_DEST)}, {pl.co_dest.data(), (size_t)no, 0, dv(B_DP_CO_DEST)},
            {pl.cam_ac.data(), (size_t)nc, 0, nullptr},
            {pl.pt_ptr.data(), (size_t)n_ap + 1, 0, nullptr}, {pl.pt_idx.data(), (size_t)n_ap, 0, dv(B_DP_PT_IDX)},
            {pl.seg_ptr.data(), pl.seg_ptr.size(), 0}, {pl.seg_cam.data(), pl.seg_cam.size(), 0},
            {pl.seg_ac.data(), pl.seg_ac.size(), 0}, {pl.ac_seg.data(), pl.ac_seg.size(), 0},
            {pl.ac_cam.data(), (size_t)nac, 0}, {pl.fcol.data(), (size_t)nb, 0},
            {pl.tile_chunk.data(), pl.tile_chunk.size(), 0}, {pl.tile_base.data(), pl.tile_base.size(), 0},
            {pl.tile_span.data(), pl.tile_span.size(), 0}, {pl.chunk_ap.data(), pl.chunk_ap.size(), 0},
            {pl.bs_chunk.data(), pl.bs_chunk.size(), 0}, {pl.ovf_obs.data(), (size_t)pl.n_ovf(), 0, dv(B_DP_OVF)},
            {pl.rptr.data(), (size_t)nb + 1, 0}, {pl.rows.data(), pl.rows.size(), 0},
            {pl.env_tile.data(), pl.env_tile.size(), 0}, {trange.data(), trange.size(), 0}};
        enum { PO_DEST, CO_DEST, CAM_AC, PT_PTR, PT_IDX, SEG_PTR, SEG_CAM, SEG_AC, AC_SEG, AC_CAM, FCOL, TILE_CHUNK,
               TILE_BASE, TILE_SPAN, CHUNK_AP, BS_CHUNK, OVF_OBS, RPTR, ROWS, ENV_TILE, TRANGE };
        size_t plan_ints = 0;
        for (Part& q : parts) {
            q.off = plan_ints;
            plan_ints += (q.n + 63) / 64 * 64 + 64;
        }
        const size_t raw_off = (raw_bytes + 255) / 256 * 256;  // after the raw region, which may still be in flight
        if (ctx->stage_cap < raw_off + 4 * plan_ints) {
            // growing frees the buffer the raw DMAs read: the index DMA on `stream`, the device plan's pixel /
            // depth DMA on the copy stream
            HIPCHECK(ctx, hipStreamSynchronize(s));
            if (ctx->uv_pending) HIPCHECK(ctx, hipEventSynchronize(ctx->ev_uv));
            if (int rc = stage_ensure(ctx, raw_off + 4 * plan_ints, raw_bytes)) return rc;
        }
        int* sp = reinterpret_cast<int*>(ctx->stage + raw_off);
        {
            std::vector<StageCopy> cp;
            for (const Part& q : parts)
                if (q.n && !q.dev) cp.push_back({sp + q.off, q.src, 4 * q.n});
            stage_copy(cp);
        }
        fmark("stage_plan");
        HIPCHECK(ctx, ctx->buf[B_PLAN].ensure(4 * plan_ints));
        int* dp = ctx->buf[B_PLAN].as<int>();
        {  // device plan: from the first host part on (po_dest / co_dest lead and come device-to-device)
            const size_t lo = pl.dev ? parts[CAM_AC].off : 0;
            HIPCHECK(ctx, hipMemcpyAsync(dp + lo, sp + lo, 4 * (plan_ints - lo), hipMemcpyHostToDevice, s));
        }
        ctx->plan_parts.clear();
        for (const Part& q : parts) {
            ctx->plan_parts.emplace_back(q.off, q.n);
            if (q.n && q.dev) HIPCHECK(ctx, hipMemcpyAsync(dp + q.off, q.dev, 4 * q.n, hipMemcpyDeviceToDevice, s));
        }
        auto dptr = [&](int k) { return dp + parts[k].off; };
        if (!params_up)
            if (int rc = upload_params(ctx, p, s)) return rc;
        // the observation layouts, gathered on the device from the raw window and the plan's orderings
        // ... in ONE layout: the 16-byte records on obs32 windows, the f64 arrays otherwise (the index arrays always)
        HIPCHECK(ctx, ctx->buf[B_PO_AC].ensure(4 * std::max<size_t>(n_adm, 1)));
        HIPCHECK(ctx, ctx->buf[B_PO_AP].ensure(4 * std::max<size_t>(n_adm, 1)));
        HIPCHECK(ctx, ctx->buf[B_PO_PT].ensure(4 * std::max<size_t>(n_adm, 1)));
        if (pl.obs32) {
            HIPCHECK(ctx, ctx->buf[B_PO_REC].ensure(16 * std::max<size_t>(n_adm, 1)));
            HIPCHECK(ctx, ctx->buf[B_CO_REC].ensure(16 * std::max<size_t>(n_adm, 1)));
        } else {
            HIPCHECK(ctx, ctx->buf[B_PO_CAM].ensure(4 * std::max<size_t>(n_adm, 1)));
            HIPCHECK(ctx, ctx->buf[B_PO_UV].ensure(16 * std::max<size_t>(n_adm, 1)));
            HIPCHECK(ctx, ctx->buf[B_PO_DEP].ensure(8 * std::max<size_t>(n_adm, 1)));
            HIPCHECK(ctx, ctx->buf[B_CO_PT].ensure(4 * std::max<size_t>(n_adm, 1)));
            HIPCHECK(ctx, ctx->buf[B_CO_UV].ensure(16 * std::max<size_t>(n_adm, 1)));
            HIPCHECK(ctx, ctx->buf[B_CO_DEP].ensure(8 * std::max<size_t>(n_adm, 1)));
        }
        ctx->ac_cam = pl.ac_cam;
        ctx->pt_idx = pl.pt_idx;
        const std::vector<int>& tile_base = pl.tile_base;

        const int nblk_pt = pp_blocks(n_ap, PP_LANES_MAX);  // part slots sized for the widest lane grouping
        // (+ the small-window launch's per-tile and non-tiled point partials, §3 of DESIGN)
        const int part_stride = std::max({nblk_pt, (nac + 1 + 255) / 256, n_bs_chunks, (nac + BCR_CAMS - 1) / BCR_CAMS,
                                          (int)pl.tile_base.size() + pp_blocks(n_ap - n_tiled, PP_LANES_MAX), 1});
        HIPCHECK(ctx, ctx->buf[B_CAMDATA].ensure(sizeof(double) * ((size_t)CAMDATA * std::max(nac, 1) + 16)));
        // landmark sharding: pack buffers of the envelope tiles of S, exchange scalars
        if (shard) {
            // envelope tiles + rhs (+ the camera and intrinsics sums of the folded exchange)
            const size_t ne = (size_t)n_env * 256 + (size_t)npad + (size_t)nac * CAMDATA + SEGINTR + 1;
            HIPCHECK(ctx, ctx->buf[B_CAMDATA_LOC].ensure(sizeof(double) * ((size_t)CAMDATA * std::max(nac, 1) + 16)));
            HIPCHECK(ctx, hipMemsetAsync(ctx->buf[B_CAMDATA_LOC].p, 0, sizeof(double) * ((size_t)CAMDATA * std::max(nac, 1) + 16), s));
            HIPCHECK(ctx, ctx->buf[B_ENV_LOC].ensure(sizeof(double) * ne));
            const size_t nred = RED_X + 4 + 2 * (size_t)ctx->W.comm.nranks;
            HIPCHECK(ctx, ctx->buf[B_RED].ensure(sizeof(double) * nred));
            HIPCHECK(ctx, hipMemsetAsync(ctx->buf[B_RED].p, 0, sizeof(double) * nred, s));
        }
        HIPCHECK(ctx, ctx->buf[B_SEGINTR].ensure(sizeof(double) * SEGINTR * std::max(n_seg, 1)));
        HIPCHECK(ctx, ctx->buf[B_CAMPART].ensure(sizeof(double) * CAMDATA * std::max(n_seg, 1)));
        HIPCHECK(ctx, ctx->buf[B_LIN].ensure(sizeof(double) * LIN_N));
        HIPCHECK(ctx, ctx->buf[B_SCALE].ensure(sizeof(double) * (6 * nac + 3 * (size_t)n_ap + 4)));
        HIPCHECK(ctx, ctx->buf[B_CNP].ensure(sizeof(double) * 3 * std::max(n_ap, 1)));
        HIPCHECK(ctx, ctx->buf[B_PDATA].ensure(sizeof(double) * PDATA * std::max(n_ap, 1)));
        HIPCHECK(ctx, ctx->buf[B_S].ensure(sizeof(double) * (size_t)npad * npad));
        HIPCHECK(ctx, hipMemsetAsync(ctx->buf[B_S].p, 0, sizeof(double) * (size_t)npad * npad, s));
        HIPCHECK(ctx, ctx->buf[B_RHS].ensure(sizeof(double) * npad));
        HIPCHECK(ctx, hipMemsetAsync(ctx->buf[B_RHS].p, 0, sizeof(double) * npad, s));
        HIPCHECK(ctx, ctx->buf[B_DELTA].ensure(sizeof(double) * npad));
        HIPCHECK(ctx, ctx->buf[B_PART].ensure(sizeof(double) * PART_NSLOTS * part_stride));
        HIPCHECK(ctx, ctx->buf[B_SCAL].ensure(sizeof(double) * SC_N));
        HIPCHECK(ctx, ctx->buf[B_FLAG].ensure(sizeof(int) * 8));
        HIPCHECK(ctx, ctx->buf[B_STATE].ensure(sizeof(LmState)));
        HIPCHECK(ctx, ctx->buf[B_LOG].ensure(sizeof(double) * LOG_W * (std::max(o.max_num_iterations, 0) + 2)));
        HIPCHECK(ctx, hipMemsetAsync(ctx->buf[B_PART].p, 0, sizeof(double) * PART_NSLOTS * part_stride, s));
        HIPCHECK(ctx, empty_tail_slots(ctx->buf[B_PART].as<double>(), part_stride, s));

        DevProblem& P = ctx->P;
        P.cams[0] = ctx->buf[B_CAMS0].as<double>(); P.cams[1] = ctx->buf[B_CAMS1].as<double>();
        P.pts[0] = ctx->buf[B_PTS0].as<double>(); P.pts[1] = ctx->buf[B_PTS1].as<double>();
        P.K[0] = ctx->buf[B_K0].as<double>(); P.K[1] = ctx->buf[B_K1].as<double>();
        P.prior = ctx->buf[B_PRIOR].as<double>();
        const bool f64l = !pl.obs32;  // the f64 layout (else nullptr: no kernel of an obs32 window reads it)
        P.po_cam = f64l ? ctx->buf[B_PO_CAM].as<int>() : nullptr; P.po_ac = ctx->buf[B_PO_AC].as<int>();
        P.po_uv = f64l ? ctx->buf[B_PO_UV].as<double2>() : nullptr;
        P.po_depth = f64l ? ctx->buf[B_PO_DEP].as<double>() : nullptr;
        P.po_ap = ctx->buf[B_PO_AP].as<int>(); P.po_pt = ctx->buf[B_PO_PT].as<int>();
        P.pt_ptr = dptr(PT_PTR);
        P.pt_idx = dptr(PT_IDX);
        P.co_pt = f64l ? ctx->buf[B_CO_PT].as<int>() : nullptr;
        P.co_uv = f64l ? ctx->buf[B_CO_UV].as<double2>() : nullptr;
        P.co_depth = f64l ? ctx->buf[B_CO_DEP].as<double>() : nullptr;
        P.obs32 = pl.obs32 ? 1 : 0;
        P.po_rec = pl.obs32 ? ctx->buf[B_PO_REC].as<float4>() : nullptr;
        P.co_rec = pl.obs32 ? ctx->buf[B_CO_REC].as<float4>() : nullptr;
        P.seg_ptr = dptr(SEG_PTR); P.seg_cam = dptr(SEG_CAM);
        P.seg_ac = dptr(SEG_AC); P.ac_cam = dptr(AC_CAM);
        P.ac_seg = reinterpret_cast<const int2*>(dptr(AC_SEG));
        P.tile_chunk = dptr(TILE_CHUNK); P.tile_base = dptr(TILE_BASE);
        P.tile_span = dptr(TILE_SPAN); P.chunk_ap = dptr(CHUNK_AP);
        P.ovf_obs = dptr(OVF_OBS);
        P.bs_chunk = dptr(BS_CHUNK);
        P.n_bs_chunks = n_bs_chunks;
        P.n_tiles = (int)tile_base.size(); P.n_ovf_obs = pl.n_ovf();
        P.n_tiled_pts = n_tiled;
        ctx->n_tiles = P.n_tiles; ctx->n_ovf_obs = P.n_ovf_obs; ctx->n_tiled_pts = n_tiled;
        P.n_seg = n_seg; P.n_ap = n_ap; P.n_adm = n_adm; P.nac = nac; P.n_cams = nc;
        P.n = n; P.npad = npad; P.kb = 6 * nac;
        P.off_pt = 6 * nac; P.off_k = 6 * nac + 3 * n_ap;
        {
            PrepRaw R;
            R.cam = ctx->buf[B_RAW_CAM].as<int>();
            R.pt = ctx->buf[B_RAW_PT].as<int>();
            R.uv = ctx->buf[B_RAW_UV].as<double2>();
            R.depth = ctx->buf[B_RAW_DEP].as<double>();
            R.cam_ac = dptr(CAM_AC);
            R.po_dest = dptr(PO_DEST);
            R.co_dest = dptr(CO_DEST);
            R.n_obs = no;
            ctx->raw = R;
            if (ctx->uv_pending) {  // the device plan's pixel DMA (copy stream)
                HIPCHECK(ctx, hipStreamWaitEvent(s, ctx->ev_uv, 0));
                ctx->uv_pending = false;
            }
            HIPCHECK(ctx, launch_prep_gather(P, R, s));
        }
        fmark("allocs_gather");
        P.part_stride = part_stride;
        P.band_w = (nb >= 2 && nb <= 2048 && band_w <= 6) ? std::max(band_w, 1) : 0;
        P.cam_band = cam_band;
        // reduced-system solver: block cyclic reduction when the camera band fits a 64-dof block (a window of
        // <= 10 active cameras is one block: the root alone, its factorization on the split kernel's look-ahead
        // pivot chain — C1 4.9 ms per solve against 5.6 with the band Cholesky); else the banded LDS Cholesky;
        // else the dense envelope kernel.
        const int bcr_nblk = (nac + BCR_CAMS - 1) / BCR_CAMS;
        P.solver = (cam_band < BCR_CAMS && bcr_nblk >= 1) ? 2 : (P.band_w > 0 ? 1 : 0);
        if (const char* e = std::getenv("MIBA_SOLVER")) {
            if (!std::strcmp(e, "dense")) P.solver = 0;
            else if (!std::strcmp(e, "band") && P.band_w > 0) P.solver = 1;
            else if (!std::strcmp(e, "bcr") && cam_band < BCR_CAMS && bcr_nblk >= 1) P.solver = 2;
        }
        if (const char* e = std::getenv("MIBA_DENSE_CHOL")) if (e[0] == '1') P.solver = 0;
        {
            const char* ef = std::getenv("MIBA_FUSED");
            const char* et = std::getenv("MIBA_TAIL");
            ctx->tail_possible = !shard && !det && n_ap > 0 && n_seg > 0 && !(ef && ef[0] == '0') &&
                                 !(et && et[0] == '0') && n_bs_chunks + 2 <= 128;
        }
        if (P.solver == 2) {
            const size_t bytes = bcr_bytes(bcr_nblk);
            HIPCHECK(ctx, ctx->buf[B_BCR].ensure(bytes));
            double* base = ctx->buf[B_BCR].as<double>();
            BcrWork& Bw = ctx->W.bcr;
            Bw.nblk = bcr_nblk;
            Bw.levels = 0;
            while ((1 << Bw.levels) < bcr_nblk) ++Bw.levels;
            // balanced elimination tree for the split kernels: K = floor(log2 nblk), v = i + 2^K - nblk/2,
            // so [voff, voff + nblk) holds one multiple of 2^K (the root, block nblk/2) and none of 2^(K+1)
            Bw.vlevels = 0;
            while ((2 << Bw.vlevels) <= bcr_nblk) ++Bw.vlevels;
            Bw.voff = (1 << Bw.vlevels) - bcr_nblk / 2;
            Bw.vroot = bcr_nblk / 2;
            const size_t b64 = (size_t)64 * 64 * bcr_nblk, b8 = (size_t)64 * 8 * bcr_nblk;
            Bw.Cf = base;
            Bw.X = Bw.Cf + b64;
            Bw.UL = Bw.X + (size_t)64 * BCR_XW * bcr_nblk;
            Bw.UR = Bw.UL + b64;
            Bw.F = Bw.UR + b64;
            Bw.Dacc = Bw.F + b64;
            Bw.rL = Bw.Dacc + b64;
            Bw.rR = Bw.rL + b8;
            Bw.Racc = Bw.rR + b8;
            Bw.Y = Bw.Racc + b8;
            Bw.Bp = Bw.Y + b8;
            Bw.rd = Bw.Bp + (size_t)32 * bcr_nblk;
            Bw.F2 = Bw.rd + (size_t)64 * bcr_nblk;
            Bw.bk = Bw.F2 + b64;
            Bw.flags = reinterpret_cast<unsigned*>(Bw.bk + 16);  // zeroed with the workspace above
            if (int rc = bcr_setup(ctx)) return rc;
        }
        fmark("solver_setup");
        DevWork& W = ctx->W;
        W.camdata = ctx->buf[B_CAMDATA].as<double>(); W.seg_intr = ctx->buf[B_SEGINTR].as<double>();
        W.camdata_loc = shard ? ctx->buf[B_CAMDATA_LOC].as<double>() : W.camdata;
        W.camdata_part = ctx->buf[B_CAMPART].as<double>();
        W.env_tile = reinterpret_cast<const int2*>(dptr(ENV_TILE));
        W.n_env = n_env;
        W.env_loc = shard ? ctx->buf[B_ENV_LOC].as<double>() : nullptr;
        W.red = shard ? ctx->buf[B_RED].as<double>() : nullptr;
        P.rank = W.comm.rank;
        P.nranks = W.comm.nranks;
        {
            const char* e = std::getenv("MIBA_XCD_MAP");
            P.xcd_map = (e && e[0] == '0') ? 0 : 1;
        }
        W.lin = ctx->buf[B_LIN].as<double>(); W.scale = ctx->buf[B_SCALE].as<double>();
        W.cnp = ctx->buf[B_CNP].as<double>(); W.pdata = ctx->buf[B_PDATA].as<double>();
        W.S = ctx->buf[B_S].as<double>(); W.rhs = ctx->buf[B_RHS].as<double>();
        W.delta = ctx->buf[B_DELTA].as<double>(); W.part = ctx->buf[B_PART].as<double>();
        W.scal = ctx->buf[B_SCAL].as<double>(); W.chol_flag = ctx->buf[B_FLAG].as<int>();
        W.fcol = dptr(FCOL); W.rptr = dptr(RPTR); W.rows = dptr(ROWS);
        W.st = ctx->buf[B_STATE].as<LmState>(); W.log = ctx->buf[B_LOG].as<double>();
        // deterministic mode: the Schur tiles write per-tile slabs, summed in tile order per element of S
        W.det_tbuf = nullptr;
        W.det_trange = nullptr;
        if (det) {
            HIPCHECK(ctx, ctx->buf[B_DET_TBUF].ensure(sizeof(double) * SCH_TBUF * (size_t)P.n_tiles));
            W.det_tbuf = ctx->buf[B_DET_TBUF].as<double>();
            W.det_trange = reinterpret_cast<const int2*>(dptr(TRANGE));
        }
        // fused LM-loop linearisation (k_lin_point + envelope tiles in k_schur_tile, S / rhs zeroed by the previous
        // iteration): the unsharded default-mode path with points and camera segments
        {
            const char* e = std::getenv("MIBA_FUSED");
            const bool off = e && e[0] == '0';
            // landmark shards: the same choice on every rank (it fixes the collective sequence), so only uniform inputs
            W.fused = (shard ? (!o.deterministic && !off)
                             : (!W.det_tbuf && n_ap > 0 && n_seg > 0 && !off)) ? 1 : 0;
            // small windows: the point side inside the Schur tiles, the camera side and the non-tiled points as
            // extra workgroups of the Schur launch (no k_lin_point in the LM loop) when the whole launch is one
            // resident round (its envelope tiles wait for its camera side); MIBA_SW=0 keeps the two launches
            // the band solve's tail (back-substitution chunks + decision) in its launch: unsharded default-mode band
            // windows whose tail fits one resident round; MIBA_TAIL=0 keeps the separate launches
            const char* e4 = std::getenv("MIBA_TAIL");
            W.tail = (P.solver == 2 && W.bcr.band && W.fused && !shard && !W.det_tbuf && band_tail_blocks(P, W.bcr.band) > 0 &&
                      !(e4 && e4[0] == '0')) ? 1 : 0;
            // larger windows, opt-in (MIBA_BSFIN=1): the back-substitution chunks and the decision in one launch
            // (k_backsub_final). Measured slower at C4 (4035-4070 vs 4154-4195 LM it/s, same box: the chunks'
            // drained agent-scope partial stores and the decision workgroup's agent-scope loads cost more than the
            // k_final launch they save) and even at C2, so k_backsub_chunk + k_final stay the default
            const char* e5 = std::getenv("MIBA_BSFIN");
            W.bsfin = (!W.tail && W.fused && !shard && !W.det_tbuf && n_ap > 0 && P.n_bs_chunks > 0 &&
                       (e5 && e5[0] == '1')) ? 1 : 0;
            W.tail_flags = reinterpret_cast<unsigned*>(ctx->buf[B_FLAG].as<int>() + 4);
            // the band tail's y hand-off: two npad-double buffers by launch parity (flag-free, emptied by launch_reset)
            W.tail_y = nullptr;
            if (W.tail) {
                HIPCHECK(ctx, ctx->buf[B_TAIL_Y].ensure(sizeof(double) * 2 * (size_t)P.npad));
                W.tail_y = ctx->buf[B_TAIL_Y].as<double>();
            }
            W.tail_seq = 0;
            HIPCHECK(ctx, hipMemsetAsync(W.tail_flags, 0, 3 * sizeof(unsigned), s));
            const char* e2 = std::getenv("MIBA_SW");
            const int n_sw = P.n_tiles + 1 + n_seg + pp_blocks(n_ap - n_tiled, 1) + n_env;
            // one-block windows (<= BCR_CAMS active cameras) and the band tail's windows. The camera side hands
            // its sums to the envelope tiles without a release fence (round 5): C3 with the tail launch 58.8-58.9 us
            // per LM iteration against 62.1-62.3 with k_lin_point (same box); round 4's fenced hand-off measured
            // 3 us slower than k_lin_point there. MIBA_SW=0: off; 2: every window that fits
            const bool sw_fit = W.fused && !shard && P.n_tiles > 0 && n_sw <= 256;
            W.sw = (sw_fit && (nac <= BCR_CAMS || W.tail) && !(e2 && e2[0] == '0')) ? 1 : 0;
            if (e2 && e2[0] == '2') W.sw = sw_fit ? 1 : 0;  // A/B
            // larger windows, opt-in (MIBA_FPL=1): the tiled points' point side in the Schur tiles. k_lin_point
            // 48 -> 25 us at C4 but the tiles 76 -> 133 us (their per-chunk point reduction and tail run on one
            // wave between two barriers, and the registers spill), 4140 -> 3650 LM it/s
            const char* e3 = std::getenv("MIBA_FPL");
            W.fpl = (W.fused && !shard && !W.det_tbuf && P.n_tiles > 0 && !W.sw && e3 && e3[0] == '1') ? 1 : 0;
            W.sw_cnt = reinterpret_cast<unsigned*>(ctx->buf[B_FLAG].as<int>() + 2);
            W.sw_seq = 0;
            HIPCHECK(ctx, hipMemsetAsync(W.sw_cnt, 0, sizeof(unsigned), s));
        }
        ctx->n_adm_all = n_adm_all;
        ctx->sw_full = W.sw;
        ctx->tail_full = W.tail;
        ctx->bsfin_full = W.bsfin;
        set_consts(ctx);
        ctx->nblk_pt = nblk_pt;
        ctx->prepared = true;
        ctx->prep_nc = nc; ctx->prep_np = np; ctx->prep_no = no;
        // Algorithmic (compulsory) traffic per launch, DESIGN.md §Roofline:
        // each input byte read once, each output byte written once.
        {
            const double A = n_adm, Pn = n_ap, Cn = nac, Sg = n_seg;
            double env = 0;  // envelope tiles of the reduced system
            for (int k = 0; k < nb; ++k) env += (double)(pl.rptr[k + 1] - pl.rptr[k]) + 1.0;
            const double env_bytes = env * 16 * 16 * 8;
            double* kb = ctx->k_bytes;
            double* kf = ctx->k_flops;
            // observation record per sweep: obs32 {u, v, depth, index} 16 B; f64 arrays: index 4 + pixel 16 + depth 8
            const double rec = P.obs32 ? 16.0 : 28.0;
            kb[K_CAM_SIDE] = A * rec + Pn * 24 + (Cn + 1) * 56 + 32 + Sg * (CAMDATA + SEGINTR) * 8;
            kb[K_CAM_REDUCE] = Sg * CAMDATA * 8 + Cn * CAMDATA * 8;
            kf[K_CAM_SIDE] = A * 420;
            kb[K_LIN_FINALIZE] = Sg * SEGINTR * 8 + Cn * (56 + 48) + LIN_N * 8;
            kb[K_POINT_COLNORM] = A * rec + Pn * (8 + 24 + 24);
            kb[K_SCALE] = (6 * Cn + 3 * Pn + 4) * 16;
            kb[K_MEMSET_S] = (double)n_env * 256 * 8;
            kb[K_ASSEMBLE] = Cn * CAMDATA * 8 + Cn * 36 * 8 + Cn * 24 * 8;
            kb[K_POINT_PREP] = A * rec + Pn * (8 + 24 + 24) + Pn * PDATA * 8;
            kf[K_POINT_PREP] = A * 300 + Pn * 200;
            kb[K_SCHUR_TILE] = A * (rec + 12) + Pn * (PDATA * 8 + 24 + 24 + 8) + env_bytes + npad * 8.0;
            kf[K_SCHUR_TILE] = A * 350 + Pn * 13300;
            kb[K_OBS_PAIRS] = ctx->n_ovf_obs * 40.0;
            kb[K_CHOL] = 2 * env_bytes + 3 * npad * 8.0;
            kf[K_CHOL] = 0;
            for (int k = 0; k < nb; ++k) {
                const double r = pl.rptr[k + 1] - pl.rptr[k];
                kf[K_CHOL] += (r * (r + 1) / 2) * 2.0 * 16 * 16 * 16 + r * 16 * 16 * 16 + 16 * 16 * 16 / 3.0;
            }
            if (P.solver == 2) {
                // block cyclic reduction: per eliminated 64-dof block, Cholesky 64^3/3 + forward solve of
                // 136 columns 64^2*136 (elim); 44 16x16x64 contribution tiles (contrib); per launch =
                // solve total / launches per solve. Bytes: the blocks each kernel must read / write.
                const int nblk = ctx->W.bcr.nblk, L = ctx->W.bcr.levels;
                const double blk = 64.0 * 64 * 8, xblk = 64.0 * 136 * 8;
                double e_fl = 64.0 * 64 * 64 / 3 + 2.0 * 64 * 64 * 8, e_by = 3 * blk + 2 * 64 * 8 * 8;  // root
                double c_fl = 0, c_by = 0, b_by = 0;
                for (int m = 0; m < L; ++m) {
                    const int s_ = 1 << m, nel = (nblk - s_ + 2 * s_ - 1) / (2 * s_);
                    e_fl += nel * (64.0 * 64 * 64 / 3 + 64.0 * 64 * 136 * 2);
                    e_by += nel * (5 * blk + blk + xblk);
                    c_fl += nel * 44.0 * 16 * 16 * 64 * 2;
                    c_by += nel * (xblk + 3 * blk + 2 * 64 * 8 * 8);
                    b_by += nel * (blk + xblk + 3 * 64 * 8 * 8);
                }
                kf[K_BCR_ELIM] = e_fl / (L + 1); kb[K_BCR_ELIM] = e_by / (L + 1);
                kf[K_BCR_CONTRIB] = c_fl / std::max(L, 1); kb[K_BCR_CONTRIB] = c_by / std::max(L, 1);
                kf[K_BCR_BACK] = nblk * 2.0 * 64 * 64 * 8 * 2 / std::max(L, 1); kb[K_BCR_BACK] = b_by / std::max(L, 1);
                kb[K_BCR_BORDER] = nblk * (32.0 + 64 * 8) * 8;
                // persistent kernel = the whole elimination + contributions + back-substitution in one
                // launch; bytes: S blocks read once (D, level-0 couplings, border rows, rhs), the
                // contributions written once and read by the two neighbours, y written / read twice.
                // (k_bcr_split hands the eliminated blocks' X rows over instead — XL, XR, x written once and
                // read once by the survivors — which the per-launch model below counts.)
                double p_by = nblk * (blk + 4 * 64 * 8.0 + 64 * 8 * 8.0), n_el = 0;
                for (int m = 0; m < L; ++m) {
                    const int s_ = 1 << m, nel = (nblk - s_ + 2 * s_ - 1) / (2 * s_);
                    n_el += nel;
                    if (m == 0) p_by += nel * 2 * blk;
                }
                p_by += (ctx->W.bcr.persist >= 2 ? n_el * 2 * (2 * blk + 64 * 8 * 8.0) : n_el * 3 * (3 * blk + 2 * 64 * 8 * 8.0)) +
                        nblk * 3 * 64 * 8 * 8.0;
                kf[K_BCR_PERSIST] = e_fl + c_fl + kf[K_BCR_BACK] * std::max(L, 1);
                kb[K_BCR_PERSIST] = p_by;
            }
            kb[K_UPDATE_CAMS] = Cn * (56 * 2 + 48 * 3) + 4 * 8 * 4;
            kb[K_BACKSUB_EVAL] = A * (rec + 8) + Pn * (8 + 24 * 2 + 24 + PDATA * 8) + npad * 16.0;  // obs records read once
            kf[K_BACKSUB_EVAL] = A * 450;
            kb[K_FINAL] = (double)PART_NSLOTS * part_stride * 8;
            kb[K_LIN_POINT] = kb[K_CAM_SIDE] + kb[K_POINT_PREP];  // the whole linearisation pass of an accepted step
            kf[K_LIN_POINT] = kf[K_CAM_SIDE] + kf[K_POINT_PREP];
        }
        fmark("work_accounting");
        if (std::getenv("MIBA_PREP_TIMES"))  // diagnostic: host phases of ba_prepare (the device work is still in flight)
            std::fprintf(stderr, "prepare: raw staging %.3f ms, plan %.3f ms, plan staging + enqueue %.3f ms (%d host threads)\n",
                         tp_raw - tp0, tp_plan - tp_raw, now_ms() - tp_plan, host_threads());
        ctx->pinfo.plan_ms = tp_plan - tp_raw;
        ctx->pinfo.upload_ms = (tp_raw - tp0) + (now_ms() - tp_plan);
        ctx->pinfo.obs_uploaded = 1;
        ctx->pinfo.bcr_path = P.solver == 2 ? bcr_path_id(ctx->W.bcr) : -1;
        ctx->pinfo.lin_path = ctx->W.sw;
    ctx->pinfo.tail = ctx->W.tail;
    ctx->pinfo.bsfin = ctx->W.bsfin;
        return BA_OK;
    };
    int rc = finish();
    if (shard) {
        int bad = rc != BA_OK ? 1 : 0;
        const std::string my_err = ctx->err;
        const int rc2 = host_allreduce_i32(ctx, &bad, 1, COMM_MAX);
        if (rc == BA_OK && rc2 != BA_OK) rc = rc2;
        else if (rc == BA_OK && bad) {
            ctx->err = "another landmark shard failed its prepare (device allocation / upload)";
            rc = BA_E_DEVICE;
        } else if (rc != BA_OK) ctx->err = my_err;
        if (rc != BA_OK) ctx->prepared = false;
        return rc;
    }
    if (rc != BA_OK) return rc;
    // plan cache (unsharded, not gathered): this window's structure is the context's from now on
    ctx->key = key;
    ctx->key.obs32 = pl.obs32 ? 1 : 0;
    ctx->plan_ok = !force_det;
    ctx->pinfo.total_ms = now_ms() - tp0;
    return BA_OK;
}

// Fresh LM state (Ceres IterationZero): radius = initial_trust_region_radius.
static LmState fresh_state(const ba_options& o, double radius) {
    LmState st{};
    st.radius = radius;
    st.decrease_factor = 2.0;
    st.n_succ = 1;  // iteration 0 counts as successful (Ceres convention)
    st.step_ok = 1;
    st.termination = -1;
    st.stop_next = o.max_num_iterations <= 0;
    return st;
}

static void format_message(const LmState& S, char* out, size_t n) {
    switch (S.msg) {
        case MSG_MAX_ITER: std::snprintf(out, n, "Maximum number of iterations reached. Number of iterations: %d.", (int)S.msg_a); break;
        case MSG_GRAD_TOL: std::snprintf(out, n, "Gradient tolerance reached. Gradient max norm: %e <= %e", S.msg_a, S.msg_b); break;
        case MSG_MIN_RADIUS: std::snprintf(out, n, "Minimum trust region radius reached. Trust region radius: %e <= %e", S.msg_a, S.msg_b); break;
        case MSG_PARAM_TOL: std::snprintf(out, n, "Parameter tolerance reached. Relative step_norm: %e <= %e.", S.msg_a, S.msg_b); break;
        case MSG_FUNC_TOL: std::snprintf(out, n, "Function tolerance reached. |cost_change|/cost: %e <= %e", S.msg_a, S.msg_b); break;
        case MSG_INVALID: std::snprintf(out, n, "Number of consecutive invalid steps more than Solver::Options::max_num_consecutive_invalid_steps: %d", (int)S.msg_a); break;
        case MSG_EVAL_FAIL: std::snprintf(out, n, "Residual and Jacobian evaluation failed."); break;
        case MSG_TIMEOUT: std::snprintf(out, n, "Reduced camera solve failed: an inter-workgroup hand-off of the resident BCR kernel timed out."); break;
        default: std::snprintf(out, n, "unknown"); break;
    }
}

static void print_header() {
    std::printf("iter      cost      cost_change  |gradient|   |step|    tr_ratio  tr_radius  ls_iter  iter_time  total_time\n");
}
static void print_row(int it, double cost, double dc, double g, double st, double rho, double rad, double ti, double tt) {
    std::printf("% 4d % 3.6e % 3.2e % 3.2e % 3.2e % 3.2e % 3.2e % 4d % 3.2e % 3.2e\n", it, cost, dc, g, st, rho, rad, 0,
                ti * 1e-3, tt * 1e-3);
    std::fflush(stdout);
}

// The spin bound is a per-device global of the BCR module: remembered per device, set under the context's
// device (the caller has made it current), serialised across contexts / threads.
static int apply_spin_limit(ba_context* ctx) {
    static std::mutex mu;
    static std::vector<unsigned> applied;  // per device; 0 = not yet set
    // tests: force the hand-off timeout path of the resident BCR kernels and of the small-window launch's wait
    const char* e = std::getenv("MIBA_BCR_SPIN_LIMIT");
    unsigned want = e ? (unsigned)std::strtoul(e, nullptr, 10) : (1u << 22);
    if (want == 0) want = 1;
    const unsigned want_sw = e ? want : (1u << 20);
    std::lock_guard<std::mutex> lock(mu);
    if ((int)applied.size() <= ctx->device) applied.resize(ctx->device + 1, 0u);
    if (applied[ctx->device] != want) {
        HIPCHECK(ctx, bcr_set_spin_limit(want));
        HIPCHECK(ctx, sw_set_spin_limit(want_sw));
        HIPCHECK(ctx, tail_set_spin_limit(want_sw));
        applied[ctx->device] = want;
    }
    return BA_OK;
}

// A hand-off of the resident BCR kernel timed out (its workgroups were not all co-resident: another context
// or process held CUs). The decision stopped the device loop without a termination and without counting the
// iteration (x, radius and the trust-region state untouched): from now on this context runs the per-level
// launches (no inter-workgroup waits), and the host re-enqueues the iteration. The in-flight iterations behind
// the decision were no-ops. S / rhs are cleared here for the re-run's assembly.
static int bcr_timeout_retry(ba_context* ctx, LmState& S) {
    hipStream_t s = ctx->stream;
    HIPCHECK(ctx, hipStreamSynchronize(s));
    BcrWork& Bw = ctx->W.bcr;
    Bw.persist = 0;
    Bw.dense1 = 0;  // (k_bcr_dense1 waits only inside its workgroup: a forced spin bound can still time it out)
    ctx->W.sw = 0;  // the small-window Schur launch's envelope tiles wait for its camera side
    ctx->W.tail = 0;  // the band tail's chunks and decision wait for the solve / the chunks
    ctx->W.bsfin = 0;  // the back-substitution launch's decision workgroup waits for its chunks
    ctx->bcr_fallback = true;
    if (Bw.flags) HIPCHECK(ctx, hipMemsetAsync(Bw.flags, 0, sizeof(unsigned) * (16 + 6 * Bw.nblk), s));
    HIPCHECK(ctx, bcr_reset_pull_slots(Bw, false, s));
    // S and rhs as after a prepare: a band-tail chunk whose own wait also timed out may have zeroed S / rhs while
    // the solve workgroup had not yet run, and the solve may then have written y into rhs behind the zeroing
    // (ADVICE r5); the re-run's assembly must start from zeros
    {
        const DevProblem& P = ctx->P;
        HIPCHECK(ctx, hipMemsetAsync(ctx->buf[B_S].p, 0, sizeof(double) * (size_t)P.npad * P.npad, s));
        HIPCHECK(ctx, hipMemsetAsync(ctx->buf[B_RHS].p, 0, sizeof(double) * P.npad, s));
    }
    S.done = 0;
    S.termination = -1;
    S.msg = MSG_NONE;
    static thread_local LmState h_retry;
    h_retry = S;
    HIPCHECK(ctx, hipMemcpyAsync(ctx->W.st, &h_retry, sizeof(LmState), hipMemcpyHostToDevice, s));
    HIPCHECK(ctx, hipStreamSynchronize(s));
    if (ctx->hprog) __atomic_store_n(ctx->hprog, (unsigned)S.n_decide, __ATOMIC_RELEASE);
    ++ctx->bcr_retries;
    return BA_OK;
}

extern "C" int32_t ba_prepare(ba_context* ctx, const ba_problem* p) {
    if (!ctx) { g_err = "null context"; return BA_E_INVALID; }
    miba_maybe_dump_window(p, &ctx->opts);
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    if (int rc = apply_spin_limit(ctx)) return rc;
    const double t0 = now_ms();
    int rc = prepare(ctx, p);
    if (rc) return rc;
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    ctx->pinfo.total_ms = now_ms() - t0;  // device work included
    return BA_OK;
}

// Sized out-structs (BA_API_VERSION 2): the caller's struct_size says how many bytes its struct has; write no more
// than that, keep its struct_size, and refuse a size below the version's minimum.
template <class T>
static bool sized_out_ok(const T* out, int32_t min_size) {
    return out && out->struct_size >= min_size;
}
template <class T>
static void sized_copy_out(T* out, const T& full) {
    const size_t n = std::min<size_t>((size_t)out->struct_size, sizeof(T));
    const int32_t keep = out->struct_size;
    std::memcpy(out, &full, n);
    out->struct_size = keep;
}

extern "C" int32_t ba_last_prepare(const ba_context* ctx, ba_prepare_info* info) {
    if (!ctx || !info) return BA_E_INVALID;
    if (!sized_out_ok(info, BA_PREPARE_INFO_MIN_SIZE)) {
        g_err = "ba_last_prepare: info->struct_size below BA_PREPARE_INFO_MIN_SIZE (set it with BA_PREPARE_INFO_INIT)";
        return BA_E_INVALID;
    }
    sized_copy_out(info, ctx->pinfo);
    return BA_OK;
}

static int32_t solve_prepared(ba_context* ctx, ba_problem* p, ba_summary* sum, double t0);

// the LM loop into a full-size summary, copied out at the caller's size
static int32_t solve_prepared_out(ba_context* ctx, ba_problem* p, ba_summary* out, double t0) {
    ba_summary full{};
    const int32_t rc = solve_prepared(ctx, p, &full, t0);
    full.struct_size = (int32_t)sizeof(ba_summary);
    sized_copy_out(out, full);
    return rc;
}

static const char* const kSummarySizeErr =
    "ba_summary.struct_size below BA_SUMMARY_MIN_SIZE (set it with BA_SUMMARY_INIT)";

extern "C" int32_t ba_solve(ba_context* ctx, ba_problem* p, ba_summary* sum) {
    if (!ctx) { g_err = "null context"; return BA_E_INVALID; }
    if (!sum) { ctx->err = "null summary"; return BA_E_INVALID; }
    if (!sized_out_ok(sum, BA_SUMMARY_MIN_SIZE)) { ctx->err = kSummarySizeErr; return BA_E_INVALID; }
    miba_maybe_dump_window(p, &ctx->opts);
    const double t0 = now_ms();
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    if (int rc = apply_spin_limit(ctx)) return rc;
    int rc = prepare(ctx, p);
    if (rc) return rc;
    return solve_prepared_out(ctx, p, sum, t0);
}

extern "C" int32_t ba_solve_prepared(ba_context* ctx, ba_problem* p, ba_summary* sum) {
    if (!ctx) { g_err = "null context"; return BA_E_INVALID; }
    if (!sum || !p) { ctx->err = "null argument"; return BA_E_INVALID; }
    if (!sized_out_ok(sum, BA_SUMMARY_MIN_SIZE)) { ctx->err = kSummarySizeErr; return BA_E_INVALID; }
    if (!ctx->prepared || p->n_cams != ctx->prep_nc || p->n_points != ctx->prep_np || p->n_obs != ctx->prep_no) {
        ctx->err = "ba_solve_prepared: problem does not match the last ba_prepare()";
        return BA_E_INVALID;
    }
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    return solve_prepared_out(ctx, p, sum, now_ms());
}

static int32_t solve_prepared(ba_context* ctx, ba_problem* p, ba_summary* sum, double t0) {
    std::memset(sum, 0, sizeof(*sum));
    ctx->err.clear();  // ba_last_error() describes this solve from here on
    const ba_options& o = ctx->opts;
    Prof* pf = ctx->pf();
    DevProblem& P = ctx->P;
    DevWork& W = ctx->W;
    const BaConsts& C = ctx->C;
    hipStream_t s = ctx->stream;
    const int max_iter = std::max(o.max_num_iterations, 0);
    HIPCHECK(ctx, ctx->buf[B_LOG].ensure(sizeof(double) * LOG_W * (max_iter + 2)));
    W.log = ctx->buf[B_LOG].as<double>();
    static thread_local LmState h_state;  // host staging (outlives the async copies)
    h_state = fresh_state(o, o.initial_trust_region_radius);
    // the split BCR kernel's flags hold 4 * epoch + panel (one epoch per launch): re-initialise the hand-off
    // state long before 4 * epoch wraps (2^30 launches) on a context that re-solves one prepared window forever
    if (P.solver == 2 && ctx->bcr_launches > (1ull << 28))
        if (int rc = bcr_init_handoffs(ctx)) return rc;
    // start from the parameters of the last ba_prepare() (device-to-device) and a fresh state
    HIPCHECK(ctx, launch_reset(P, W, h_state, ctx->buf[B_CAMS_INIT].as<double>(), ctx->buf[B_PTS_INIT].as<double>(),
                               ctx->buf[B_K_INIT].as<double>(), p->n_cams, ctx->dev_np, s));
    sum->num_obs_admissible = ctx->n_adm_all;
    sum->num_active_cams = P.nac;
    sum->num_active_points = P.n_ap;
    sum->reduced_system_size = P.n;
    sum->linear_solver = P.solver;
    sum->camera_band = P.cam_band;
    const double tl0 = now_ms();
    sum->time_setup_ms = tl0 - t0;
    double kms0[K_COUNT];
    std::memcpy(kms0, ctx->k_ms, sizeof(kms0));

    LmParams prm{};
    prm.min_relative_decrease = o.min_relative_decrease;
    prm.max_radius = o.max_trust_region_radius;
    prm.min_radius = o.min_trust_region_radius;
    prm.function_tolerance = o.function_tolerance;
    prm.gradient_tolerance = o.gradient_tolerance;
    prm.parameter_tolerance = o.parameter_tolerance;
    prm.max_iter = max_iter;
    prm.max_invalid = o.max_num_consecutive_invalid_steps;
    prm.progress = ctx->dprog;
    if (ctx->hprog) __atomic_store_n(ctx->hprog, 0u, __ATOMIC_RELEASE);

    // fused path: S and rhs, the atomic targets of the first assembly (later ones are zeroed in-loop), were
    // zeroed by k_reset
    // IterationZero: cost, gradient, column norms -> Jacobi scale, |x|
    HIPCHECK(ctx, launch_linearize(P, C, 0, W, s, pf));
    HIPCHECK(ctx, launch_scale(P, C, o.jacobi_scaling, W, s, pf));
    HIPCHECK(ctx, launch_init_state(P, W, ctx->hprog ? ctx->dprog : nullptr, s, pf));
    // LM iterations: fixed launch sequence, device-side decisions; the host follows the device.
    // Iterations enqueued after the termination are no-ops (their kernels exit at once).
    int launched = 0;
    int batch = 2;
    int retries = 0;  // decisions that re-ran an iteration after a BCR hand-off timeout (not LM iterations)
    LmState& S = h_state;
    const bool shard = W.comm.on();
    auto launch_iter = [&]() -> int {
        HIPCHECK(ctx, launch_linearize(P, C, 1, W, s, pf));
        HIPCHECK(ctx, launch_build(P, C, W, s, pf));
        HIPCHECK(ctx, launch_factor(P, C, W, s, pf));
        HIPCHECK(ctx, launch_update(P, C, prm, W, s, pf));
        if (P.solver == 2 && W.bcr.persist >= 2) ++ctx->bcr_launches;
        ++launched;
        return BA_OK;
    };
    // at most max_iter + 1 iterations can run (max_iter steps, then the terminal re-linearisation of the
    // stop_next iteration), plus one per re-run iteration
    auto launch_cap = [&]() { return max_iter + 1 + retries; };
    auto is_retry = [](const LmState& st) { return st.done && st.msg == MSG_TIMEOUT && st.termination < 0; };
    if (!pf && ctx->hprog) {
        // Unprofiled: keep LM_AHEAD iterations in flight and follow the device through the host-mapped
        // progress word (n_decide | done << 31, written by every decision and by a failed initial
        // evaluation) instead of synchronising the stream per batch: the GPU never waits for the host.
        // When no launch is allowed and the word has not moved for 2 ms, the host also checks that the stream
        // still runs: an idle or failed stream without a published decision (a device fault) ends the polling
        // instead of spinning. (Not sooner: a hipStreamQuery on a busy stream enqueues a marker behind the
        // last launch, which cost ~5.5 us between k_final and the next iteration's first kernel when it was
        // issued every 256 spins.)
        constexpr int LM_AHEAD = 2;
        volatile unsigned* hp = ctx->hprog;
        for (;;) {
            unsigned w = 0, w_seen = ~0u;
            auto t_seen = std::chrono::steady_clock::now();
            for (;;) {
                w = __atomic_load_n(hp, __ATOMIC_ACQUIRE);
                if (w >> 31) break;
                const auto t_now = std::chrono::steady_clock::now();
                if (w != w_seen) { w_seen = w; t_seen = t_now; }
                // no look-ahead launch past the last iteration that can run
                if (launched - (int)(w & 0x7fffffffu) < LM_AHEAD && launched < launch_cap()) {
                    if (int rc = launch_iter()) return rc;
                } else if (t_now - t_seen > std::chrono::milliseconds(2)) {
                    t_seen = t_now;
                    const hipError_t q = hipStreamQuery(s);
                    if (q == hipSuccess) {  // idle: re-read the word once (it is written before the kernel ends)
                        w = __atomic_load_n(hp, __ATOMIC_ACQUIRE);
                        break;
                    }
                    if (q != hipErrorNotReady) HIPCHECK(ctx, q);
                    std::this_thread::yield();
                } else {
                    std::this_thread::yield();
                }
            }
            // Landmark shards: every iteration issues collectives, so every rank must enqueue the same number
            // of iterations. The decisions are identical on all ranks; the host has enqueued between d and
            // d + LM_AHEAD - 1 iterations when it sees the terminating (or re-run) decision d: pad to
            // d + LM_AHEAD - 1.
            if (shard && (w >> 31)) {
                const int target = std::min((int)(w & 0x7fffffffu) + LM_AHEAD - 1, launch_cap());
                while (launched < target)
                    if (int rc = launch_iter()) return rc;
            }
            if (w >> 31) {  // the terminal state was stored to the host-mapped block before the done bit
                std::memcpy(&S, reinterpret_cast<const char*>(ctx->hprog) + PROG_STATE_OFF, sizeof(LmState));
            } else {
                HIPCHECK(ctx, hipMemcpyAsync(&S, W.st, sizeof(LmState), hipMemcpyDeviceToHost, s));
                HIPCHECK(ctx, hipStreamSynchronize(s));
            }
            if (!is_retry(S)) break;
            if (int rc = bcr_timeout_retry(ctx, S)) return rc;
            ++retries;
            launched = S.n_decide;  // every enqueued iteration has run (the ones behind the decision as no-ops)
        }
    }
    // profiled (HIP events around every launch) or no host-mapped word: batches of iterations, one
    // stream synchronisation per batch (the same batch sizes on every landmark shard)
    for (; !S.done;) {
        for (int i = 0; i < batch && launched <= launch_cap(); ++i)
            if (int rc = launch_iter()) return rc;
        HIPCHECK(ctx, hipMemcpyAsync(&S, W.st, sizeof(LmState), hipMemcpyDeviceToHost, s));
        HIPCHECK(ctx, hipStreamSynchronize(s));
        flush_prof(ctx);
        if (is_retry(S)) {
            if (int rc = bcr_timeout_retry(ctx, S)) return rc;
            ++retries;
            launched = S.n_decide;
            continue;
        }
        if (S.done || launched > launch_cap()) break;
        batch = std::min(batch * 2, 8);
    }
    if (!S.done || S.msg == MSG_TIMEOUT) {  // cannot happen (max_iter bounds the loop; timeouts are re-run)
        ctx->err = "LM loop did not terminate";
        return BA_E_INTERNAL;
    }
    sum->initial_cost = S.initial_cost;
    sum->final_cost = S.final_cost;
    sum->num_successful_steps = S.n_succ;
    sum->num_unsuccessful_steps = S.n_unsucc;
    sum->num_iterations = S.iter;
    sum->termination_type = S.termination;
    ctx->last_iter = S.iter;
    format_message(S, sum->message, sizeof(sum->message));
    if (o.minimizer_progress_to_stdout) {
        std::vector<double> lg((size_t)LOG_W * (S.iter + 1));
        HIPCHECK(ctx, hipMemcpy(lg.data(), W.log, sizeof(double) * lg.size(), hipMemcpyDeviceToHost));
        print_header();
        for (int it = 0; it <= S.iter; ++it) {
            const double* r = &lg[(size_t)it * LOG_W];
            print_row(it, r[0], r[1], r[2], r[3], r[4], r[5], 0.0, 0.0);
        }
    }
    // copy the best (= last accepted) parameters back in place: cameras + intrinsics by DMA into pinned
    // staging (no host-side staging round trip per copy), the points straight into the caller's buffer
    const int cur = S.cur;
    const size_t ncd = 7 * (size_t)p->n_cams;
    if (ctx->hres_cap < ncd + 4) {
        if (ctx->hres) HIPCHECK(ctx, hipHostFree(ctx->hres));
        ctx->hres = nullptr;
        ctx->hres_cap = 0;
        HIPCHECK(ctx, hipHostMalloc((void**)&ctx->hres, sizeof(double) * (ncd + 4), hipHostMallocDefault));
        ctx->hres_cap = ncd + 4;
    }
    if (ncd) HIPCHECK(ctx, hipMemcpyAsync(ctx->hres, P.cams[cur], sizeof(double) * ncd, hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipMemcpyAsync(ctx->hres + ncd, P.K[cur], sizeof(double) * 4, hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipMemcpyAsync(p->points, P.pts[cur] + 3 * (size_t)ctx->gather_off, sizeof(double) * 3 * (size_t)p->n_points,
                                 hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipStreamSynchronize(s));
    if (ncd) std::memcpy(p->cams, ctx->hres, sizeof(double) * ncd);
    std::memcpy(p->intr, ctx->hres + ncd, sizeof(double) * 4);
    const double t1 = now_ms();
    sum->time_lm_ms = t1 - tl0;
    sum->time_total_ms = t1 - t0;
    if (retries)  // informational (rc stays BA_OK): ba_last_error() says why the context left the resident kernel
        ctx->err = std::to_string(retries) + " LM iteration(s) re-run with the per-level BCR launches after an "
                   "inter-workgroup hand-off of the resident BCR kernel timed out; the context keeps the per-level "
                   "launches from now on.";
    auto dk = [&](int k) { return ctx->k_ms[k] - kms0[k]; };
    sum->time_linearize_ms = dk(K_CAM_SIDE) + dk(K_LIN_FINALIZE) + dk(K_POINT_COLNORM) + dk(K_SCALE);
    sum->time_schur_ms = dk(K_MEMSET_S) + dk(K_ASSEMBLE) + dk(K_POINT_PREP) + dk(K_SCHUR_TILE) + dk(K_OBS_PAIRS);
    sum->time_factor_ms = dk(K_CHOL) + dk(K_BCR_ELIM) + dk(K_BCR_CONTRIB) + dk(K_BCR_BACK) + dk(K_BCR_BORDER);
    sum->time_update_ms = dk(K_UPDATE_CAMS) + dk(K_BACKSUB_EVAL) + dk(K_FINAL) + dk(K_DECIDE);
    return BA_OK;
}

extern "C" int32_t ba_debug_linearize(ba_context* ctx, const ba_problem* p, double* cost, double* res, double* jcam,
                                      double* jpt, double* jint) {
    if (!ctx) return BA_E_INVALID;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    int rc = prepare(ctx, p);
    if (rc) return rc;
    DevProblem& P = ctx->P;
    hipStream_t s = ctx->stream;
    const size_t na = P.n_adm;
    HIPCHECK(ctx, ctx->buf[B_DBG0].ensure(sizeof(double) * 3 * na));
    HIPCHECK(ctx, ctx->buf[B_DBG1].ensure(sizeof(double) * 18 * na));
    HIPCHECK(ctx, ctx->buf[B_DBG2].ensure(sizeof(double) * 9 * na));
    HIPCHECK(ctx, ctx->buf[B_DBG3].ensure(sizeof(double) * 8 * na));
    static thread_local LmState h_st;
    h_st = fresh_state(ctx->opts, ctx->opts.initial_trust_region_radius);
    HIPCHECK(ctx, hipMemcpyAsync(ctx->W.st, &h_st, sizeof(LmState), hipMemcpyHostToDevice, s));
    HIPCHECK(ctx, launch_linearize(P, ctx->C, 0, ctx->W, s, nullptr));
    HIPCHECK(ctx, launch_debug_lin(P, ctx->C, ctx->W, ctx->buf[B_DBG0].as<double>(), ctx->buf[B_DBG1].as<double>(),
                                   ctx->buf[B_DBG2].as<double>(), ctx->buf[B_DBG3].as<double>(), s));
    std::vector<double> r(3 * na), jc(18 * na), jp(9 * na), jk(8 * na);
    double lin_h[LIN_N];
    HIPCHECK(ctx, hipMemcpyAsync(r.data(), ctx->buf[B_DBG0].p, sizeof(double) * r.size(), hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipMemcpyAsync(jc.data(), ctx->buf[B_DBG1].p, sizeof(double) * jc.size(), hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipMemcpyAsync(jp.data(), ctx->buf[B_DBG2].p, sizeof(double) * jp.size(), hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipMemcpyAsync(jk.data(), ctx->buf[B_DBG3].p, sizeof(double) * jk.size(), hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipMemcpyAsync(lin_h, ctx->W.lin, sizeof(lin_h), hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipStreamSynchronize(s));
    if (cost) *cost = lin_h[0];
    const size_t no = p->n_obs;
    if (res) std::memset(res, 0, sizeof(double) * 3 * no);
    if (jcam) std::memset(jcam, 0, sizeof(double) * 18 * no);
    if (jpt) std::memset(jpt, 0, sizeof(double) * 9 * no);
    if (jint) std::memset(jint, 0, sizeof(double) * 8 * no);
    // original index -> point-major slot (the plan's po_dest, on the device for both plans)
    std::vector<int> pdest(no);
    if (no) HIPCHECK(ctx, hipMemcpy(pdest.data(), ctx->raw.po_dest, sizeof(int) * no, hipMemcpyDeviceToHost));
    for (size_t k = 0; k < no; ++k) {
        if (pdest[k] < 0) continue;
        const size_t q = pdest[k];
        if (res) std::memcpy(res + 3 * k, &r[3 * q], sizeof(double) * 3);
        if (jcam) std::memcpy(jcam + 18 * k, &jc[18 * q], sizeof(double) * 18);
        if (jpt) std::memcpy(jpt + 9 * k, &jp[9 * q], sizeof(double) * 9);
        if (jint) std::memcpy(jint + 8 * k, &jk[8 * q], sizeof(double) * 8);
    }
    return BA_OK;
}

extern "C" int32_t ba_debug_reduced_system(ba_context* ctx, const ba_problem* p, double radius, int32_t* n_out,
                                           double* S, double* rhs) {
    if (!ctx) return BA_E_INVALID;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    int rc = prepare(ctx, p);
    if (rc) return rc;
    DevProblem& P = ctx->P;
    hipStream_t s = ctx->stream;
    if (n_out) *n_out = P.n;
    if (!S || !rhs) return BA_OK;
    if (radius <= 0) radius = ctx->opts.initial_trust_region_radius;
    static thread_local LmState h_st;
    h_st = fresh_state(ctx->opts, radius);
    HIPCHECK(ctx, hipMemcpyAsync(ctx->W.st, &h_st, sizeof(LmState), hipMemcpyHostToDevice, s));
    HIPCHECK(ctx, launch_linearize(P, ctx->C, 0, ctx->W, s, nullptr));
    HIPCHECK(ctx, launch_scale(P, ctx->C, ctx->opts.jacobi_scaling, ctx->W, s, nullptr));
    HIPCHECK(ctx, launch_build(P, ctx->C, ctx->W, s, nullptr));
    std::vector<double> Sp((size_t)P.npad * P.npad);
    HIPCHECK(ctx, hipMemcpyAsync(Sp.data(), ctx->W.S, sizeof(double) * Sp.size(), hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipMemcpyAsync(rhs, ctx->W.rhs, sizeof(double) * P.n, hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipStreamSynchronize(s));
    const int n = P.n;
    for (int i = 0; i < n; ++i)
        for (int j = 0; j <= i; ++j) {
            const double v = Sp[(size_t)i * P.npad + j];
            S[(size_t)i * n + j] = v;
            S[(size_t)j * n + i] = v;
        }
    return BA_OK;
}

extern "C" int32_t ba_debug_camera_sums(ba_context* ctx, const ba_problem* p, int32_t* nac, double* camdata,
                                        double* lin, int32_t* ac_cam) {
    if (!ctx) return BA_E_INVALID;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    int rc = prepare(ctx, p);
    if (rc) return rc;
    DevProblem& P = ctx->P;
    hipStream_t s = ctx->stream;
    if (nac) *nac = P.nac;
    if (!camdata || !lin) return BA_OK;
    static thread_local LmState h_st;
    h_st = fresh_state(ctx->opts, ctx->opts.initial_trust_region_radius);
    HIPCHECK(ctx, hipMemcpyAsync(ctx->W.st, &h_st, sizeof(LmState), hipMemcpyHostToDevice, s));
    HIPCHECK(ctx, launch_linearize(P, ctx->C, 0, ctx->W, s, nullptr));
    HIPCHECK(ctx, hipMemcpyAsync(camdata, ctx->W.camdata, sizeof(double) * CAMDATA * P.nac, hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipMemcpyAsync(lin, ctx->W.lin, sizeof(double) * LIN_N, hipMemcpyDeviceToHost, s));
    HIPCHECK(ctx, hipStreamSynchronize(s));
    if (ac_cam) std::copy(ctx->ac_cam.begin(), ctx->ac_cam.end(), ac_cam);
    return BA_OK;
}

extern "C" int32_t ba_kernel_stats(const ba_context* ctx, ba_kernel_stat* out, int32_t max_n) {
    if (!ctx || !out) return 0;
    int n = 0;
    for (int k = 0; k < K_COUNT && n < max_n; ++k, ++n) {
        std::memset(&out[n], 0, sizeof(ba_kernel_stat));
        // the resident BCR id times whichever resident kernel the window runs: name it after that kernel
        const char* nm = (k == K_BCR_PERSIST && ctx->W.bcr.band) ? "bcr_band"
                         : (k == K_BCR_PERSIST && ctx->W.bcr.dense1) ? "bcr_dense1"
                         : (k == K_BCR_PERSIST && ctx->W.bcr.persist >= 2) ? "bcr_split" : kKernelNames[k];
        std::snprintf(out[n].name, sizeof(out[n].name), "%s", nm);
        out[n].launches = ctx->k_launches[k];
        out[n].total_ms = ctx->k_ms[k];
        out[n].bytes_per_launch = ctx->k_bytes[k];
        out[n].flops_per_launch = ctx->k_flops[k];
    }
    return n;
}

extern "C" void ba_reset_kernel_stats(ba_context* ctx) {
    if (!ctx) return;
    for (int k = 0; k < K_COUNT; ++k) { ctx->k_launches[k] = 0; ctx->k_ms[k] = 0; }
}

extern "C" int32_t ba_debug_plan_digest(ba_context* ctx, uint64_t* out, int32_t max_n) {
    if (!ctx || !ctx->prepared) return BA_E_INVALID;
    HIPCHECK(ctx, hipSetDevice(ctx->device));
    HIPCHECK(ctx, hipStreamSynchronize(ctx->stream));
    const int n = (int)ctx->plan_parts.size();
    for (int k = 0; k < n && k < max_n; ++k) {
        const auto [off, len] = ctx->plan_parts[k];
        std::vector<int32_t> v(len);
        if (len)
            HIPCHECK(ctx, hipMemcpy(v.data(), ctx->buf[B_PLAN].as<int>() + off, sizeof(int32_t) * len,
                                    hipMemcpyDeviceToHost));
        uint64_t h = 1469598103934665603ull;
        for (int32_t x : v)
            for (int b = 0; b < 4; ++b) h = (h ^ ((uint32_t)x >> (8 * b) & 0xffu)) * 1099511628211ull;
        h = (h ^ (uint64_t)len) * 1099511628211ull;
        out[k] = h;
    }
    return n;
}
