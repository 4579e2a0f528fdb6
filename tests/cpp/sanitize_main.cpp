// sanitize_main.cpp — host-code sanitizer harness (ASan + UBSan, built by tests/test_sanitizers.py).
//
// Links the host-only window-file code of libmiba (csrc/ba_io.cpp: .miba dump / replay, BAL reader
// and writer, MIBA_DUMP_DIR capture) and the CPU oracle (oracle/ba_oracle.c, test infrastructure),
// both compiled with -fsanitize=address,undefined -fno-sanitize-recover=all, and drives them over
// well-formed and malformed inputs: every truncation of a .miba file, corrupted headers, garbage and
// hostile BAL text. Any out-of-bounds access, leak-free use-after-free or UB aborts the process.
#include <sys/stat.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ba.h"
#include "ba_io.h"

// libmiba's ba_solver.cpp owns the context-free error text; the harness provides it.
static std::string g_last;
void miba_set_error(const std::string& msg) { g_last = msg; }

extern "C" {
void oracle_default_options(ba_options* o);
int oracle_solve(ba_problem* p, const ba_options* opt, ba_summary* sum);
void oracle_config(int32_t threads, int32_t profile);
// ba_solver.cpp's defaults (ceresGlobalProblem + Ceres 2.0); the oracle restates the same values
void ba_default_options(ba_options* o) { oracle_default_options(o); }
}
void miba_maybe_dump_window(const ba_problem* p, const ba_options* o);

static uint64_t g_rng = 0x9e3779b97f4a7c15ull;
static double urand() {  // splitmix64 -> [0, 1)
    uint64_t z = (g_rng += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return (double)((z ^ (z >> 31)) >> 11) * (1.0 / 9007199254740992.0);
}

struct Window {
    std::vector<double> cams, pts, uv, depth;
    std::vector<int32_t> oc, op;
    double intr[4] = {525, 525, 319.5, 239.5}, prior[4] = {525, 525, 319.5, 239.5};
    ba_problem view() {
        ba_problem p{};
        p.n_cams = (int32_t)(cams.size() / 7);
        p.n_points = (int32_t)(pts.size() / 3);
        p.n_obs = (int32_t)oc.size();
        p.fixed_cam = 0;
        p.cams = cams.data();
        p.points = pts.data();
        p.intr = intr;
        p.intr_prior = prior;
        p.obs_cam = oc.data();
        p.obs_pt = op.data();
        p.obs_uv = uv.data();
        p.obs_depth = depth.data();
        return p;
    }
};

// a small window: cameras on a line looking down +z, points in front, each seen by 2-4 cameras
static Window make_window(int nc, int np) {
    Window w;
    for (int c = 0; c < nc; ++c) {
        const double a = 0.01 * (urand() - 0.5);
        w.cams.insert(w.cams.end(), {0.0, std::sin(a), 0.0, std::cos(a), 0.05 * c, 0.01 * urand(), 0.0});
    }
    for (int i = 0; i < np; ++i) {
        const double X[3] = {urand() - 0.5 + 0.05 * nc / 2, urand() - 0.5, 2.0 + urand()};
        w.pts.insert(w.pts.end(), X, X + 3);
        const int k = 2 + (int)(urand() * 3), c0 = (int)(urand() * (nc - k + 1));
        for (int c = c0; c < c0 + k; ++c) {
            const double* T = &w.cams[7 * (size_t)c];
            const double x = X[0] - T[4], y = X[1] - T[5], z = X[2] - T[6];
            w.oc.push_back(c);
            w.op.push_back(i);
            w.uv.push_back(525 * x / z + 319.5 + urand() - 0.5);
            w.uv.push_back(525 * y / z + 239.5 + urand() - 0.5);
            w.depth.push_back(urand() < 0.05 ? 0.0 : z * (1 + 0.01 * (urand() - 0.5)));
        }
    }
    return w;
}

static std::vector<char> slurp(const std::string& path) {
    std::vector<char> b;
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return b;
    char buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) b.insert(b.end(), buf, buf + n);
    std::fclose(f);
    return b;
}
static void spit(const std::string& path, const char* d, size_t n) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { std::perror("fopen"); std::exit(2); }
    if (n) std::fwrite(d, 1, n, f);
    std::fclose(f);
}

#define CHECK(x)                                                              \
    do {                                                                      \
        if (!(x)) {                                                           \
            std::fprintf(stderr, "CHECK failed: %s (line %d)\n", #x, __LINE__); \
            std::exit(3);                                                     \
        }                                                                     \
    } while (0)

// read a file through the dims + read API into owned buffers; returns the read status
static int read_back(const std::string& path, bool bal, Window* out) {
    int32_t nc = 0, np = 0, no = 0;
    int rc = bal ? ba_bal_read_dims(path.c_str(), &nc, &np, &no) : ba_problem_read_dims(path.c_str(), &nc, &np, &no);
    if (rc != BA_OK) return rc;
    if (nc < 0 || np < 0 || no < 0 || nc > (1 << 20) || np > (1 << 22) || no > (1 << 24)) return -100;
    Window w;
    w.cams.resize(7 * (size_t)nc);
    w.pts.resize(3 * (size_t)np);
    w.uv.resize(2 * (size_t)no);
    w.depth.resize(no);
    w.oc.resize(no);
    w.op.resize(no);
    ba_problem p = w.view();
    p.n_cams = nc; p.n_points = np; p.n_obs = no;
    ba_options o;
    rc = bal ? ba_bal_read(path.c_str(), &p) : ba_problem_read(path.c_str(), &p, &o);
    if (out && rc == BA_OK) *out = w;
    return rc;
}

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    Window w = make_window(6, 40);
    ba_problem p = w.view();
    ba_options o;
    oracle_default_options(&o);
    o.minimizer_progress_to_stdout = 0;
    // 1. .miba round trip (with and without options), then every truncation and corrupted headers
    const std::string mf = dir + "/w.miba";
    CHECK(ba_problem_write(mf.c_str(), &p, &o) == BA_OK);
    Window r;
    CHECK(read_back(mf, false, &r) == BA_OK);
    CHECK(r.cams == w.cams && r.pts == w.pts && r.uv == w.uv && r.depth == w.depth && r.oc == w.oc && r.op == w.op);
    const std::vector<char> img = slurp(mf);
    CHECK(!img.empty());
    const std::string tf = dir + "/t.miba";
    int rejected = 0;
    for (size_t n = 0; n < img.size(); n += (n < 160 ? 1 : 37)) {
        spit(tf, img.data(), n);
        rejected += read_back(tf, false, nullptr) != BA_OK;
    }
    CHECK(rejected > 0);
    for (int k = 0; k < 200; ++k) {  // random byte flips: header fields, sizes, checksum, payload
        std::vector<char> b = img;
        const size_t at = k < 120 ? (size_t)k : (size_t)(urand() * b.size());
        b[at] ^= (char)(1 + (int)(urand() * 255));
        spit(tf, b.data(), b.size());
        (void)read_back(tf, false, nullptr);
    }
    // 2. BAL round trip and hostile text
    const std::string bf = dir + "/w.bal";
    CHECK(ba_bal_write(bf.c_str(), &p) == BA_OK);
    CHECK(read_back(bf, true, &r) == BA_OK);
    const char* bad_bal[] = {
        "", "3", "1 1 1\n", "-1 2 3\n", "2 2 2\n0 0 1 2\n", "1 1 1\n0 0 nan inf\n",
        "1 1 1\n5 9 1.0 2.0\n1 2 3 4 5 6 7 8 9\n1 2 3\n", "100000000 100000000 100000000\n",
        "1 1 1\n0 0 1e308 -1e308\n0 0 0 0 0 0 0 0 0\n0 0 0\n",
        "1 1 2\n0 0 1 2\n0 0 3 4\n0.1 0.2 0.3 0 0 0 500 0 0\n1 1 5\n",
    };
    for (const char* t : bad_bal) {
        spit(bf, t, std::strlen(t));
        (void)read_back(bf, true, nullptr);
    }
    // 3. MIBA_DUMP_DIR capture
    setenv("MIBA_DUMP_DIR", dir.c_str(), 1);
    miba_maybe_dump_window(&p, &o);
    unsetenv("MIBA_DUMP_DIR");
    // 4. the oracle on the window read back from disk: 1 thread dense, 3 threads profile
    for (int mode = 0; mode < 2; ++mode) {
        oracle_config(mode ? 3 : 1, mode);
        Window q = make_window(6, 40);
        ba_problem qp = q.view();
        ba_summary s;
        CHECK(oracle_solve(&qp, &o, &s) == 0);
        CHECK(std::isfinite(s.final_cost) && s.final_cost <= s.initial_cost);
    }
    // an all-inadmissible window and an empty one (the IntrinsicsPrior block alone)
    for (int mode = 0; mode < 2; ++mode) {
        Window q = make_window(4, 10);
        for (double& d : q.depth) d = 0.0;
        if (mode) { q.pts.clear(); q.oc.clear(); q.op.clear(); q.uv.clear(); q.depth.clear(); }
        q.intr[2] += 3.0;
        ba_problem qp = q.view();
        ba_summary s;
        CHECK(oracle_solve(&qp, &o, &s) == 0);
        CHECK(std::fabs(q.intr[2] - q.prior[2]) < 1e-2);
    }
    oracle_config(1, 0);
    std::printf("sanitize_main: ok (%d truncations rejected)\n", rejected);
    return 0;
}
