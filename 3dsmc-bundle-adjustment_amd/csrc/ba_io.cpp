// ba_io.cpp — window dump/replay (.miba) and BAL text problems; layout and conventions in
// include/ba_io.h. Host code only (no HIP calls): usable on machines without a GPU.
#include "../../include/ba_io.h"

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ba_host.h"

namespace {

constexpr char kMagic[8] = {'M', 'I', 'B', 'A', 'W', 'I', 'N', '1'};
constexpr size_t kHeaderBytes = 112;

struct Header {
    char magic[8];
    uint32_t version;
    uint32_t options_bytes;
    int32_t n_cams, n_points, n_obs, fixed_cam;
    double intr[4], intr_prior[4];
    uint64_t checksum;
    uint64_t reserved;
};
static_assert(sizeof(Header) == kHeaderBytes, "dump header layout");

int fail(const std::string& m, int rc = BA_E_INVALID) {
    miba_set_error(m);
    return rc;
}

uint64_t fnv1a(const void* data, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* p = static_cast<const unsigned char*>(data);
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 1099511628211ull;
    }
    return h;
}

size_t pad8(size_t n) { return (n + 7) & ~size_t(7); }

struct Section {
    const void* p;
    size_t bytes;
};

std::vector<Section> payload_sections(const ba_problem* p) {
    const size_t nc = p->n_cams, np = p->n_points, no = p->n_obs;
    return {{p->cams, nc * 7 * 8}, {p->points, np * 3 * 8}, {p->obs_uv, no * 2 * 8},
            {p->obs_depth, no * 8},  {p->obs_cam, no * 4},    {p->obs_pt, no * 4}};
}

size_t payload_bytes(int64_t nc, int64_t np, int64_t no) { return pad8(nc * 56 + np * 24 + no * 32); }

bool dims_ok(int64_t nc, int64_t np, int64_t no) { return nc >= 0 && np >= 0 && no >= 0; }

int check_problem(const ba_problem* p) {
    if (!p) return fail("null problem");
    if (!dims_ok(p->n_cams, p->n_points, p->n_obs)) return fail("negative problem size");
    if ((p->n_cams && !p->cams) || (p->n_points && !p->points) || !p->intr || !p->intr_prior ||
        (p->n_obs && (!p->obs_cam || !p->obs_pt || !p->obs_uv || !p->obs_depth)))
        return fail("null array in problem");
    return BA_OK;
}

struct File {
    FILE* f = nullptr;
    explicit File(const char* path, const char* mode) { f = path ? std::fopen(path, mode) : nullptr; }
    ~File() {
        if (f) std::fclose(f);
    }
};

int read_header(FILE* f, const char* path, Header& h) {
    if (std::fread(&h, 1, kHeaderBytes, f) != kHeaderBytes) return fail(std::string(path) + ": truncated header");
    if (std::memcmp(h.magic, kMagic, 8) != 0) return fail(std::string(path) + ": not a .miba window dump");
    if (h.version != BA_DUMP_VERSION)
        return fail(std::string(path) + ": unsupported dump version " + std::to_string(h.version));
    if (!dims_ok(h.n_cams, h.n_points, h.n_obs)) return fail(std::string(path) + ": negative sizes");
    if (h.options_bytes != 0 && h.options_bytes != sizeof(ba_options))
        return fail(std::string(path) + ": options record of " + std::to_string(h.options_bytes) +
                    " bytes does not match this library's ba_options (" + std::to_string(sizeof(ba_options)) + ")");
    return BA_OK;
}

// ---- BAL text ----------------------------------------------------------------------------
struct Text {
    std::string buf;
    const char* p = nullptr;
    const char* end = nullptr;
    bool load(const char* path) {
        File fl(path, "rb");
        if (!fl.f) return false;
        std::fseek(fl.f, 0, SEEK_END);
        long n = std::ftell(fl.f);
        std::fseek(fl.f, 0, SEEK_SET);
        if (n < 0) return false;
        buf.resize((size_t)n);
        if (n && std::fread(&buf[0], 1, (size_t)n, fl.f) != (size_t)n) return false;
        p = buf.c_str();
        end = p + buf.size();
        return true;
    }
    bool num(double& v) {
        char* e = nullptr;
        v = std::strtod(p, &e);
        if (e == p) return false;
        p = e;
        return true;
    }
    bool inum(long long& v) {
        char* e = nullptr;
        errno = 0;
        v = std::strtoll(p, &e, 10);
        if (e == p || errno) return false;
        p = e;
        return true;
    }
};

int bal_dims(Text& t, const char* path, int32_t& nc, int32_t& np, int32_t& no) {
    long long a, b, c;
    if (!t.inum(a) || !t.inum(b) || !t.inum(c)) return fail(std::string(path) + ": missing BAL size line");
    if (a < 0 || b < 0 || c < 0 || a > INT32_MAX || b > INT32_MAX || c > INT32_MAX)
        return fail(std::string(path) + ": BAL sizes out of range");
    nc = (int32_t)a;
    np = (int32_t)b;
    no = (int32_t)c;
    return BA_OK;
}

void quat_mul(const double* a, const double* b, double* o) {  // [x,y,z,w] Hamilton product
    o[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
    o[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
    o[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
    o[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
}

void quat_rotate(const double* q, const double* v, double* o) {  // R(q) v
    const double x = q[0], y = q[1], z = q[2], w = q[3];
    const double u0 = 2 * (y * v[2] - z * v[1]), u1 = 2 * (z * v[0] - x * v[2]), u2 = 2 * (x * v[1] - y * v[0]);
    o[0] = v[0] + w * u0 + (y * u2 - z * u1);
    o[1] = v[1] + w * u1 + (z * u0 - x * u2);
    o[2] = v[2] + w * u2 + (x * u1 - y * u0);
}

void rodrigues_to_quat(const double* r, double* q) {
    const double th = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (th > 0) {
        const double s = std::sin(0.5 * th) / th;
        q[0] = r[0] * s; q[1] = r[1] * s; q[2] = r[2] * s; q[3] = std::cos(0.5 * th);
    } else {
        q[0] = q[1] = q[2] = 0; q[3] = 1;
    }
}

void quat_to_rodrigues(const double* q_in, double* r) {
    double q[4] = {q_in[0], q_in[1], q_in[2], q_in[3]};
    const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    for (double& v : q) v /= n;
    if (q[3] < 0) for (double& v : q) v = -v;
    const double s = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
    const double f = s > 0 ? 2.0 * std::atan2(s, q[3]) / s : 2.0;
    r[0] = q[0] * f; r[1] = q[1] * f; r[2] = q[2] * f;
}

// Undistort a BAL pixel: find p with f (1 + k1|p|^2 + k2|p|^4) p = d (Newton on the radius).
void bal_undistort(double f, double k1, double k2, double dx, double dy, double& px, double& py) {
    const double rd = std::sqrt(dx * dx + dy * dy) / f;
    if (!(rd > 0)) { px = dx / f; py = dy / f; return; }
    double r = rd;
    for (int it = 0; it < 20; ++it) {
        const double r2 = r * r;
        const double g = r * (1 + k1 * r2 + k2 * r2 * r2) - rd;
        const double dg = 1 + 3 * k1 * r2 + 5 * k2 * r2 * r2;
        if (dg == 0) break;
        const double rn = r - g / dg;
        if (rn == r) break;
        r = rn;
    }
    const double s = r / rd / f;
    px = dx * s;
    py = dy * s;
}

constexpr double kQuatFlip[4] = {1, 0, 0, 0};  // rotation by pi about x: diag(1,-1,-1)

}  // namespace

extern "C" int32_t ba_problem_write(const char* path, const ba_problem* p, const ba_options* opts) {
    if (int rc = check_problem(p)) return rc;
    if (!path) return fail("null path");
    Header h{};
    std::memcpy(h.magic, kMagic, 8);
    h.version = BA_DUMP_VERSION;
    h.options_bytes = opts ? (uint32_t)sizeof(ba_options) : 0;
    h.n_cams = p->n_cams; h.n_points = p->n_points; h.n_obs = p->n_obs; h.fixed_cam = p->fixed_cam;
    std::memcpy(h.intr, p->intr, 32);
    std::memcpy(h.intr_prior, p->intr_prior, 32);
    uint64_t c = 1469598103934665603ull;
    size_t raw = 0;
    for (const Section& s : payload_sections(p)) { c = fnv1a(s.p, s.bytes, c); raw += s.bytes; }
    static const char zeros[8] = {0};
    const size_t padn = pad8(raw) - raw;
    c = fnv1a(zeros, padn, c);
    if (opts) c = fnv1a(opts, sizeof(ba_options), c);
    h.checksum = c;
    const std::string tmp = std::string(path) + ".part";
    {
        File fl(tmp.c_str(), "wb");
        if (!fl.f) return fail(std::string("cannot open ") + tmp + ": " + std::strerror(errno));
        bool ok = std::fwrite(&h, 1, kHeaderBytes, fl.f) == kHeaderBytes;
        for (const Section& s : payload_sections(p)) ok = ok && (s.bytes == 0 || std::fwrite(s.p, 1, s.bytes, fl.f) == s.bytes);
        ok = ok && (padn == 0 || std::fwrite(zeros, 1, padn, fl.f) == padn);
        if (opts) ok = ok && std::fwrite(opts, 1, sizeof(ba_options), fl.f) == sizeof(ba_options);
        ok = ok && std::fflush(fl.f) == 0;
        if (!ok) {
            std::remove(tmp.c_str());
            return fail(std::string("write failed: ") + tmp);
        }
    }
    if (std::rename(tmp.c_str(), path) != 0) return fail(std::string("rename failed: ") + path);
    return BA_OK;
}

extern "C" int32_t ba_problem_read_dims(const char* path, int32_t* nc, int32_t* np, int32_t* no) {
    File fl(path, "rb");
    if (!fl.f) return fail(std::string("cannot open ") + (path ? path : "(null)"));
    Header h;
    if (int rc = read_header(fl.f, path, h)) return rc;
    if (nc) *nc = h.n_cams;
    if (np) *np = h.n_points;
    if (no) *no = h.n_obs;
    return BA_OK;
}

extern "C" int32_t ba_problem_read(const char* path, ba_problem* p, ba_options* opts_out) {
    File fl(path, "rb");
    if (!fl.f) return fail(std::string("cannot open ") + (path ? path : "(null)"));
    Header h;
    if (int rc = read_header(fl.f, path, h)) return rc;
    if (!p || p->n_cams != h.n_cams || p->n_points != h.n_points || p->n_obs != h.n_obs)
        return fail(std::string(path) + ": problem buffers are not sized from ba_problem_read_dims");
    if (int rc = check_problem(p)) return rc;
    std::fseek(fl.f, 0, SEEK_END);
    const long fsize = std::ftell(fl.f);
    const size_t want = kHeaderBytes + payload_bytes(h.n_cams, h.n_points, h.n_obs) + h.options_bytes;
    if (fsize < 0 || (size_t)fsize != want)
        return fail(std::string(path) + ": file is " + std::to_string(fsize) + " bytes, header implies " +
                    std::to_string(want));
    std::fseek(fl.f, (long)kHeaderBytes, SEEK_SET);
    uint64_t c = 1469598103934665603ull;
    size_t raw = 0;
    for (const Section& s : payload_sections(p)) {
        if (s.bytes && std::fread(const_cast<void*>(s.p), 1, s.bytes, fl.f) != s.bytes)
            return fail(std::string(path) + ": short read");
        c = fnv1a(s.p, s.bytes, c);
        raw += s.bytes;
    }
    char padb[8];
    const size_t padn = pad8(raw) - raw;
    if (padn && std::fread(padb, 1, padn, fl.f) != padn) return fail(std::string(path) + ": short read");
    c = fnv1a(padb, padn, c);
    ba_options o;
    if (h.options_bytes) {
        if (std::fread(&o, 1, sizeof(o), fl.f) != sizeof(o)) return fail(std::string(path) + ": short read");
        c = fnv1a(&o, sizeof(o), c);
    } else {
        ba_default_options(&o);
    }
    if (c != h.checksum) return fail(std::string(path) + ": checksum mismatch (corrupt dump)");
    for (int32_t k = 0; k < h.n_obs; ++k)
        if (p->obs_cam[k] < 0 || p->obs_cam[k] >= h.n_cams || p->obs_pt[k] < 0 || p->obs_pt[k] >= h.n_points)
            return fail(std::string(path) + ": observation " + std::to_string(k) + " indexes out of range");
    p->fixed_cam = h.fixed_cam;
    std::memcpy(p->intr, h.intr, 32);
    std::memcpy(const_cast<double*>(p->intr_prior), h.intr_prior, 32);
    if (opts_out) *opts_out = o;
    return BA_OK;
}

extern "C" int32_t ba_bal_read_dims(const char* path, int32_t* nc, int32_t* np, int32_t* no) {
    File fl(path, "rb");
    if (!fl.f) return fail(std::string("cannot open ") + (path ? path : "(null)"));
    long long v[3];
    for (long long& x : v)
        if (std::fscanf(fl.f, "%lld", &x) != 1 || x < 0 || x > INT32_MAX)
            return fail(std::string(path) + ": missing BAL size line");
    if (nc) *nc = (int32_t)v[0];
    if (np) *np = (int32_t)v[1];
    if (no) *no = (int32_t)v[2];
    return BA_OK;
}

extern "C" int32_t ba_bal_read(const char* path, ba_problem* p) {
    Text t;
    if (!path || !t.load(path)) return fail(std::string("cannot read ") + (path ? path : "(null)"));
    int32_t nc, np, no;
    if (int rc = bal_dims(t, path, nc, np, no)) return rc;
    if (!p || p->n_cams != nc || p->n_points != np || p->n_obs != no)
        return fail(std::string(path) + ": problem buffers are not sized from ba_bal_read_dims");
    if (int rc = check_problem(p)) return rc;
    std::vector<double> meas((size_t)no * 2);
    for (int32_t k = 0; k < no; ++k) {
        long long c, q;
        if (!t.inum(c) || !t.inum(q) || !t.num(meas[2 * k]) || !t.num(meas[2 * k + 1]))
            return fail(std::string(path) + ": malformed observation " + std::to_string(k));
        if (c < 0 || c >= nc || q < 0 || q >= np)
            return fail(std::string(path) + ": observation " + std::to_string(k) + " indexes out of range");
        const_cast<int32_t*>(p->obs_cam)[k] = (int32_t)c;
        const_cast<int32_t*>(p->obs_pt)[k] = (int32_t)q;
    }
    std::vector<double> cam((size_t)nc * 9);
    for (size_t i = 0; i < cam.size(); ++i)
        if (!t.num(cam[i])) return fail(std::string(path) + ": malformed camera block");
    for (int32_t i = 0; i < np * 3; ++i)
        if (!t.num(p->points[i])) return fail(std::string(path) + ": malformed point block");
    // shared focal = median of the cameras' f
    std::vector<double> fs(nc);
    for (int32_t i = 0; i < nc; ++i) fs[i] = cam[9 * i + 6];
    double f_s = 1.0;
    if (nc) {
        std::sort(fs.begin(), fs.end());
        f_s = (nc % 2) ? fs[nc / 2] : 0.5 * (fs[nc / 2 - 1] + fs[nc / 2]);
    }
    if (!(f_s > 0)) return fail(std::string(path) + ": non-positive focal length");
    for (int32_t i = 0; i < nc; ++i) {
        const double* c = &cam[9 * i];
        double qb[4], qcw[4];
        rodrigues_to_quat(c, qb);
        quat_mul(kQuatFlip, qb, qcw);  // R_cw = diag(1,-1,-1) R
        double* T = p->cams + 7 * i;
        T[0] = -qcw[0]; T[1] = -qcw[1]; T[2] = -qcw[2]; T[3] = qcw[3];  // q_wc = conj(q_cw)
        if (T[3] < 0) for (int j = 0; j < 4; ++j) T[j] = -T[j];
        const double qbc[4] = {-qb[0], -qb[1], -qb[2], qb[3]};
        double tw[3];
        quat_rotate(qbc, c + 3, tw);  // t_wc = -R^T t
        T[4] = -tw[0]; T[5] = -tw[1]; T[6] = -tw[2];
    }
    for (int32_t k = 0; k < no; ++k) {
        const double* c = &cam[9 * (size_t)p->obs_cam[k]];
        double px, py;
        bal_undistort(c[6], c[7], c[8], meas[2 * k], meas[2 * k + 1], px, py);
        double* uv = const_cast<double*>(p->obs_uv) + 2 * k;
        uv[0] = f_s * px;
        uv[1] = -f_s * py;
        double qb[4], P[3];
        rodrigues_to_quat(c, qb);
        quat_rotate(qb, p->points + 3 * (size_t)p->obs_pt[k], P);
        const double z = -(P[2] + c[5]);
        const_cast<double*>(p->obs_depth)[k] = z > 1e-15 ? z : 0.0;
    }
    p->intr[0] = p->intr[1] = f_s;
    p->intr[2] = p->intr[3] = 0.0;
    double* ip = const_cast<double*>(p->intr_prior);
    for (int j = 0; j < 4; ++j) ip[j] = p->intr[j];
    p->fixed_cam = nc > 0 ? 0 : -1;
    return BA_OK;
}

extern "C" int32_t ba_bal_write(const char* path, const ba_problem* p) {
    if (int rc = check_problem(p)) return rc;
    if (!path) return fail("null path");
    File fl(path, "w");
    if (!fl.f) return fail(std::string("cannot open ") + path + ": " + std::strerror(errno));
    FILE* f = fl.f;
    const double fx = p->intr[0], cx = p->intr[2], cy = p->intr[3];
    std::fprintf(f, "%d %d %d\n", p->n_cams, p->n_points, p->n_obs);
    for (int32_t k = 0; k < p->n_obs; ++k)
        std::fprintf(f, "%d %d %.17g %.17g\n", p->obs_cam[k], p->obs_pt[k], p->obs_uv[2 * k] - cx,
                     -(p->obs_uv[2 * k + 1] - cy));
    for (int32_t i = 0; i < p->n_cams; ++i) {
        const double* T = p->cams + 7 * i;
        const double qcw[4] = {-T[0], -T[1], -T[2], T[3]};
        double qb[4], r[3], tcw[3];
        quat_mul(kQuatFlip, qcw, qb);  // R = diag(1,-1,-1) R_cw
        quat_to_rodrigues(qb, r);
        quat_rotate(qcw, T + 4, tcw);  // t_cw = -R_cw t_wc
        const double tb[3] = {-tcw[0], tcw[1], tcw[2]};
        std::fprintf(f, "%.17g\n%.17g\n%.17g\n%.17g\n%.17g\n%.17g\n%.17g\n0\n0\n", r[0], r[1], r[2], tb[0], tb[1], tb[2],
                     fx);
    }
    for (int32_t i = 0; i < p->n_points * 3; ++i) std::fprintf(f, "%.17g\n", p->points[i]);
    if (std::fflush(f) != 0) return fail(std::string("write failed: ") + path);
    return BA_OK;
}

// MIBA_DUMP_DIR capture hook, called by ba_solve / ba_prepare before the window is uploaded.
void miba_maybe_dump_window(const ba_problem* p, const ba_options* o) {
    static std::atomic<int> seq{0};
    const char* dir = std::getenv("MIBA_DUMP_DIR");
    if (!dir || !*dir || !p) return;
    char name[64];
    std::snprintf(name, sizeof(name), "/window_%d_%06d.miba", (int)getpid(), seq.fetch_add(1));
    const std::string path = std::string(dir) + name;
    if (ba_problem_write(path.c_str(), p, o) != BA_OK)
        std::fprintf(stderr, "[miba] MIBA_DUMP_DIR: could not write %s\n", path.c_str());
}
