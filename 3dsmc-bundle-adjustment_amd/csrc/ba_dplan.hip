// ba_dplan.hip — the window plan's observation passes on the device (see ba_dplan.h).
//
// The host plan's orderings (ba_plan.cpp), restated as integer passes over HBM:
//   count      per observation: index validation, per-point counts (one atomic per run of equal points in a
//              wave), per-range camera histograms (LDS; a range is one wave's ro observations)
//   cameras    the histograms' row scans -> per-camera counts and camera-major segment starts; active cameras
//   lists      point lists (atomic slots), each sorted on the unique key (active camera + 1, observation index):
//              registers for <= 16 observations, one workgroup's LDS for longer lists; first / last active
//              camera, duplicate links and the point class (tiled / overflow / gauge-only) from the sorted list
//   orders     camera-major (stable bucket scatter by camera, index order) and the active point order (stable
//              bucket scatter by class and first camera, point order): one wave per range ranks each item among
//              the equal buckets before it (ballot match), so both are the host's total orders
//   point-major the sorted lists in the active point order; the overflow slots on active cameras
// Prefix sums are single-pass (each block's exclusive prefix from its predecessors' published aggregates, blocks
// ordered by a ticket). One summary goes back to the host. Every pass is O(observations), 16 launches, no host
// sync between them; admissibility comes in as one byte per observation (the host computes it while staging), so
// the passes read neither depths nor pixels, whose DMA runs beside them on the copy stream.
#include "ba_dplan.h"

#include <algorithm>
#include <climits>

namespace miba {
namespace {

constexpr int TPB = 256;
constexpr int SCAN_ITEMS = 4;                 // per thread; a scan block covers TPB * SCAN_ITEMS items
constexpr int SCAN_BLK = TPB * SCAN_ITEMS;
constexpr int SHORT_MAX = 16;                 // point lists sorted in registers
constexpr unsigned SPIN_MAX = 1u << 20;       // look-back polls before a scan gives up (DP_TOOLONG: host plan)
constexpr long long HIST_MAX = 1LL << 22;     // bucket histogram entries (ranges x buckets)

// every device pointer of the plan (kernel argument, by value)
struct DP {
    const int* cam; const int* pt; const unsigned char* adm;
    int no, np, nc, fixed_cam, tile_win, chunk_obs;
    int ro, rp, nwo, nwp;                     // observations / points per range, ranges
    int* po_dest; int* co_dest; int* cam_ac; int* pt_idx; int* ovf_obs;
    int* hdr; int* cam_cnt; int* fc; int* pt_ptr; int* pmm;
    int* pt_cnt; int* pptr; int* cursor; int* plist; int* pmin; int* pmax; int* pbk;
    int* Hc; int* Tc; int* Bc; int* Hp; int* Tp;
    int* co_orig; int* po_orig; int* longl;
    unsigned long long* status;               // [3][nsb] look-back words of the three scans
    int* ticket;                              // [3]
    int nsb;
};

// exclusive scan of one int per thread over the block (TPB threads); total = the block's sum
__device__ inline int block_excl(int v, int* sh, int& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int j = 0; j < TPB / 64; ++j) {
        const int s = sh[j];
        off += j < w ? s : 0;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return off + x - v;
}

// exclusive scan of one int per lane over the wave; total = the wave's sum
__device__ inline int wave_excl(int v, int& total) {
    const int lane = threadIdx.x & 63;
    int x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    total = __shfl(x, 63, 64);
    return x - v;
}

// runs of equal values among consecutive lanes: whether this lane starts one, the run's first lane, its length
struct Run { bool head; int first, len; };
__device__ inline Run lane_run(int v) {
    const int lane = threadIdx.x & 63;
    const int prev = __shfl_up(v, 1, 64);
    const unsigned long long b = __ballot(lane == 0 || v != prev);
    Run r;
    r.head = (b >> lane) & 1ull;
    r.first = 63 - __clzll(b & ((2ull << lane) - 1ull));
    const unsigned long long after = lane == 63 ? 0ull : b >> (lane + 1);
    r.len = (after ? lane + __ffsll((long long)after) : 64) - lane;
    return r;
}

__global__ __launch_bounds__(TPB) void k_dp_init(DP d) {
    const int i = blockIdx.x * TPB + threadIdx.x;
    if (i <= d.np) d.pt_cnt[i] = 0;
    if (i < d.np) d.cursor[i] = 0;
    if (i < DP_HDR) d.hdr[i] = (i == DP_BAD) ? INT_MAX : 0;
    if (i < 3 * d.nsb) d.status[i] = 0ull;
    if (i < 3) d.ticket[i] = 0;
}

// pass 1 over the observations, one wave per range: validation, per-point counts, the range's camera histogram
__global__ __launch_bounds__(64) void k_dp_count(DP d) {
    extern __shared__ int hist[];
    const int w = blockIdx.x, lane = threadIdx.x;
    for (int c = lane; c < d.nc; c += 64) hist[c] = 0;
    __syncthreads();
    const int lo = w * d.ro, hi = min(d.no, lo + d.ro);
    int nadm = 0;
    for (int base = lo; base < hi; base += 64) {
        const int k = base + lane;
        int c = -1, p = -1;
        if (k < hi) {
            const int c0 = d.cam[k], p0 = d.pt[k];
            if (c0 < 0 || c0 >= d.nc || p0 < 0 || p0 >= d.np) atomicMin(&d.hdr[DP_BAD], k);
            else if (d.adm[k]) { c = c0; p = p0; ++nadm; }
        }
        const Run rp = lane_run(p);
        if (rp.head && p >= 0) atomicAdd(&d.pt_cnt[p], rp.len);
        const Run rc = lane_run(c);
        if (rc.head && c >= 0) atomicAdd(&hist[c], rc.len);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) nadm += __shfl_xor(nadm, o, 64);
    if (lane == 0 && nadm) atomicAdd(&d.hdr[DP_NADM], nadm);
    __syncthreads();
    for (int c = lane; c < d.nc; c += 64) d.Hc[(size_t)c * d.nwo + w] = hist[c];
}

// the point buckets' histogram of one range of points: bucket = class 0: first camera; class 1: nc + first
// camera; class 2: 2 nc (host plan: tiled by first camera, overflow by first camera, gauge-only; point order)
__global__ __launch_bounds__(64) void k_dp_count_points(DP d) {
    extern __shared__ int hist[];
    const int w = blockIdx.x, lane = threadIdx.x, nbk = 2 * d.nc + 1;
    for (int c = lane; c < nbk; c += 64) hist[c] = 0;
    __syncthreads();
    const int lo = w * d.rp, hi = min(d.np, lo + d.rp);
    for (int base = lo; base < hi; base += 64) {
        const int i = base + lane;
        const int b = i < hi ? d.pbk[i] : -1;
        const Run r = lane_run(b);
        if (r.head && b >= 0) atomicAdd(&hist[b], r.len);
    }
    __syncthreads();
    for (int c = lane; c < nbk; c += 64) d.Hp[(size_t)c * d.nwp + w] = hist[c];
}

// row b of a bucket histogram H[b][nw]: exclusive scan in place, T[b] = the bucket's total
__global__ __launch_bounds__(TPB) void k_dp_rowscan(int* H, int nw, int* T) {
    __shared__ int sh[TPB / 64];
    int* row = H + (size_t)blockIdx.x * nw;
    int carry = 0;
    for (int base = 0; base < nw; base += TPB) {
        const int j = base + threadIdx.x;
        const int v = j < nw ? row[j] : 0;
        int tot;
        const int e = block_excl(v, sh, tot);
        if (j < nw) row[j] = carry + e;
        carry += tot;
    }
    if (threadIdx.x == 0) T[blockIdx.x] = carry;
}

// cameras: counts (summary), camera-major segment starts, active cameras (observed, not the gauge), fc[a] = a
__global__ __launch_bounds__(TPB) void k_dp_cams(DP d) {
    __shared__ int sh[TPB / 64];
    int cb = 0, ca = 0;
    for (int base = 0; base < d.nc; base += TPB) {
        const int c = base + threadIdx.x;
        const int cnt = c < d.nc ? d.Tc[c] : 0;
        const int act = (c < d.nc && cnt > 0 && c != d.fixed_cam) ? 1 : 0;
        int tb, ta;
        const int eb = block_excl(cnt, sh, tb);
        const int ea = block_excl(act, sh, ta);
        if (c < d.nc) {
            d.Bc[c] = cb + eb;
            d.cam_cnt[c] = cnt;
            d.cam_ac[c] = act ? ca + ea : -1;
            if (act) d.fc[ca + ea] = ca + ea;
        }
        cb += tb;
        ca += ta;
    }
    if (threadIdx.x == 0) d.hdr[DP_NAC] = ca;
}

// ---- single-pass scans over n items in blocks of SCAN_BLK (blocks ordered by a ticket; each publishes its
// aggregate, then its inclusive prefix once the predecessors' are known: flag 1 / 2 in the high word)
enum { SM_PPTR = 0, SM_PTPTR, SM_OVF };

template <int MODE>
__device__ inline int scan_in(const DP& d, int i) {
    if (MODE == SM_PPTR) return i < d.np ? d.pt_cnt[i] : 0;
    if (MODE == SM_PTPTR) return i < d.hdr[DP_NAP] ? d.pt_cnt[d.pt_idx[i]] : 0;
    // SM_OVF: point-major slots of overflow points (after the tiled ones) whose camera is active
    if (i >= d.no) return 0;
    const int q0 = d.pt_ptr[d.hdr[DP_NTILED]], q1 = d.pt_ptr[d.hdr[DP_NAP]];
    if (i < q0 || i >= q1) return 0;
    return d.cam_ac[d.cam[d.po_orig[i]]] >= 0 ? 1 : 0;
}

template <int MODE>
__global__ __launch_bounds__(TPB) void k_dp_scan(DP d, int n) {
    __shared__ int sh[TPB / 64];
    __shared__ int s_blk, s_excl;
    unsigned long long* st = d.status + (size_t)MODE * d.nsb;
    if (threadIdx.x == 0) s_blk = atomicAdd(&d.ticket[MODE], 1);
    __syncthreads();
    const int blk = s_blk;
    const int base = blk * SCAN_BLK + threadIdx.x * SCAN_ITEMS;
    int v[SCAN_ITEMS], s = 0;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        v[j] = base + j < n ? scan_in<MODE>(d, base + j) : 0;
        s += v[j];
    }
    int tot;
    const int pre = block_excl(s, sh, tot);
    if (threadIdx.x == 0) {
        int excl = 0;
        if (blk > 0) {
            __hip_atomic_store(&st[blk], (1ull << 32) | (unsigned)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            unsigned spins = 0;
            for (int j = blk - 1; j >= 0;) {
                const unsigned long long w = __hip_atomic_load(&st[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned f = (unsigned)(w >> 32);
                if (f == 0) {  // the predecessor holds a smaller ticket, so it runs: wait for its aggregate
                    if (++spins > SPIN_MAX) { atomicOr(&d.hdr[DP_TOOLONG], 2); break; }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += (int)(unsigned)w;
                if (f == 2) break;
                --j;
            }
        }
        __hip_atomic_store(&st[blk], (2ull << 32) | (unsigned)(excl + tot), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        s_excl = excl;
    }
    __syncthreads();
    int run = s_excl + pre;
#pragma unroll
    for (int j = 0; j < SCAN_ITEMS; ++j) {
        const int i = base + j;
        if (i < n) {
            if (MODE == SM_PPTR) d.pptr[i] = run;
            else if (MODE == SM_PTPTR) d.pt_ptr[i] = run;
            else {
                if (v[j]) d.ovf_obs[run] = i;
                if (i == n - 1) d.hdr[DP_NOVF] = run + v[j];
            }
        }
        run += v[j];
    }
}

// pass 2: each admissible observation into a slot of its point's list (one atomic per run of equal points; the
// list order is fixed by the sort below)
__global__ __launch_bounds__(TPB) void k_dp_fill(DP d) {
    const int k = blockIdx.x * TPB + threadIdx.x;
    int p = -1;
    if (k < d.no) {
        const int c = d.cam[k], p0 = d.pt[k];
        if (c >= 0 && c < d.nc && p0 >= 0 && p0 < d.np && d.adm[k]) p = p0;
    }
    const Run r = lane_run(p);
    int slot = (r.head && p >= 0) ? atomicAdd(&d.cursor[p], r.len) : 0;
    slot = __shfl(slot, r.first, 64) + ((int)(threadIdx.x & 63) - r.first);
    if (p >= 0) d.plist[d.pptr[p] + slot] = k;
}

__device__ inline unsigned long long pkey(const DP& d, int k) {
    return ((unsigned long long)(unsigned)(d.cam_ac[d.cam[k]] + 1) << 32) | (unsigned)k;
}

// the point's class and bucket from its sorted list (host plan: ba_plan.cpp point_sort_class)
__device__ inline void point_class(const DP& d, int i, int m, int lo, int hi, bool dup) {
    d.pmin[i] = lo;
    d.pmax[i] = hi;
    int b;
    if (hi < 0) b = 2 * d.nc;                                                   // gauge-only
    else if (dup || hi - lo + 1 > d.tile_win || m > d.chunk_obs) b = d.nc + lo;  // overflow
    else b = lo;                                                                 // tiled
    d.pbk[i] = b;
}

// per point: sort the list on (active camera + 1, observation index) — registers for <= SHORT_MAX observations,
// longer lists queued for k_dp_psort_long
__global__ __launch_bounds__(TPB) void k_dp_psort(DP d) {
    const int i = blockIdx.x * TPB + threadIdx.x;
    if (i >= d.np) return;
    const int m = d.pt_cnt[i];
    if (m == 0) {
        d.pmin[i] = INT_MAX;
        d.pmax[i] = -1;
        d.pbk[i] = -1;
        return;
    }
    if (m > SHORT_MAX) {
        d.longl[atomicAdd(&d.hdr[DP_NLONG], 1)] = i;
        return;
    }
    int* L = d.plist + d.pptr[i];
    unsigned long long v[SHORT_MAX];
#pragma unroll
    for (int j = 0; j < SHORT_MAX; ++j) v[j] = j < m ? pkey(d, L[j]) : ~0ull;
    // odd-even transposition network (the padding sorts last)
#pragma unroll
    for (int r = 0; r < SHORT_MAX; ++r) {
#pragma unroll
        for (int j = r & 1; j + 1 < SHORT_MAX; j += 2) {
            const unsigned long long a = v[j], b = v[j + 1];
            const bool sw = a > b;
            v[j] = sw ? b : a;
            v[j + 1] = sw ? a : b;
        }
    }
    int lo = INT_MAX, hi = -1, prev = -2;
    bool dup = false;
#pragma unroll
    for (int j = 0; j < SHORT_MAX; ++j) {
        if (j < m) {
            L[j] = (int)(unsigned)(v[j] & 0xffffffffull);
            const int a = (int)(v[j] >> 32) - 1;
            if (a >= 0) {
                lo = min(lo, a);
                hi = max(hi, a);
                dup = dup || a == prev;
                prev = a;
            }
        }
    }
    point_class(d, i, m, lo, hi, dup);
}

// lists of more than SHORT_MAX observations: one workgroup each, rank sort in LDS (the keys are unique);
// a duplicate link is a second key with the same camera
__global__ __launch_bounds__(TPB) void k_dp_psort_long(DP d) {
    __shared__ unsigned long long key[DP_LONG_MAX];
    __shared__ int red[3];
    const int nl = d.hdr[DP_NLONG];
    for (int t = blockIdx.x; t < nl; t += gridDim.x) {
        const int i = d.longl[t];
        const int m = d.pt_cnt[i];
        if (m > DP_LONG_MAX) {  // the host plan rebuilds the window; the passes below skip the point
            if (threadIdx.x == 0) {
                atomicOr(&d.hdr[DP_TOOLONG], 1);
                d.pmin[i] = INT_MAX;
                d.pmax[i] = -1;
                d.pbk[i] = -1;
            }
            continue;
        }
        int* L = d.plist + d.pptr[i];
        if (threadIdx.x == 0) { red[0] = INT_MAX; red[1] = -1; red[2] = 0; }
        for (int j = threadIdx.x; j < m; j += TPB) key[j] = pkey(d, L[j]);
        __syncthreads();
        int lo = INT_MAX, hi = -1, dup = 0;
        for (int j = threadIdx.x; j < m; j += TPB) {
            const unsigned long long kj = key[j];
            const unsigned cj = (unsigned)(kj >> 32);
            int r = 0, same = 0;
            for (int q = 0; q < m; ++q) {
                const unsigned long long kq = key[q];
                r += kq < kj ? 1 : 0;
                same += (unsigned)(kq >> 32) == cj ? 1 : 0;
            }
            L[r] = (int)(unsigned)(kj & 0xffffffffull);
            const int a = (int)cj - 1;
            if (a >= 0) {
                lo = min(lo, a);
                hi = max(hi, a);
                dup |= same > 1 ? 1 : 0;
            }
        }
        atomicMin(&red[0], lo);
        atomicMax(&red[1], hi);
        if (dup) atomicOr(&red[2], 1);
        __syncthreads();
        if (threadIdx.x == 0) point_class(d, i, m, red[0], red[1], red[2] != 0);
        __syncthreads();
    }
}

// stable bucket scatter of one range by one wave, in index order: each item's rank among the equal buckets
// before it in its 64-item chunk (ballot match) + the bucket's count in the earlier chunks (LDS) + the range's
// offset in the bucket (row-scanned histogram) + the bucket's start (the points' starts scanned here, in LDS)
template <bool OBS>
__global__ __launch_bounds__(64) void k_dp_scatter(DP d) {
    extern __shared__ int lds[];
    const int w = blockIdx.x, lane = threadIdx.x;
    const int nbk = OBS ? d.nc : 2 * d.nc + 1;
    const int nw = OBS ? d.nwo : d.nwp;
    const int r = OBS ? d.ro : d.rp;
    const int* H = OBS ? d.Hc : d.Hp;
    int* run = lds;
    int* start = lds + nbk;  // points: bucket starts
    for (int c = lane; c < nbk; c += 64) run[c] = 0;
    if (!OBS) {
        int carry = 0;
        for (int base = 0; base < nbk; base += 64) {
            const int c = base + lane;
            int tot;
            const int e = wave_excl(c < nbk ? d.Tp[c] : 0, tot);
            if (c < nbk) start[c] = carry + e;
            carry += tot;
        }
        if (w == 0 && lane == 0) {
            d.hdr[DP_NAP] = carry;
            d.hdr[DP_NTILED] = start[d.nc];
        }
    }
    __syncthreads();
    const int* B = OBS ? d.Bc : start;
    const int lo = w * r, hi = min(OBS ? d.no : d.np, lo + r);
    const unsigned long long lt = (1ull << lane) - 1;
    for (int base = lo; base < hi; base += 64) {
        const int i = base + lane;
        int b = -1;
        if (i < hi) {
            if (OBS) {
                const int c = d.cam[i], p = d.pt[i];
                if (c >= 0 && c < d.nc && p >= 0 && p < d.np && d.adm[i]) b = c;
                else {
                    d.co_dest[i] = -1;
                    d.po_dest[i] = -1;
                }
            } else {
                b = d.pbk[i];
            }
        }
        unsigned long long pend = __ballot(b >= 0);
        while (pend) {
            const int leader = __ffsll((long long)pend) - 1;
            const int vb = __builtin_amdgcn_readlane(b, leader);
            const unsigned long long mk = __ballot(b == vb);
            if (b == vb) {
                const int pos = B[vb] + H[(size_t)vb * nw + w] + run[vb] + __popcll(mk & lt);
                if (OBS) {
                    d.co_orig[pos] = i;
                    d.co_dest[i] = pos;
                } else {
                    d.pt_idx[pos] = i;
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (lane == leader) run[vb] += __popcll(mk);
            __builtin_amdgcn_wave_barrier();
            pend &= ~mk;
        }
    }
}

// first co-visible active camera of each active camera: min over its observations of their points' first camera
// (FC_SPLIT workgroups per camera, atomicMin into fc[a] = a)
constexpr int FC_SPLIT = 8;
__global__ __launch_bounds__(TPB) void k_dp_fc(DP d) {
    const int c = blockIdx.x / FC_SPLIT, part = blockIdx.x % FC_SPLIT;
    const int a = d.cam_ac[c];
    if (a < 0) return;
    const int q0 = d.Bc[c], n = d.Tc[c];
    int m = INT_MAX;
    for (int j = part * TPB + threadIdx.x; j < n; j += FC_SPLIT * TPB) m = min(m, d.pmin[d.pt[d.co_orig[q0 + j]]]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = min(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0 && m < a) atomicMin(&d.fc[a], m);
}

// point-major observations (each active point's sorted list at its slot range) and the summary's per-point
// column: first / last active camera (16 bits each)
__global__ __launch_bounds__(TPB) void k_dp_pmajor(DP d) {
    const int a = blockIdx.x * TPB + threadIdx.x;
    if (a >= d.np) return;
    if (a >= d.hdr[DP_NAP]) {
        d.pmm[a] = 0;
        return;
    }
    const int i = d.pt_idx[a];
    d.pmm[a] = (int)(((unsigned)d.pmin[i] << 16) | ((unsigned)d.pmax[i] & 0xffffu));
    const int m = d.pt_cnt[i];
    const int* L = d.plist + d.pptr[i];
    const int q0 = d.pt_ptr[a];
    for (int j = 0; j < m; ++j) {
        const int k = L[j];
        d.po_orig[q0 + j] = k;
        d.po_dest[k] = q0 + j;
    }
}

// the summary's live ranges into mapped host memory (the host reads it after the stream's work is done): header,
// camera counts, fc of the active cameras, pt_ptr of the active points, the tiled points' camera ranges
__global__ __launch_bounds__(TPB) void k_dp_publish(DP d, int* out) {
    const int i = blockIdx.x * TPB + threadIdx.x;
    const int nc = d.nc, np = d.np;
    const int o_fc = DP_HDR + nc, o_ptp = o_fc + nc, o_pmm = o_ptp + np + 1;
    bool live;
    if (i < o_fc) live = true;
    else if (i < o_ptp) live = i - o_fc < d.hdr[DP_NAC];
    else if (i < o_pmm) live = i - o_ptp <= d.hdr[DP_NAP];
    else live = i - o_pmm < d.hdr[DP_NTILED];
    if (live && i < o_pmm + np) out[i] = d.hdr[i];
}

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// items per range: 256, doubled while the histogram (ranges x buckets) exceeds HIST_MAX entries
inline int range_items(int n, int nbk) {
    int r = 256;
    while ((long long)cdiv(n, r) * nbk > HIST_MAX && r < (1 << 20)) r *= 2;
    return r;
}

struct Geo {
    int ro, rp, nwo, nwp, nsb;
    Geo(int no, int np, int nc) {
        ro = range_items(no, nc);
        rp = range_items(np, 2 * nc + 1);
        nwo = std::max(1, cdiv(no, ro));
        nwp = std::max(1, cdiv(np, rp));
        nsb = cdiv((long long)std::max(no, np) + 1, SCAN_BLK) + 1;
    }
};

}  // namespace

size_t dplan_scratch_ints(int no, int np, int nc) {
    const Geo g(no, np, nc);
    const size_t nbp = 2 * (size_t)nc + 1;
    return 3 * ((size_t)np + 1) + 4 * (size_t)np + 3 * (size_t)no + (size_t)nc * g.nwo + 3 * (size_t)nc +
           nbp * g.nwp + nbp + 2 * 3 * (size_t)g.nsb + 64;
}

bool dplan_fits(int no, int np, int nc) {
    // the points' scatter keeps run counters and starts for 2 nc + 1 buckets in 64 KB of LDS
    return no > 0 && np > 0 && nc > 0 && nc <= 4000 && no < (1 << 30);
}

hipError_t dplan_enqueue(const DPlanArgs& a, hipStream_t s) {
    const Geo g(a.no, a.np, a.nc);
    DP d{};
    d.cam = a.cam; d.pt = a.pt; d.adm = a.adm;
    d.no = a.no; d.np = a.np; d.nc = a.nc; d.fixed_cam = a.fixed_cam; d.tile_win = a.tile_win;
    d.chunk_obs = a.chunk_obs;
    d.ro = g.ro; d.rp = g.rp; d.nwo = g.nwo; d.nwp = g.nwp; d.nsb = g.nsb;
    d.po_dest = a.po_dest; d.co_dest = a.co_dest; d.cam_ac = a.cam_ac; d.pt_idx = a.pt_idx; d.ovf_obs = a.ovf_obs;
    d.hdr = a.sum;
    d.cam_cnt = d.hdr + DP_HDR;
    d.fc = d.cam_cnt + a.nc;
    d.pt_ptr = d.fc + a.nc;
    d.pmm = d.pt_ptr + a.np + 1;
    const int nbp = 2 * a.nc + 1;
    int* p = a.scratch;
    auto take = [&](size_t n) { int* r = p; p += n; return r; };
    d.status = reinterpret_cast<unsigned long long*>(take(2 * 3 * (size_t)g.nsb + 2));  // scratch is 256-B aligned
    d.ticket = take(4);
    d.pt_cnt = take(a.np + 1); d.pptr = take(a.np + 1); d.cursor = take(a.np);
    d.pmin = take(a.np); d.pmax = take(a.np); d.pbk = take(a.np); d.longl = take(a.np);
    d.plist = take(a.no); d.co_orig = take(a.no); d.po_orig = take(a.no);
    d.Hc = take((size_t)a.nc * g.nwo); d.Tc = take(a.nc); d.Bc = take(a.nc);
    d.Hp = take((size_t)nbp * g.nwp); d.Tp = take(nbp);

    const int ninit = std::max(std::max(a.np + 1, (int)DP_HDR), 3 * g.nsb);
    k_dp_init<<<cdiv(ninit, TPB), TPB, 0, s>>>(d);
    k_dp_count<<<g.nwo, 64, sizeof(int) * a.nc, s>>>(d);
    k_dp_rowscan<<<a.nc, TPB, 0, s>>>(d.Hc, g.nwo, d.Tc);
    k_dp_cams<<<1, TPB, 0, s>>>(d);
    k_dp_scan<SM_PPTR><<<cdiv((long long)a.np + 1, SCAN_BLK), TPB, 0, s>>>(d, a.np + 1);
    k_dp_fill<<<cdiv(a.no, TPB), TPB, 0, s>>>(d);
    k_dp_psort<<<cdiv(a.np, TPB), TPB, 0, s>>>(d);
    k_dp_psort_long<<<256, TPB, 0, s>>>(d);
    k_dp_scatter<true><<<g.nwo, 64, sizeof(int) * a.nc, s>>>(d);
    k_dp_fc<<<a.nc * FC_SPLIT, TPB, 0, s>>>(d);
    k_dp_count_points<<<g.nwp, 64, sizeof(int) * nbp, s>>>(d);
    k_dp_rowscan<<<nbp, TPB, 0, s>>>(d.Hp, g.nwp, d.Tp);
    k_dp_scatter<false><<<g.nwp, 64, 2 * sizeof(int) * nbp, s>>>(d);
    k_dp_scan<SM_PTPTR><<<cdiv((long long)a.np + 1, SCAN_BLK), TPB, 0, s>>>(d, a.np + 1);
    k_dp_pmajor<<<cdiv(a.np, TPB), TPB, 0, s>>>(d);
    k_dp_scan<SM_OVF><<<cdiv((long long)a.no + 1, SCAN_BLK), TPB, 0, s>>>(d, a.no + 1);
    if (a.sum_host) k_dp_publish<<<cdiv((long long)dplan_sum_ints(a.nc, a.np), TPB), TPB, 0, s>>>(d, a.sum_host);
    return hipGetLastError();
}

}  // namespace miba
