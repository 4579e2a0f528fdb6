// handoff_probe.hip — one-way latency of an in-launch hand-off between two workgroups (the BCR's store -> poll
// protocol), by XCD placement and load / store cache policy. Workgroup b of a launch runs on XCD (b mod 8)
// (round-robin dispatch; the probe prints every workgroup's HW_REG_XCC_ID to check it). Two workgroups ping-pong
// N rounds through two 8-byte slots: A stores k, B polls until it reads k and stores k, A polls for it, ...
// one-way latency = elapsed / (2 N). Policies (load, store):
//   0  agent-scope relaxed atomic load / store (the kernels' ld_u64 / st_pub)
//   1  global_load sc0 (L1 bypass) / global_store sc0
//   2  global_load sc0 sc1 / global_store sc0 sc1 (system scope)
// build: hipcc --offload-arch=gfx950 -O3 tools/handoff_probe.hip -o tools/_build/hop
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((address_space(1))) unsigned long long gu64;

__device__ __forceinline__ unsigned long long rt() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
template <int POL>
__device__ __forceinline__ unsigned long long ld(unsigned long long* p) {
    if constexpr (POL == 0) {
        return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        unsigned long long v;
        if constexpr (POL == 1)
            asm volatile("global_load_dwordx2 %0, %1, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
        else
            asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
        return v;
    }
}
template <int POL>
__device__ __forceinline__ void st(unsigned long long* p, unsigned long long v) {
    if constexpr (POL == 0) {
        __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if constexpr (POL == 1) {
        asm volatile("global_store_dwordx2 %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
    } else {
        asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    }
}

template <int POL>
__global__ __launch_bounds__(64) void k_pingpong(unsigned long long* slots, int a, int b, int n,
                                                 unsigned long long* out, unsigned* xcc) {
    const int w = blockIdx.x;
    if (threadIdx.x == 0) {
        unsigned id;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
        xcc[w] = id;
    }
    if (w != a && w != b) return;
    if (threadIdx.x != 0) return;
    unsigned long long* mine = slots + (w == a ? 0 : 16);
    unsigned long long* other = slots + (w == a ? 16 : 0);
    const unsigned long long t0 = rt();
    unsigned long long fails = 0;
    for (int k = 1; k <= n && fails < 3; ++k) {
        if (w == a) {
            st<POL>(mine, (unsigned long long)k);
            unsigned long long g = 0;
            for (unsigned s = 0; (g = ld<POL>(other)) != (unsigned long long)k; ++s)
                if (s > (1u << 18)) { ++fails; break; }
        } else {
            unsigned long long g = 0;
            for (unsigned s = 0; (g = ld<POL>(other)) != (unsigned long long)k; ++s)
                if (s > (1u << 18)) { ++fails; break; }
            st<POL>(mine, (unsigned long long)k);
        }
    }
    const unsigned long long t1 = rt();
    if (w == a) { out[0] = t1 - t0; out[1] = fails; }
}

int main() {
    const int nwg = 16, n = 2000;
    unsigned long long *slots, *out;
    unsigned* xcc;
    (void)hipMalloc(&slots, 4096);
    (void)hipMalloc(&out, 64);
    (void)hipMalloc(&xcc, 4 * nwg);
    const int pairs[3][2] = {{0, 8}, {0, 1}, {0, 4}};
    const char* pn[3] = {"same XCD (0, 8)", "XCDs 0 / 1", "XCDs 0 / 4"};
    const char* pol[3] = {"agent atomic", "sc0", "sc0 sc1"};
    for (int rep = 0; rep < 2; ++rep)
        for (int p = 0; p < 3; ++p)
            for (int q = 0; q < 3; ++q) {
                (void)hipMemset(slots, 0, 4096);
                (void)hipMemset(out, 0, 64);
                if (q == 0) hipLaunchKernelGGL(k_pingpong<0>, dim3(nwg), dim3(64), 0, 0, slots, pairs[p][0], pairs[p][1], n, out, xcc);
                if (q == 1) hipLaunchKernelGGL(k_pingpong<1>, dim3(nwg), dim3(64), 0, 0, slots, pairs[p][0], pairs[p][1], n, out, xcc);
                if (q == 2) hipLaunchKernelGGL(k_pingpong<2>, dim3(nwg), dim3(64), 0, 0, slots, pairs[p][0], pairs[p][1], n, out, xcc);
                if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
                unsigned long long h[2];
                unsigned x[nwg];
                (void)hipMemcpy(h, out, 16, hipMemcpyDeviceToHost);
                (void)hipMemcpy(x, xcc, 4 * nwg, hipMemcpyDeviceToHost);
                printf("rep %d  %-16s %-13s one-way %7.1f ns  (fails %llu)  xcc[a]=%u xcc[b]=%u\n", rep, pn[p], pol[q],
                       h[0] * 10.0 / (2.0 * n), h[1], x[pairs[p][0]], x[pairs[p][1]]);
                if (rep == 0 && p == 0 && q == 0) {
                    printf("xcc ids:");
                    for (int w = 0; w < nwg; ++w) printf(" %u", x[w]);
                    printf("\n");
                }
            }
    return 0;
}
