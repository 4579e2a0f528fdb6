// latency_probe.hip — dependent-latency micro-benchmark of the primitives k_bcr_band chains on (gfx950, one
// workgroup of 1024 threads): f64 FMA, v_rsq_f64, a 16-lane DPP broadcast + FMA, an LDS store->load round trip, a
// workgroup barrier. Each probe runs N dependent steps between two s_memrealtime (100 MHz) / s_memtime (shader clock)
// stamps on wave 0; prints ns and clocks per step.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ unsigned long long rt() {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
__device__ __forceinline__ unsigned long long ct() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
constexpr int N = 256;
__global__ __launch_bounds__(1024) void k(double* out, unsigned long long* tt, double seed) {
    __shared__ double L[2048];
    const int tid = threadIdx.x;
    double x = seed + tid * 1e-9, y = 1.0 + tid * 1e-12;
    unsigned long long r0, c0;
    // 0: dependent FMA
    __syncthreads(); r0 = rt(); c0 = ct();
    for (int i = 0; i < N; ++i) x = __builtin_fma(x, y, 1e-3);
    __syncthreads(); if (tid == 0) { tt[0] = rt() - r0; tt[1] = ct() - c0; }
    // 1: dependent rsq
    __syncthreads(); r0 = rt(); c0 = ct();
    for (int i = 0; i < N; ++i) x = __builtin_amdgcn_rsq(x + 1.0);
    __syncthreads(); if (tid == 0) { tt[2] = rt() - r0; tt[3] = ct() - c0; }
    // 2: DPP row broadcast + FMA
    __syncthreads(); r0 = rt(); c0 = ct();
    for (int i = 0; i < N; ++i) {
        const unsigned long long u = __double_as_longlong(x);
        const int lo = __builtin_amdgcn_update_dpp(0, (int)(unsigned)u, 0x150 + 3, 0xF, 0xF, false);
        const int up = __builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), 0x150 + 3, 0xF, 0xF, false);
        x = __builtin_fma(__longlong_as_double((long long)(((unsigned long long)(unsigned)up << 32) | (unsigned)lo)), y, 1e-3);
    }
    __syncthreads(); if (tid == 0) { tt[4] = rt() - r0; tt[5] = ct() - c0; }
    // 3: LDS store -> load round trip (own slot)
    __syncthreads(); r0 = rt(); c0 = ct();
    for (int i = 0; i < N; ++i) {
        L[tid] = x;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        x = L[tid ^ 1] + 1e-3;
    }
    __syncthreads(); if (tid == 0) { tt[6] = rt() - r0; tt[7] = ct() - c0; }
    // 4: barrier (1024 threads)
    __syncthreads(); r0 = rt(); c0 = ct();
    for (int i = 0; i < N; ++i) { x += 1e-3; __syncthreads(); }
    __syncthreads(); if (tid == 0) { tt[8] = rt() - r0; tt[9] = ct() - c0; }
    // 5: v_readlane pair + FMA
    __syncthreads(); r0 = rt(); c0 = ct();
    for (int i = 0; i < N; ++i) {
        const unsigned long long u = __double_as_longlong(x);
        const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, 3), hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), 3);
        x = __builtin_fma(__longlong_as_double(((unsigned long long)hi << 32) | lo), y, 1e-3);
    }
    __syncthreads(); if (tid == 0) { tt[10] = rt() - r0; tt[11] = ct() - c0; }
    out[tid] = x;
}
int main() {
    double* d; unsigned long long* t;
    hipMalloc(&d, 1024 * 8); hipMalloc(&t, 16 * 8);
    const char* nm[] = {"f64 fma", "v_rsq_f64", "dpp bcast + fma", "lds store->load", "barrier(1024)", "readlane + fma"};
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(1024), 0, 0, d, t, 1.0 + rep);
        unsigned long long h[16];
        hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
        for (int i = 0; i < 6; ++i)
            printf("%-18s %6.1f ns %6.1f clk per step (clock %.2f GHz)\n", nm[i], h[2 * i] * 10.0 / N,
                   (double)h[2 * i + 1] / N, (double)h[2 * i + 1] / (h[2 * i] * 10.0));
        printf("--\n");
    }
    return 0;
}
