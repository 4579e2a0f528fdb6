// Microbenchmark: v_mfma_f64_16x16x4_f64 issue rate and dependent latency on one SIMD
// (one wave per SIMD: 4 waves per workgroup, one workgroup per CU), and the f64 VALU FMA
// issue rate, measured with s_memtime inside the kernel.
// build: hipcc --offload-arch=gfx950 -O3 tools/mfma_f64_rate.hip -o tools/_build/mfma_f64_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int NACC>
__global__ __launch_bounds__(512) void k_mfma(double* out, unsigned long long* cyc, int iters) {
    d4 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    __syncthreads();
    const unsigned long long t0 = now();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    const unsigned long long t1 = now();
    double s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * 512 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

template <int NCH>
__global__ __launch_bounds__(512) void k_fma(double* out, unsigned long long* cyc, int iters) {
    double x[NCH];
    for (int i = 0; i < NCH; ++i) x[i] = threadIdx.x + i;
    const double m = 0.999999, c = 1e-7;
    __syncthreads();
    const unsigned long long t0 = now();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) x[i] = __builtin_fma(x[i], m, c);
    }
    const unsigned long long t1 = now();
    double s = 0;
    for (int i = 0; i < NCH; ++i) s += x[i];
    out[blockIdx.x * 512 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    double* out;
    unsigned long long *cyc, h;
    hipMalloc(&out, sizeof(double) * 256 * 512);
    hipMalloc(&cyc, 8);
    const int iters = 4096;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
#define RUN(K, N, label, per, flops_per_inst)                                                           \
    do {                                                                                                \
        for (int tpb = 256; tpb <= 512; tpb += 256) {                                                   \
            hipLaunchKernelGGL((K<N>), dim3(256), dim3(tpb), 0, 0, out, cyc, iters);                    \
            hipEventRecord(e0, 0);                                                                      \
            hipLaunchKernelGGL((K<N>), dim3(256), dim3(tpb), 0, 0, out, cyc, iters);                    \
            hipEventRecord(e1, 0);                                                                      \
            hipEventSynchronize(e1);                                                                    \
            float ms = 0;                                                                               \
            hipEventElapsedTime(&ms, e0, e1);                                                           \
            hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);                                               \
            const double tf = 256.0 * (tpb / 64) * (double)iters * (per) * (flops_per_inst) / (ms * 1e-3) / 1e12; \
            printf("%-40s waves/SIMD %d: %7.2f memtime-ticks/inst/wave, wall %.3f ms = %6.1f TFLOP/s, tick %.2f GHz\n", \
                   label, tpb / 256, (double)h / (iters * (per)), ms, tf, (double)h / (ms * 1e6));     \
        }                                                                                               \
    } while (0)
    RUN(k_mfma, 1, "mfma_f64_16x16x4 1 chain", 1, 2048.0);
    RUN(k_mfma, 4, "mfma_f64_16x16x4 4 chains", 4, 2048.0);
    RUN(k_mfma, 8, "mfma_f64_16x16x4 8 chains", 8, 2048.0);
    RUN(k_fma, 1, "v_fma_f64 1 chain", 1, 128.0);
    RUN(k_fma, 8, "v_fma_f64 8 chains", 8, 128.0);
    RUN(k_fma, 16, "v_fma_f64 16 chains", 16, 128.0);
    hipDeviceSynchronize();
    return 0;
}
