// Accuracy and dependent latency of v_rsq_f64 and of its Newton refinements on gfx950
// (for the Cholesky pivot path). build: hipcc --offload-arch=gfx950 -O3 tools/rsq_f64_check.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__device__ __forceinline__ unsigned long long now() {
    unsigned long long t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

__global__ void k_rsq(const double* x, double* y0, double* y1, double* y2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    const double r0 = __builtin_amdgcn_rsq(v);
    const double e1 = __builtin_fma(-v * r0, r0, 1.0);
    const double r1 = __builtin_fma(0.5 * r0, e1, r0);
    const double e2 = __builtin_fma(-v * r1, r1, 1.0);
    const double r2 = __builtin_fma(0.5 * r1, e2, r1);
    y0[i] = r0;
    y1[i] = r1;
    y2[i] = r2;
}

__global__ void k_lat(double* out, unsigned long long* cyc, int iters, int mode) {
    double v = 1.0 + threadIdx.x * 1e-12;
    const unsigned long long t0 = now();
    for (int it = 0; it < iters; ++it) {
        if (mode == 0) v = __builtin_amdgcn_rsq(v) + 1.0;
        else if (mode == 1) {
            const double r0 = __builtin_amdgcn_rsq(v);
            const double e1 = __builtin_fma(-v * r0, r0, 1.0);
            v = __builtin_fma(0.5 * r0, e1, r0) + 1.0;
        } else {
            v = 1.0 / sqrt(v) + 1.0;
        }
    }
    const unsigned long long t1 = now();
    out[threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
    const int n = 1 << 20;
    std::vector<double> x(n);
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> u(-30.0, 30.0), m(1.0, 2.0);
    for (auto& v : x) v = m(g) * std::exp2(std::floor(u(g)));
    double *dx, *d0, *d1, *d2, *dout;
    unsigned long long* dc;
    (void)hipMalloc(&dx, n * 8); (void)hipMalloc(&d0, n * 8); (void)hipMalloc(&d1, n * 8); (void)hipMalloc(&d2, n * 8);
    (void)hipMalloc(&dout, 64 * 8); (void)hipMalloc(&dc, 8);
    (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_rsq, dim3(n / 256), dim3(256), 0, 0, dx, d0, d1, d2, n);
    std::vector<double> y0(n), y1(n), y2(n);
    (void)hipMemcpy(y0.data(), d0, n * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(y1.data(), d1, n * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(y2.data(), d2, n * 8, hipMemcpyDeviceToHost);
    double e0 = 0, e1 = 0, e2 = 0;
    for (int i = 0; i < n; ++i) {
        const long double r = 1.0L / std::sqrt((long double)x[i]);
        e0 = std::fmax(e0, (double)std::fabs((y0[i] - r) / r));
        e1 = std::fmax(e1, (double)std::fabs((y1[i] - r) / r));
        e2 = std::fmax(e2, (double)std::fabs((y2[i] - r) / r));
    }
    printf("max rel err: rsq %.3e  rsq+1NR %.3e  rsq+2NR %.3e  (f64 eps %.3e)\n", e0, e1, e2, 2.220446e-16);
    const char* names[3] = {"rsq", "rsq+1NR", "1/sqrt (libm)"};
    for (int mode = 0; mode < 3; ++mode) {
        unsigned long long c;
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, dout, dc, 1000, mode);
        (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
        printf("dependent latency %-14s %.1f cycles (incl. one add)\n", names[mode], c / 1000.0);
    }
    return 0;
}
