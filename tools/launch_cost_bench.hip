// Launch-cost micro-benchmark: average time per launch in a chain of dependent single-workgroup launches on one
// stream, for kernels that differ only in what they touch:
//   0  nothing
//   1  one 4-byte store to device memory
//   2  one 4-byte system-scope store to host-mapped memory (k_final's progress word)
//   3  one load of the word the previous launch stored + one store (a dependent chain through memory)
//   4  variant 3 + variant 2 (k_final's shape: state in, state out, progress word out)
//   5  variant 3 with 256 threads and an LDS reduction (two barriers) before the store
//   6  variant 3 after a 10 us spin on the 100 MHz wall clock (the host enqueues far ahead of the GPU: what is
//      left per launch above 10 us is the GPU-side gap between dependent kernels)
// build: hipcc --offload-arch=gfx950 -O3 tools/launch_cost_bench.hip -o tools/_build/launch_cost_bench
#include <hip/hip_runtime.h>

#include <cstdio>

template <int V>
__global__ void k(unsigned* __restrict__ dev, unsigned* __restrict__ host) {
    if constexpr (V == 0) return;
    if constexpr (V == 1) {
        if (threadIdx.x == 0) dev[0] = 1u;
    }
    if constexpr (V == 2) {
        if (threadIdx.x == 0) __hip_atomic_store(host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if constexpr (V == 3 || V == 4) {
        if (threadIdx.x == 0) {
            const unsigned v = dev[0] + 1u;
            dev[0] = v;
            if constexpr (V == 4) __hip_atomic_store(host, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    if constexpr (V == 6) {
        const unsigned long long t0 = wall_clock64();
        while (wall_clock64() - t0 < 1000ull) __builtin_amdgcn_s_sleep(1);
        if (threadIdx.x == 0) dev[0] = dev[0] + 1u;
    }
    if constexpr (V == 5) {
        __shared__ unsigned red[4];
        unsigned v = dev[threadIdx.x & 63];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) dev[0] = red[0] + red[1] + red[2] + red[3];
    }
}

int main() {
    unsigned *dev, *host;
    (void)hipMalloc(&dev, 4096);
    (void)hipMemset(dev, 0, 4096);
    (void)hipHostMalloc(&host, 4096, hipHostMallocMapped);
    hipStream_t s;
    (void)hipStreamCreate(&s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int n = 2000;
    const char* names[7] = {"empty", "device store", "host-mapped store", "device load+store", "load+store+host store",
                            "256 thr, reduce, store", "10 us spin + load/store"};
    for (int round = 0; round < 2; ++round)
        for (int v = 0; v < 7; ++v) {
            auto launch = [&]() {
                const int tpb = v == 5 ? 256 : 64;
                switch (v) {
                    case 0: hipLaunchKernelGGL(k<0>, dim3(1), dim3(tpb), 0, s, dev, host); break;
                    case 1: hipLaunchKernelGGL(k<1>, dim3(1), dim3(tpb), 0, s, dev, host); break;
                    case 2: hipLaunchKernelGGL(k<2>, dim3(1), dim3(tpb), 0, s, dev, host); break;
                    case 3: hipLaunchKernelGGL(k<3>, dim3(1), dim3(tpb), 0, s, dev, host); break;
                    case 4: hipLaunchKernelGGL(k<4>, dim3(1), dim3(tpb), 0, s, dev, host); break;
                    case 5: hipLaunchKernelGGL(k<5>, dim3(1), dim3(tpb), 0, s, dev, host); break;
                    default: hipLaunchKernelGGL(k<6>, dim3(1), dim3(tpb), 0, s, dev, host); break;
                }
            };
            for (int i = 0; i < 100; ++i) launch();
            (void)hipEventRecord(e0, s);
            for (int i = 0; i < n; ++i) launch();
            (void)hipEventRecord(e1, s);
            (void)hipEventSynchronize(e1);
            float ms = 0.f;
            (void)hipEventElapsedTime(&ms, e0, e1);
            printf("round %d  %-24s %6.2f us per launch\n", round, names[v], ms * 1000.0 / n);
        }
    // the same chains captured into one hipGraph (host launch cost out of the picture)
    // and a graph of 5 dependent launches (one LM iteration's shape) launched back to back
    for (int v = 0; v < 7; v += (v == 0 ? 5 : 1)) {
        hipGraph_t g;
        hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int i = 0; i < n; ++i) {
            if (v == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, s, dev, host);
            else if (v == 5) hipLaunchKernelGGL(k<5>, dim3(1), dim3(256), 0, s, dev, host);
            else hipLaunchKernelGGL(k<6>, dim3(1), dim3(64), 0, s, dev, host);
        }
        (void)hipStreamEndCapture(s, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        (void)hipGraphLaunch(ge, s);
        (void)hipStreamSynchronize(s);
        (void)hipEventRecord(e0, s);
        (void)hipGraphLaunch(ge, s);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("graph    %-24s %6.2f us per launch\n", names[v], ms * 1000.0 / n);
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(g);
    }
    for (int v = 0; v < 7; v += 6) {
        hipGraph_t g;
        hipGraphExec_t ge;
        (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int i = 0; i < 5; ++i) {
            if (v == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, s, dev, host);
            else hipLaunchKernelGGL(k<6>, dim3(1), dim3(64), 0, s, dev, host);
        }
        (void)hipStreamEndCapture(s, &g);
        (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        for (int i = 0; i < 20; ++i) (void)hipGraphLaunch(ge, s);
        (void)hipStreamSynchronize(s);
        (void)hipEventRecord(e0, s);
        for (int i = 0; i < n / 5; ++i) (void)hipGraphLaunch(ge, s);
        (void)hipEventRecord(e1, s);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("graph5   %-24s %6.2f us per launch\n", names[v], ms * 1000.0 / n);
        (void)hipGraphExecDestroy(ge);
        (void)hipGraphDestroy(g);
    }
    return 0;
}
