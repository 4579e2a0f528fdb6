// sort_probe.hip — rocPRIM radix sort / scan timings at plan sizes (diagnostic for the device-side plan).
// usage: sort_probe [n=1000000] [bits=25]
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 1000000;
    const int bits = argc > 2 ? std::atoi(argv[2]) : 25;
    std::vector<unsigned> hk(n), hv(n);
    unsigned s = 12345;
    for (int i = 0; i < n; ++i) {
        s = s * 1664525u + 1013904223u;
        hk[i] = (unsigned)(((unsigned long long)i * 10 / 10) * 0 + (s >> (32 - bits)));
        hv[i] = i;
    }
    unsigned *k0, *k1, *v0, *v1;
    CK(hipMalloc(&k0, 4ull * n)); CK(hipMalloc(&k1, 4ull * n)); CK(hipMalloc(&v0, 4ull * n)); CK(hipMalloc(&v1, 4ull * n));
    CK(hipMemcpy(k0, hk.data(), 4ull * n, hipMemcpyHostToDevice));
    CK(hipMemcpy(v0, hv.data(), 4ull * n, hipMemcpyHostToDevice));
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tb, k0, k1, v0, v1, n, 0, bits));
    void* tmp;
    CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a, 0));
        CK(rocprim::radix_sort_pairs(tmp, tb, k0, k1, v0, v1, n, 0, bits));
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        std::printf("radix_sort_pairs n=%d bits=%d: %.1f us (temp %zu B)\n", n, bits, ms * 1e3, tb);
    }
    std::vector<unsigned> ok(n), ov(n);
    CK(hipMemcpy(ok.data(), k1, 4ull * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ov.data(), v1, 4ull * n, hipMemcpyDeviceToHost));
    bool good = true;
    for (int i = 1; i < n; ++i)
        if (ok[i - 1] > ok[i] || (ok[i - 1] == ok[i] && ov[i - 1] > ov[i])) good = false;
    std::printf("sorted and stable: %d\n", good);
    size_t ts = 0;
    CK(rocprim::exclusive_scan(nullptr, ts, k0, k1, 0u, n, rocprim::plus<unsigned>()));
    void* tmp2;
    CK(hipMalloc(&tmp2, ts));
    for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(a, 0));
        CK(rocprim::exclusive_scan(tmp2, ts, k0, k1, 0u, n, rocprim::plus<unsigned>()));
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        std::printf("exclusive_scan n=%d: %.1f us\n", n, ms * 1e3);
    }
    return 0;
}
