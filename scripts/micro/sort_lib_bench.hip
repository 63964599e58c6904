// Micro-benchmark (dev aid): rocPRIM's radix sort (onesweep) on the config-2 pair sort -- 8.4 M
// (17-bit key, value) pairs with a u32 and a u64 value -- against the in-tree LSD sort's stages
// (rs_upsweep x2 + scans + rs_downsweep<8>, <9>: ~200 us on config 2, profiles/r06_fin3).
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <typename V>
static int run(const char *name, uint32_t n, const uint32_t *dk, uint32_t *dk2, V *dv, V *dv2, hipStream_t st)
{
    size_t tb = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tb, dk, dk2, dv, dv2, n, 0, 17, st));
    void *tmp;
    CK(hipMalloc(&tmp, tb));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 5; ++i) CK(rocprim::radix_sort_pairs(tmp, tb, dk, dk2, dv, dv2, n, 0, 17, st));
    const int it = 50;
    CK(hipEventRecord(a, st));
    for (int i = 0; i < it; ++i) CK(rocprim::radix_sort_pairs(tmp, tb, dk, dk2, dv, dv2, n, 0, 17, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"sort\": \"%s\", \"n\": %u, \"us\": %.1f, \"temp_bytes\": %zu}\n", name, n, 1000.0 * ms / it, tb);
    fflush(stdout);
    CK(hipFree(tmp));
    return 0;
}

int main()
{
    const uint32_t n = 8388608;
    std::vector<uint32_t> hk(n);
    uint64_t s = 88172645463325252ull;
    for (uint32_t i = 0; i < n; ++i) {           // skewed 17-bit keys (hot low ids), 100 k keyspace
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const double u = (double)(s >> 11) / 9007199254740992.0;
        hk[i] = (uint32_t)(100000.0 * u * u * u) % 100000u;
    }
    uint32_t *dk, *dk2, *dv, *dv2;
    uint64_t *dw, *dw2;
    CK(hipMalloc(&dk, n * 4)); CK(hipMalloc(&dk2, n * 4));
    CK(hipMalloc(&dv, n * 4)); CK(hipMalloc(&dv2, n * 4));
    CK(hipMalloc(&dw, n * 8)); CK(hipMalloc(&dw2, n * 8));
    CK(hipMemcpy(dk, hk.data(), n * 4, hipMemcpyHostToDevice));
    CK(hipMemset(dv, 0, n * 4));
    CK(hipMemset(dw, 0, n * 8));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    if (run<uint32_t>("rocprim u32 value", n, dk, dk2, dv, dv2, st)) return 1;
    if (run<uint64_t>("rocprim u64 value", n, dk, dk2, dw, dw2, st)) return 1;
    return 0;
}
