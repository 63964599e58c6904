// Micro-benchmark (dev aid): cost of writing 8.4 M per-pair records txn-major from key-major order
// (random 16-B / 8-B / 4-B scatters) against coalesced writes and random 8-B gathers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <random>
#include <algorithm>

struct alignas(16) Rec { uint32_t a, b, c, d; };

__global__ void scatter16(uint32_t n, const uint32_t *__restrict__ perm, Rec *__restrict__ out)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        out[perm[i]] = Rec{i, i + 1, i + 2, 0};
}
__global__ void scatter8(uint32_t n, const uint32_t *__restrict__ perm, uint2 *__restrict__ out)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        out[perm[i]] = make_uint2(i, i + 1);
}
__global__ void scatter4(uint32_t n, const uint32_t *__restrict__ perm, uint32_t *__restrict__ out)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        out[perm[i]] = i;
}
__global__ void coal16(uint32_t n, const uint32_t *__restrict__ perm, Rec *__restrict__ out)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        out[i] = Rec{perm[i], i + 1, i + 2, 0};
}
__global__ void gather8(uint32_t n, const uint32_t *__restrict__ perm, const uint2 *__restrict__ in,
                        uint32_t *__restrict__ out)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint2 v = in[perm[i]];
        out[i] = v.x + v.y;
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main()
{
    const uint32_t n = 8u << 20;
    // key-major -> txn-major permutation of a synthetic batch: txn t holds 8 keys; sorting by key
    std::vector<uint32_t> key(n);
    std::mt19937 g(1);
    for (uint32_t i = 0; i < n; ++i) key[i] = g() % 100000u;
    std::vector<uint32_t> idx(n);
    for (uint32_t i = 0; i < n; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) { return key[x] < key[y]; });
    uint32_t *perm; Rec *o16; uint2 *o8; uint32_t *o4;
    CK(hipMalloc(&perm, n * 4)); CK(hipMalloc(&o16, (size_t)n * 16)); CK(hipMalloc(&o8, (size_t)n * 8));
    CK(hipMalloc(&o4, (size_t)n * 4));
    CK(hipMemcpy(perm, idx.data(), n * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int B = 4096, T = 256, R = 20;
    auto run = [&](const char *name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        (void)hipEventRecord(e0);
        for (int r = 0; r < R; ++r) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
        printf("%-10s %8.1f us\n", name, 1000.0f * ms / R);
    };
    run("scatter16", [&] { hipLaunchKernelGGL(scatter16, dim3(B), dim3(T), 0, 0, n, perm, o16); });
    run("scatter8", [&] { hipLaunchKernelGGL(scatter8, dim3(B), dim3(T), 0, 0, n, perm, o8); });
    run("scatter4", [&] { hipLaunchKernelGGL(scatter4, dim3(B), dim3(T), 0, 0, n, perm, o4); });
    run("coal16", [&] { hipLaunchKernelGGL(coal16, dim3(B), dim3(T), 0, 0, n, perm, o16); });
    run("gather8", [&] { hipLaunchKernelGGL(gather8, dim3(B), dim3(T), 0, 0, n, perm, o8, o4); });
    CK(hipDeviceSynchronize());
    return 0;
}
