// Micro-benchmark (dev aid): one readiness call as five dependent kernels (rd_part, rd_summary,
// rd_filter, rd_eval, rd_host_out) against one launch whose phases meet at grid barriers
// (an arrival counter, agent-scope fences, a bounded spin).  Phases have the shapes of an
// incremental accord_ready_update call: a pass over ~90 k carried entries, a few dirty keys, a
// filter over 16 k waiting txns x 8 lanes, a few evaluations, the header copied to pinned memory.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Args {
    const uint32_t *tab;      // random table (L2 misses)
    uint32_t tmask;
    uint32_t *out;
    uint32_t *host;
    uint32_t n1, n2, n3, n4;  // phase sizes
};

__device__ __forceinline__ uint32_t chain(const Args &a, uint32_t x, int hops)
{
    for (int h = 0; h < hops; ++h) x = a.tab[(x * 2654435761u) & a.tmask];
    return x;
}

__device__ __forceinline__ void phase(const Args &a, uint32_t n, int hops, uint32_t salt, uint32_t gid, uint32_t gsz)
{
    for (uint32_t i = gid; i < n; i += gsz) {
        const uint32_t v = chain(a, i + salt, hops);
        if ((v & 1023u) == 0u) a.out[(v >> 10) & 1023u] = i;
    }
}

__global__ __launch_bounds__(256) void k_phase(Args a, uint32_t n, int hops, uint32_t salt)
{
    phase(a, n, hops, salt, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}

__global__ __launch_bounds__(256) void k_out(Args a)
{
    for (uint32_t x = threadIdx.x; x < 64; x += blockDim.x) a.host[x] = a.out[x];
}

// arrival counter: monotone over calls; target = base + blocks * (barrier index + 1)
__device__ __forceinline__ void grid_bar(uint32_t *ctr, uint32_t target, uint32_t *err)
{
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        atomicAdd(ctr, 1u);
        const uint64_t t0 = wall_clock64();
        while ((int32_t)(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
            if (wall_clock64() - t0 > 10000000ull) { atomicExch(err, 1u); break; }   // 100 ms at 100 MHz
            __builtin_amdgcn_s_sleep(1);
        }
        __threadfence();
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_fused(Args a, uint32_t *ctr, uint32_t base, uint32_t *err)
{
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x, gsz = gridDim.x * blockDim.x, B = gridDim.x;
    phase(a, a.n1, 1, 1u, gid, gsz);
    grid_bar(ctr, base + B * 1, err);
    phase(a, a.n2, 3, 2u, gid, gsz);
    grid_bar(ctr, base + B * 2, err);
    phase(a, a.n3, 3, 3u, gid, gsz);
    grid_bar(ctr, base + B * 3, err);
    phase(a, a.n4, 5, 4u, gid, gsz);
    grid_bar(ctr, base + B * 4, err);
    if (blockIdx.x == 0)
        for (uint32_t x = threadIdx.x; x < 64; x += blockDim.x) a.host[x] = a.out[x];
}

int main()
{
    const uint32_t T = 1u << 24;                  // 64 MB table
    std::vector<uint32_t> h(T);
    uint32_t s = 12345;
    for (auto &v : h) { s = s * 1664525u + 1013904223u; v = s; }
    uint32_t *tab, *out, *ctr, *err, *host, *hostd;
    CK(hipMalloc(&tab, T * 4));
    CK(hipMemcpy(tab, h.data(), T * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&out, 4096 * 4));
    CK(hipMalloc(&ctr, 64));
    CK(hipMalloc(&err, 64));
    CK(hipMemset(ctr, 0, 64));
    CK(hipMemset(err, 0, 64));
    CK(hipHostMalloc(&host, 4096, hipHostMallocDefault));
    CK(hipHostGetDevicePointer((void **)&hostd, host, 0));
    hipStream_t st;
    CK(hipStreamCreate(&st));
    Args a{tab, T - 1, out, hostd, 90000, 64, 16384 * 8, 64};
    const int iters = 2000;
    auto sep = [&]() {
        hipLaunchKernelGGL(k_phase, dim3((a.n1 + 255) / 256), dim3(256), 0, st, a, a.n1, 1, 1u);
        hipLaunchKernelGGL(k_phase, dim3(256), dim3(256), 0, st, a, a.n2, 3, 2u);
        hipLaunchKernelGGL(k_phase, dim3((a.n3 + 255) / 256), dim3(256), 0, st, a, a.n3, 3, 3u);
        hipLaunchKernelGGL(k_phase, dim3(1024), dim3(256), 0, st, a, a.n4, 5, 4u);
        hipLaunchKernelGGL(k_out, dim3(1), dim3(256), 0, st, a);
        (void)hipStreamSynchronize(st);
    };
    uint32_t base = 0;
    for (uint32_t blocks : {64u, 128u, 256u, 512u}) {
        auto fused = [&]() {
            hipLaunchKernelGGL(k_fused, dim3(blocks), dim3(256), 0, st, a, ctr, base, err);
            base += blocks * 4;
            (void)hipStreamSynchronize(st);
        };
        for (int i = 0; i < 50; ++i) { sep(); fused(); }
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < iters; ++i) sep();
        auto t1 = std::chrono::steady_clock::now();
        for (int i = 0; i < iters; ++i) fused();
        auto t2 = std::chrono::steady_clock::now();
        uint32_t e = 0;
        CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
        printf("{\"fused_blocks\": %u, \"separate_us\": %.2f, \"fused_us\": %.2f, \"barrier_timeouts\": %u}\n", blocks,
               std::chrono::duration<double, std::micro>(t1 - t0).count() / iters,
               std::chrono::duration<double, std::micro>(t2 - t1).count() / iters, e);
        fflush(stdout);
    }
    return 0;
}
