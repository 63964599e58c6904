// Vector-memory micro-benchmark: cost per wave-instruction (per CU) of load / store shapes the deps
// kernels use -- lanes in runs of R consecutive dwords, runs on distinct 128-B lines -- with the data
// L2-resident (1 MiB footprint), to price the TA/TD path separately from HBM.
// Build: hipcc --offload-arch=gfx950 -O3 -o vmem_patterns vmem_patterns.hip ; run: ./vmem_patterns
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 2048;
constexpr int WAVES = 8;
constexpr uint32_t FOOT = 1u << 18;   // dwords (1 MiB)

template <int MODE, int W>   // MODE 0 load, 1 store; W dwords per lane (1 or 4)
__global__ __launch_bounds__(WAVES * 64) void k(uint32_t *buf, int run, uint32_t *out)
{
    const uint32_t lane = threadIdx.x & 63, wv = blockIdx.x * WAVES + (threadIdx.x >> 6);
    // lane -> address: runs of `run` lanes read consecutive W-dword elements; each run on its own line
    const uint32_t r = lane / run, e = lane % run;
    uint32_t acc = 0;
    for (int it = 0; it < ITERS; ++it) {
        const uint32_t base = ((wv * 977u + (uint32_t)it * 131u) * 64u) % FOOT;           // wave's region
        const uint32_t addr = (base + r * 4096u + e * W) % (FOOT - 4);                     // runs 16 KiB apart
        if (MODE == 0) {
            if (W == 1) acc += buf[addr];
            else { const uint4 v = *(const uint4 *)&buf[addr & ~3u]; acc += v.x ^ v.w; }
        } else {
            if (W == 1) buf[addr] = acc + (uint32_t)it;
            else *(uint4 *)&buf[addr & ~3u] = make_uint4(acc, (uint32_t)it, lane, 0u);
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main()
{
    uint32_t *buf, *out;
    hipMalloc(&buf, FOOT * 4);
    hipMalloc(&out, 4);
    hipMemset(buf, 0, FOOT * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int blocks = 256 * 4;   // 32 waves per CU
    const char *names[] = {"load dword", "load dwordx4", "store dword", "store dwordx4"};
    for (int m = 0; m < 4; ++m)
        for (int run : {1, 2, 4, 8, 16, 32, 64}) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(a);
                switch (m) {
                case 0: hipLaunchKernelGGL((k<0, 1>), dim3(blocks), dim3(WAVES * 64), 0, 0, buf, run, out); break;
                case 1: hipLaunchKernelGGL((k<0, 4>), dim3(blocks), dim3(WAVES * 64), 0, 0, buf, run, out); break;
                case 2: hipLaunchKernelGGL((k<1, 1>), dim3(blocks), dim3(WAVES * 64), 0, 0, buf, run, out); break;
                default: hipLaunchKernelGGL((k<1, 4>), dim3(blocks), dim3(WAVES * 64), 0, 0, buf, run, out); break;
                }
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                const double per_cu = 32.0 * ITERS;   // wave-instructions per CU
                if (rep) printf("%-14s run %2d (%2d lines): %.3f ms, %.2f ns per wave-instr per CU\n", names[m], run,
                                64 / run, ms, ms * 1e6 / per_cu);
            }
        }
    return 0;
}
