// LDS micro-benchmark for the fill kernel's near-bitmap construction: cost per wave instruction of
// (a) 64-bit LDS atomic OR, (b) 32-bit atomic OR, (c) byte stores, when runs of R consecutive lanes
// hit the same word (candidates of one key slice are sorted, so neighbours share bitmap words).
// Build: hipcc --offload-arch=gfx950 -O3 -o lds_patterns lds_patterns.hip ; run: ./lds_patterns
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;
constexpr int WAVES = 8;

template <int MODE>
__global__ __launch_bounds__(WAVES * 64) void k(int run, unsigned *out)
{
    __shared__ unsigned long long bm[WAVES][64];
    __shared__ unsigned char by[WAVES][4096];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    bm[w][lane] = 0;
    for (int i = lane; i < 4096; i += 64) by[w][i] = 0;
    __syncthreads();
    // lane -> word: runs of `run` lanes share a word, consecutive runs use consecutive words
    const unsigned word = (unsigned)(lane / run) & 63u;
    const unsigned bit = (unsigned)(lane % run) * 3u + 1u;
    unsigned acc = 0;
    for (int it = 0; it < ITERS; ++it) {
        const unsigned wv = (word + (unsigned)it) & 63u;
        if (MODE == 0) atomicOr(&bm[w][wv], 1ull << (bit & 63));
        if (MODE == 1) atomicOr((unsigned *)&bm[w][0] + ((wv * 2 + (bit >> 5)) & 127), 1u << (bit & 31));
        if (MODE == 2) by[w][(wv * 64 + bit) & 4095] = 1;
        if (MODE == 3) {   // plain 64-bit store to the word (same-address lanes write the same value)
            bm[w][wv] = (unsigned long long)it;
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): one instruction's latency + issue per iteration
    }
    __syncthreads();
    acc = (unsigned)bm[w][lane] + by[w][lane];
    if (acc == 0xdeadbeef) out[0] = acc;
}

int main()
{
    unsigned *out;
    hipMalloc(&out, 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const char *names[] = {"ds_or_b64 atomic", "ds_or_b32 atomic", "ds_write_b8", "ds_write_b64 plain"};
    const int blocks = 256 * 4;   // 4 blocks/CU x 8 waves = 32 waves per CU
    for (int mode = 0; mode < 4; ++mode)
        for (int run : {1, 2, 4, 8, 16, 64}) {
            for (int rep = 0; rep < 2; ++rep) {
                hipEventRecord(a);
                switch (mode) {
                case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(WAVES * 64), 0, 0, run, out); break;
                case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(WAVES * 64), 0, 0, run, out); break;
                case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(WAVES * 64), 0, 0, run, out); break;
                default: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(WAVES * 64), 0, 0, run, out); break;
                }
                hipEventRecord(b);
                hipEventSynchronize(b);
                float ms = 0;
                hipEventElapsedTime(&ms, a, b);
                // wave-instructions per CU: 32 waves x ITERS; clock ~2.4 GHz
                const double per_cu = 32.0 * ITERS;
                if (rep) printf("%-20s run %2d: %.3f ms, %.2f ns per wave-instr per CU\n", names[mode], run, ms, ms * 1e6 / per_cu);
            }
        }
    return 0;
}
