// One-workgroup sort of a resident batch's (key << ib | index) composites (radix_sort.hip's
// ms_batch_sort_kernel), timed alone with s_memtime stamps per phase, for THREADS = 256 / 512 / 1024.
// hipcc --offload-arch=gfx950 -O3 -I cassandra-accord_amd/csrc scripts/micro/batch_sort.hip -o /tmp/batch_sort
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "device_common.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr uint32_t MAXN = 16384;
constexpr int BITS = 9, BINS = 1 << BITS;

template <int THREADS>
__global__ __launch_bounds__(THREADS) void bsort(uint32_t P, uint32_t ib, int kbits, const uint32_t *__restrict__ bkey,
                                                 uint32_t *__restrict__ comp, unsigned long long *stamp)
{
    constexpr int WAVES = THREADS / 64, IT_MAX = MAXN / THREADS;
    __shared__ uint32_t sh[MAXN];
    __shared__ uint32_t wcnt[WAVES][BINS];
    __shared__ uint32_t run[BINS];
    __shared__ uint32_t wsum[WAVES];
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const uint32_t IT = (P + THREADS - 1) / THREADS;
    const uint64_t lt = lanemask_lt();
    int ns = 0;
    auto st = [&]() { __syncthreads(); if (tid == 0) stamp[ns] = __builtin_amdgcn_s_memtime(); ++ns; };
    st();
    uint32_t v[IT_MAX], lrank[IT_MAX];
#pragma unroll
    for (int r = 0; r < IT_MAX; ++r) {
        const uint32_t e = (w * IT + r) * 64 + lane;
        v[r] = (r < (int)IT && e < P) ? (bkey[e] << ib) | e : 0u;
    }
    st();
    const int passes = (kbits + BITS - 1) / BITS;
    int shift = (int)ib, left = kbits;
    for (int p = 0; p < passes; ++p) {
        const int pb = left / (passes - p);
        const uint32_t mask = (1u << pb) - 1u, bins = mask + 1u;
        for (uint32_t b = lane; b < bins; b += 64) wcnt[w][b] = 0;
        wave_lds_sync();
#pragma unroll
        for (int r = 0; r < IT_MAX; ++r) {
            if (r >= (int)IT) break;
            const uint32_t e = (w * IT + r) * 64 + lane;
            const bool valid = e < P;
            const uint32_t d = (v[r] >> shift) & mask;
            uint64_t peers = __ballot(valid);
#pragma unroll
            for (int b = 0; b < BITS; ++b) {
                if (b >= pb) break;
                const uint64_t bb = __ballot(valid && ((d >> b) & 1u));
                peers &= ((d >> b) & 1u) ? bb : ~bb;
            }
            const uint32_t rank = (uint32_t)__popcll(peers & lt);
            const uint32_t before = valid ? wcnt[w][d] : 0u;
            wave_lds_sync();
            if (valid && rank == 0) wcnt[w][d] = before + (uint32_t)__popcll(peers);
            lrank[r] = before + rank;
            wave_lds_sync();
        }
        st();
        {
            uint32_t tot = 0;
            if (tid < bins)                                      // THREADS >= BINS
#pragma unroll
                for (int ww = 0; ww < WAVES; ++ww) { const uint32_t x = wcnt[ww][tid]; wcnt[ww][tid] = tot; tot += x; }
            const uint32_t inc = wave_incl_scan(tot);
            if (lane == 63) wsum[w] = inc;
            __syncthreads();
            uint32_t ex = inc - tot;
            for (uint32_t ww = 0; ww < w; ++ww) ex += wsum[ww];
            if (tid < bins) run[tid] = ex;
        }
        st();
#pragma unroll
        for (int r = 0; r < IT_MAX; ++r) {
            if (r >= (int)IT) break;
            const uint32_t e = (w * IT + r) * 64 + lane;
            if (e < P) {
                const uint32_t d = (v[r] >> shift) & mask;
                sh[run[d] + wcnt[w][d] + lrank[r]] = v[r];
            }
        }
        st();
#pragma unroll
        for (int r = 0; r < IT_MAX; ++r) {
            if (r >= (int)IT) break;
            const uint32_t e = (w * IT + r) * 64 + lane;
            v[r] = e < P ? sh[e] : 0u;
        }
        st();
        shift += pb;
        left -= pb;
    }
#pragma unroll
    for (int r = 0; r < IT_MAX; ++r) {
        if (r >= (int)IT) break;
        const uint32_t e = (w * IT + r) * 64 + lane;
        if (e < P) comp[e] = v[r];
    }
    st();
}

template <int THREADS>
void run(uint32_t P, const uint32_t *dk, uint32_t *dc, unsigned long long *ds, const std::vector<uint32_t> &want)
{
    const uint32_t ib = 13;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(bsort<THREADS>, dim3(1), dim3(THREADS), 0, 0, P, ib, 17, dk, dc, ds);
    CK(hipEventRecord(a));
    const int R = 200;
    for (int i = 0; i < R; ++i) hipLaunchKernelGGL(bsort<THREADS>, dim3(1), dim3(THREADS), 0, 0, P, ib, 17, dk, dc, ds);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<uint32_t> got(P);
    unsigned long long s[16];
    CK(hipMemcpy(got.data(), dc, P * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(s, ds, sizeof(s), hipMemcpyDeviceToHost));
    printf("threads %4d P %5u: %.2f us/launch, ok %d; stamps (s_memtime ticks from start):", THREADS, P, ms * 1e3 / R,
           (int)(got == want));
    for (int i = 1; i < 13; ++i) printf(" %llu", s[i] - s[0]);
    printf("\n");
}

int main()
{
    for (uint32_t P : {8192u, 16384u, 2048u}) {
        std::vector<uint32_t> k(P), want(P);
        uint64_t x = 12345;
        for (uint32_t i = 0; i < P; ++i) {
            x = x * 6364136223846793005ull + 1442695040888963407ull;
            k[i] = (uint32_t)(x >> 40) % 100000u;
            want[i] = (k[i] << 13) | i;
        }
        std::sort(want.begin(), want.end());
        uint32_t *dk, *dc;
        unsigned long long *ds;
        CK(hipMalloc(&dk, P * 4)); CK(hipMalloc(&dc, P * 4)); CK(hipMalloc(&ds, 16 * 8));
        CK(hipMemcpy(dk, k.data(), P * 4, hipMemcpyHostToDevice));
        run<1024>(P, dk, dc, ds, want);
        run<512>(P, dk, dc, ds, want);
        CK(hipFree(dk)); CK(hipFree(dc)); CK(hipFree(ds));
    }
    return 0;
}
