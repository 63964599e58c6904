// Levelling resolver micro-benchmark: the serial max-plus step of one wave -- acc[row] = max over L
// late columns of (bv[col] + d[row][col]), bv of the next step taken from this step's acc (so every
// step waits on the previous one, as the chain does) -- in several broadcast forms, cycles per step.
// Build: hipcc --offload-arch=gfx950 -O3 -o lv_product lv_product.hip ; run: ./lv_product
#include <hip/hip_runtime.h>
#include <cstdio>
#include <climits>

constexpr int STEPS = 20000;

template <int L, int MODE>
__global__ __launch_bounds__(64) void k(const int *__restrict__ dsrc, const int *__restrict__ perm, int *out,
                                        unsigned long long *cyc)
{
    __shared__ __attribute__((aligned(16))) int sb[64 + 4];
    const int lane = threadIdx.x;
    int d[L];
#pragma unroll
    for (int c = 0; c < L; ++c) d[c] = dsrc[c * 64 + lane];
    const int src = perm[lane];            // the late predecessor of column `lane` in the previous step
    int acc = lane;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int s = 0; s < STEPS; ++s) {
        // the late bases: each column's predecessor value from the previous step (lane permute)
        const int bv = __builtin_amdgcn_ds_bpermute(src << 2, acc) + 1;
        int a0 = INT_MIN + 64, a1 = INT_MIN + 64;
        if (MODE == 0) {                   // v_readlane into SGPRs
#pragma unroll
            for (int c = 0; c < L; c += 2) {
                const int s0 = __builtin_amdgcn_readlane(bv, c), s1 = __builtin_amdgcn_readlane(bv, c + 1);
                a0 = max(a0, s0 + d[c]);
                a1 = max(a1, s1 + d[c + 1]);
            }
        } else if (MODE == 1) {            // LDS round trip, uniform-address b128 broadcast reads
            sb[lane] = bv;
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int c = 0; c < L; c += 4) {
                const int4 v = *(const int4 *)&sb[c];
                a0 = max(a0, max(v.x + d[c], v.y + d[c + 1]));
                a1 = max(a1, max(v.z + d[c + 2], v.w + d[c + 3]));
            }
        } else {                           // ds_bpermute broadcast per column
#pragma unroll
            for (int c = 0; c < L; c += 2) {
                const int s0 = __builtin_amdgcn_ds_bpermute(c << 2, bv), s1 = __builtin_amdgcn_ds_bpermute((c + 1) << 2, bv);
                a0 = max(a0, s0 + d[c]);
                a1 = max(a1, s1 + d[c + 1]);
            }
        }
        acc = max(a0, a1) & 0xFFFFF;       // keep values bounded
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[lane] = acc;
    if (lane == 0) *cyc = t1 - t0;
}

template <int L, int MODE>
void run(const int *d, const int *perm, int *out, unsigned long long *cyc, const char *name)
{
    hipLaunchKernelGGL((k<L, MODE>), dim3(1), dim3(64), 0, 0, d, perm, out, cyc);
    hipLaunchKernelGGL((k<L, MODE>), dim3(1), dim3(64), 0, 0, d, perm, out, cyc);
    unsigned long long h = 0;
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    // s_memtime counts at the 100 MHz reference clock on CDNA; report both raw and per step
    printf("%-22s L=%2d: %8.2f s_memtime cycles per step\n", name, L, (double)h / STEPS);
}

int main()
{
    int *d, *perm, *out;
    unsigned long long *cyc;
    hipMalloc(&d, 64 * 64 * 4);
    hipMalloc(&perm, 64 * 4);
    hipMalloc(&out, 64 * 4);
    hipMalloc(&cyc, 8);
    int hd[64 * 64], hp[64];
    for (int i = 0; i < 64 * 64; ++i) hd[i] = (i * 7919) % 5 == 0 ? INT_MIN / 2 : (i * 31) % 64 + 1;
    for (int i = 0; i < 64; ++i) hp[i] = (i * 37 + 11) % 64;
    hipMemcpy(d, hd, sizeof(hd), hipMemcpyHostToDevice);
    hipMemcpy(perm, hp, sizeof(hp), hipMemcpyHostToDevice);
    run<16, 0>(d, perm, out, cyc, "readlane");
    run<32, 0>(d, perm, out, cyc, "readlane");
    run<48, 0>(d, perm, out, cyc, "readlane");
    run<16, 1>(d, perm, out, cyc, "lds-broadcast-b128");
    run<32, 1>(d, perm, out, cyc, "lds-broadcast-b128");
    run<48, 1>(d, perm, out, cyc, "lds-broadcast-b128");
    run<16, 2>(d, perm, out, cyc, "bpermute");
    run<32, 2>(d, perm, out, cyc, "bpermute");
    run<48, 2>(d, perm, out, cyc, "bpermute");
    // the chain alone (L = 0 columns is not instantiable): one bpermute + max per step
    return 0;
}
