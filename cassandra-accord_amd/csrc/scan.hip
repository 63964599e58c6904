// Exclusive prefix sum of u32 counts (CSR offsets of the per-txn PartialDeps and radix digit
// offsets).  Three launches: tile reduce -> scan of tile sums (one block) -> tile scan + apply.
// Totals are carried in u64 so an overflow of the u32 offset space is detectable on the host.
#include "device_common.h"
#include "kernels.h"

namespace accord {

namespace {
constexpr int SC_THREADS = 256;
constexpr int SC_ITEMS = 16;
constexpr int SC_TILE = SC_THREADS * SC_ITEMS;

__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t *wsum, uint64_t *total)
{
    const uint32_t tid = threadIdx.x, w = tid >> 6, l = lane_id();
    uint64_t inc = wave_incl_scan64(v);
    if (l == 63) wsum[w] = inc;
    __syncthreads();
    uint64_t off = 0, tot = 0;
#pragma unroll
    for (int i = 0; i < SC_THREADS / 64; ++i) {
        if ((uint32_t)i < w) off += wsum[i];
        tot += wsum[i];
    }
    *total = tot;
    __syncthreads();
    return off + inc - v;
}

__global__ __launch_bounds__(SC_THREADS) void sc_reduce(const uint32_t *__restrict__ in, uint32_t n,
                                                        unsigned long long *__restrict__ sums)
{
    __shared__ uint64_t wsum[SC_THREADS / 64];
    const uint32_t base = blockIdx.x * SC_TILE;
    uint64_t acc = 0;
#pragma unroll 4
    for (int j = 0; j < SC_ITEMS; ++j) {
        uint32_t idx = base + j * SC_THREADS + threadIdx.x;
        if (idx < n) acc += in[idx];
    }
    for (int d = 32; d >= 1; d >>= 1) acc += __shfl_xor(acc, d, 64);
    if (lane_id() == 0) wsum[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int i = 0; i < SC_THREADS / 64; ++i) t += wsum[i];
        sums[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(SC_THREADS) void sc_scan_sums(unsigned long long *__restrict__ sums, uint32_t m,
                                                           unsigned long long *__restrict__ total)
{
    __shared__ uint64_t wsum[SC_THREADS / 64];
    uint64_t carry = 0;
    for (uint32_t base = 0; base < m; base += SC_THREADS) {
        uint32_t idx = base + threadIdx.x;
        uint64_t v = idx < m ? sums[idx] : 0;
        uint64_t tot;
        uint64_t ex = block_excl_scan64(v, wsum, &tot);
        if (idx < m) sums[idx] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(SC_THREADS) void sc_apply(const uint32_t *__restrict__ in, uint32_t *__restrict__ out,
                                                       uint32_t n, const unsigned long long *__restrict__ sums,
                                                       const unsigned long long *__restrict__ total)
{
    __shared__ uint32_t tile[SC_TILE];
    __shared__ uint64_t wsum[SC_THREADS / 64];
    const uint32_t base = blockIdx.x * SC_TILE, tid = threadIdx.x;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        uint32_t idx = base + j * SC_THREADS + tid;
        tile[j * SC_THREADS + tid] = idx < n ? in[idx] : 0;
    }
    __syncthreads();
    uint64_t local = 0;
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) local += tile[tid * SC_ITEMS + j];
    uint64_t tot;
    uint64_t run = block_excl_scan64(local, wsum, &tot) + sums[blockIdx.x];
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        uint32_t v = tile[tid * SC_ITEMS + j];
        tile[tid * SC_ITEMS + j] = (uint32_t)run;
        run += v;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SC_ITEMS; ++j) {
        uint32_t idx = base + j * SC_THREADS + tid;
        if (idx < n) out[idx] = tile[j * SC_THREADS + tid];
    }
    if (blockIdx.x == gridDim.x - 1 && tid == 0) out[n] = (uint32_t)*total;
}
} // namespace

size_t scan_temp_bytes(uint32_t n)
{
    uint32_t tiles = (n + SC_TILE - 1) / SC_TILE;
    return ((size_t)(tiles ? tiles : 1) + 2) * sizeof(unsigned long long);
}

void exclusive_scan_u32(const uint32_t *in, uint32_t *out, uint32_t n, unsigned long long *total_dev, void *temp,
                        hipStream_t s)
{
    uint32_t tiles = (n + SC_TILE - 1) / SC_TILE;
    if (tiles == 0) tiles = 1;
    unsigned long long *sums = (unsigned long long *)temp;
    hipLaunchKernelGGL(sc_reduce, dim3(tiles), dim3(SC_THREADS), 0, s, in, n, sums);
    hipLaunchKernelGGL(sc_scan_sums, dim3(1), dim3(SC_THREADS), 0, s, sums, tiles, total_dev);
    hipLaunchKernelGGL(sc_apply, dim3(tiles), dim3(SC_THREADS), 0, s, in, out, n, sums, total_dev);
}

} // namespace accord
