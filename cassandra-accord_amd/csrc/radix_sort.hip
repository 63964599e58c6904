// Stable LSD radix sort of (u32 key, u32 value) pairs, 8-bit digits (K2 of SURVEY.md §7:
// bucketing (key, txn) pairs into per-key CommandsForKey histories, CommandsForKey.java:415).
//
// Per pass: upsweep (per-tile digit histogram in LDS) -> exclusive scan of the digit-major
// [256][tiles] histogram -> downsweep (stable in-tile ranking with wave ballots, scatter).
// Stability matters: entries of one key must stay in TxnId (= input) order.
#include "device_common.h"
#include "kernels.h"

namespace accord {

namespace {
constexpr int RS_THREADS = 256;
constexpr int RS_ITEMS = 16;
constexpr int RS_TILE = RS_THREADS * RS_ITEMS;
constexpr int RS_BINS = 256;

__global__ __launch_bounds__(RS_THREADS) void rs_upsweep(const uint32_t *__restrict__ keys, uint32_t n, int shift,
                                                         uint32_t *__restrict__ hist, uint32_t tiles)
{
    __shared__ uint32_t h[RS_BINS];
    const uint32_t tid = threadIdx.x;
    h[tid] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * RS_TILE;
#pragma unroll 4
    for (int j = 0; j < RS_ITEMS; ++j) {
        uint32_t idx = base + j * RS_THREADS + tid;
        if (idx < n) atomicAdd(&h[(keys[idx] >> shift) & 0xFF], 1u);
    }
    __syncthreads();
    hist[tid * tiles + blockIdx.x] = h[tid];
}

__global__ __launch_bounds__(RS_THREADS) void rs_downsweep(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                           uint32_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                           uint32_t n, int shift, const uint32_t *__restrict__ offs,
                                                           uint32_t tiles)
{
    __shared__ uint32_t run[RS_BINS];
    __shared__ uint32_t wcnt[RS_THREADS / 64][RS_BINS];
    const uint32_t tid = threadIdx.x, w = tid >> 6;
    run[tid] = offs[tid * tiles + blockIdx.x];
    const uint64_t lt = lanemask_lt();
    const uint32_t base = blockIdx.x * RS_TILE;
    for (int r = 0; r < RS_ITEMS; ++r) {
        if (base + r * RS_THREADS >= n) break;                 // block-uniform
#pragma unroll
        for (int ww = 0; ww < RS_THREADS / 64; ++ww) wcnt[ww][tid] = 0;
        __syncthreads();
        const uint32_t idx = base + r * RS_THREADS + tid;
        const bool valid = idx < n;
        uint32_t key = 0, val = 0, d = 0;
        if (valid) { key = kin[idx]; val = vin[idx]; d = (key >> shift) & 0xFF; }
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            uint64_t bb = __ballot(valid && ((d >> b) & 1));
            peers &= ((d >> b) & 1) ? bb : ~bb;
        }
        const uint32_t rank = __popcll(peers & lt);
        if (valid && rank == 0) wcnt[w][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pos = run[d] + rank;
            for (uint32_t ww = 0; ww < w; ++ww) pos += wcnt[ww][d];
            kout[pos] = key;
            vout[pos] = val;
        }
        __syncthreads();
        uint32_t add = 0;
#pragma unroll
        for (int ww = 0; ww < RS_THREADS / 64; ++ww) add += wcnt[ww][tid];
        run[tid] += add;
        __syncthreads();
    }
}
} // namespace

size_t radix_sort_temp_bytes(uint32_t n)
{
    uint32_t tiles = (n + RS_TILE - 1) / RS_TILE;
    size_t hist = (size_t)RS_BINS * (tiles ? tiles : 1);
    size_t a = ((hist * 4 + (hist + 1) * 4) + 15) & ~(size_t)15;
    return a + 16 + scan_temp_bytes((uint32_t)hist);
}

void radix_sort_pairs(const uint32_t *keys_in, const uint32_t *vals_in, uint32_t *keys_out, uint32_t *vals_out,
                      uint32_t *keys_tmp, uint32_t *vals_tmp, uint32_t n, int bits, void *temp, hipStream_t s)
{
    if (n == 0) return;
    const uint32_t tiles = (n + RS_TILE - 1) / RS_TILE;
    const size_t hist_n = (size_t)RS_BINS * tiles;
    uint32_t *hist = (uint32_t *)temp;
    uint32_t *offs = hist + hist_n;
    const size_t a = ((hist_n * 4 + (hist_n + 1) * 4) + 15) & ~(size_t)15;
    unsigned long long *total = (unsigned long long *)((char *)temp + a);
    void *scan_tmp = (char *)temp + a + 16;
    int passes = (bits + 7) / 8;
    if (passes < 1) passes = 1;
    // ping-pong so that the last pass lands in *_out
    const uint32_t *ki = keys_in, *vi = vals_in;
    for (int p = 0; p < passes; ++p) {
        const bool to_out = ((passes - 1 - p) % 2) == 0;
        uint32_t *ko = to_out ? keys_out : keys_tmp;
        uint32_t *vo = to_out ? vals_out : vals_tmp;
        const int shift = p * 8;
        hipLaunchKernelGGL(rs_upsweep, dim3(tiles), dim3(RS_THREADS), 0, s, ki, n, shift, hist, tiles);
        exclusive_scan_u32(hist, offs, (uint32_t)hist_n, total, scan_tmp, s);
        hipLaunchKernelGGL(rs_downsweep, dim3(tiles), dim3(RS_THREADS), 0, s, ki, vi, ko, vo, n, shift, offs, tiles);
        ki = ko; vi = vo;
    }
}

} // namespace accord
