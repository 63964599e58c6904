// Stable LSD radix sort of (u32 key, u32 value) pairs (K2 of SURVEY.md §7: bucketing the
// batch's (key, txn) pairs into per-key CommandsForKey histories, CommandsForKey.java:415).
//
// Per pass (digit of <= 9 bits, so a 17-bit keyspace needs 2 passes):
//   upsweep   : per-tile digit histogram in LDS -> digit-major [bins][tiles] counts
//   scan      : exclusive scan of the counts (scan.hip) -> global offset per (digit, tile)
//   downsweep : stable in-tile ranking with wave ballots, the tile is re-ordered by digit in LDS
//               and written out as contiguous per-digit runs (coalesced stores).
// Stability keeps the entries of one key in TxnId (= input) order.  An optional second value
// (the history entry of each pair) rides along, so the key-major history is produced by the sort
// itself instead of by a random gather afterwards.
#include "device_common.h"
#include "kernels.h"

#include <cstdlib>

namespace accord {

namespace {
constexpr int RS_THREADS = 256;
constexpr int RS_WAVES = RS_THREADS / 64;
// items per thread: 16 for large sorts; a sort too small to give every CU several tiles of 4096
// (a resident store's batch) takes tiles of 1024 instead, so the grid still fills the chip
constexpr int RS_ITEMS_MAX = 16;
constexpr uint32_t RS_SMALL_N = 1u << 22;
__host__ __device__ constexpr int rs_tile(int items) { return RS_THREADS * items; }
constexpr int RS_MAX_BITS = 9;
constexpr int RS_MAX_BINS = 1 << RS_MAX_BITS;

template <int RS_ITEMS>
__global__ __launch_bounds__(RS_THREADS) void rs_upsweep(const uint32_t *__restrict__ keys, uint32_t n, int shift,
                                                         uint32_t mask, uint32_t *__restrict__ hist, uint32_t tiles)
{
    constexpr int RS_TILE = rs_tile(RS_ITEMS);
    __shared__ uint32_t h[RS_MAX_BINS];
    const uint32_t tid = threadIdx.x, bins = mask + 1;
    for (uint32_t b = tid; b < bins; b += RS_THREADS) h[b] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * RS_TILE;
#pragma unroll 4
    for (int j = 0; j < RS_ITEMS; ++j) {
        uint32_t idx = base + j * RS_THREADS + tid;
        if (idx < n) atomicAdd(&h[(keys[idx] >> shift) & mask], 1u);
    }
    __syncthreads();
    for (uint32_t b = tid; b < bins; b += RS_THREADS) hist[b * tiles + blockIdx.x] = h[b];
}

// Downsweep: every wave ranks its own contiguous quarter of the tile (16 rounds of 64 items) with
// wave ballots against a wave-private running digit count in LDS -- no block barrier per round --
// then one block scan of the digit totals places each wave's runs, the tile is re-ordered by digit
// in LDS and written out as contiguous per-digit runs.
template <int BITS, int RS_ITEMS>
__global__ __launch_bounds__(RS_THREADS) void rs_downsweep(const uint32_t *__restrict__ kin, const uint32_t *__restrict__ vin,
                                                           uint32_t *__restrict__ kout, uint32_t *__restrict__ vout,
                                                           const uint32_t *__restrict__ ein, uint32_t *__restrict__ eout,
                                                           uint32_t n, int shift, uint32_t mask,
                                                           const uint32_t *__restrict__ offs, uint32_t tiles)
{
    constexpr uint32_t BINS = 1u << BITS;       // LDS sizing; digits use the runtime mask (<= BINS-1)
    constexpr int RS_TILE = rs_tile(RS_ITEMS);
    const uint32_t MASK = mask;
    __shared__ uint32_t s_keys[RS_TILE];
    __shared__ uint32_t s_vals[RS_TILE];
    __shared__ uint32_t run[BINS];              // exclusive tile start of digit d
    __shared__ uint32_t glob[BINS];             // global offset of this tile's digit-d run
    __shared__ uint32_t wcnt[RS_WAVES][BINS];   // wave-private running counts, then wave offsets
    __shared__ uint32_t wsum[RS_WAVES];
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    for (uint32_t b = tid; b < BINS; b += RS_THREADS) glob[b] = b <= mask ? offs[b * tiles + blockIdx.x] : 0u;
    for (uint32_t b = tid; b < RS_WAVES * BINS; b += RS_THREADS) (&wcnt[0][0])[b] = 0;
    const uint64_t lt = lanemask_lt();
    const uint32_t base = blockIdx.x * RS_TILE;
    const uint32_t tile_n = min((uint32_t)RS_TILE, n - base);
    const uint32_t wbase = base + w * (RS_ITEMS * 64);

    uint32_t key[RS_ITEMS], val[RS_ITEMS], ent[RS_ITEMS], lrank[RS_ITEMS];
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        const uint32_t idx = wbase + r * 64 + lane;
        key[r] = idx < n ? kin[idx] : 0u;
        val[r] = idx < n ? (vin ? vin[idx] : idx) : 0u;
        ent[r] = (ein && idx < n) ? ein[idx] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        const uint32_t idx = wbase + r * 64 + lane;
        const bool valid = idx < n;
        const uint32_t d = (key[r] >> shift) & MASK;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < BITS; ++b) {
            const uint64_t bb = __ballot(valid && ((d >> b) & 1));
            peers &= ((d >> b) & 1) ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        const uint32_t before = valid ? wcnt[w][d] : 0u;
        wave_lds_sync();
        if (valid && rank == 0) wcnt[w][d] = before + (uint32_t)__popcll(peers);
        lrank[r] = before + rank;                 // rank among this wave's items of digit d
        wave_lds_sync();
    }
    __syncthreads();
    // digit totals of the tile, wave offsets per digit, exclusive scan over digits
    {
        constexpr uint32_t PER = (BINS + RS_THREADS - 1) / RS_THREADS;
        uint32_t c[PER], s = 0;
#pragma unroll
        for (uint32_t q = 0; q < PER; ++q) {
            const uint32_t b = tid * PER + q;
            uint32_t tot = 0;
            if (b < BINS) {
#pragma unroll
                for (int ww = 0; ww < RS_WAVES; ++ww) { const uint32_t x = wcnt[ww][b]; wcnt[ww][b] = tot; tot += x; }
            }
            c[q] = tot;
            s += tot;
        }
        const uint32_t inc = wave_incl_scan(s);
        if (lane == 63) wsum[w] = inc;
        __syncthreads();
        uint32_t ex = inc - s;
        for (uint32_t ww = 0; ww < w; ++ww) ex += wsum[ww];
#pragma unroll
        for (uint32_t q = 0; q < PER; ++q) {
            const uint32_t b = tid * PER + q;
            if (b < BINS) run[b] = ex;
            ex += c[q];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RS_ITEMS; ++r) {
        const uint32_t idx = wbase + r * 64 + lane;
        if (idx < n) {
            const uint32_t d = (key[r] >> shift) & MASK;
            const uint32_t q = run[d] + wcnt[w][d] + lrank[r];
            s_keys[q] = key[r];
            s_vals[q] = val[r];
        }
    }
    __syncthreads();
    for (uint32_t q = tid; q < tile_n; q += RS_THREADS) {
        const uint32_t k = s_keys[q];
        const uint32_t d = (k >> shift) & MASK;
        const uint32_t g = glob[d] + (q - run[d]);
        kout[g] = k;
        vout[g] = s_vals[q];
    }
    if (ein) {                                   // second value: same placement through s_vals
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RS_ITEMS; ++r) {
            const uint32_t idx = wbase + r * 64 + lane;
            if (idx < n) {
                const uint32_t d = (key[r] >> shift) & MASK;
                s_vals[run[d] + wcnt[w][d] + lrank[r]] = ent[r];
            }
        }
        __syncthreads();
        for (uint32_t q = tid; q < tile_n; q += RS_THREADS) {
            const uint32_t d = (s_keys[q] >> shift) & MASK;
            eout[glob[d] + (q - run[d])] = s_vals[q];
        }
    }
}
} // namespace

inline int rs_items(uint32_t n) { return n < RS_SMALL_N ? 4 : RS_ITEMS_MAX; }
inline uint32_t rs_tiles(uint32_t n) { return (n + rs_tile(rs_items(n)) - 1) / rs_tile(rs_items(n)); }

size_t radix_sort_temp_bytes(uint32_t n)
{
    uint32_t tiles = rs_tiles(n);
    size_t hist = (size_t)RS_MAX_BINS * (tiles ? tiles : 1);
    size_t a = ((hist * 4 + (hist + 1) * 4) + 15) & ~(size_t)15;
    return a + 16;
}

uint32_t radix_sort_scan_len(uint32_t n)
{
    uint32_t tiles = rs_tiles(n);
    return (uint32_t)RS_MAX_BINS * (tiles ? tiles : 1);
}

void radix_sort_pairs(const uint32_t *keys_in, const uint32_t *vals_in, uint32_t *keys_out, uint32_t *vals_out,
                      uint32_t *keys_tmp, uint32_t *vals_tmp, const uint32_t *ents_in, uint32_t *ents_out,
                      uint32_t *ents_tmp, uint32_t n, int bits, void *temp, void *scan_state, hipStream_t s)
{
    if (n == 0) return;
    const uint32_t tiles = rs_tiles(n);
    const bool small = rs_items(n) != RS_ITEMS_MAX;
    const size_t hist_cap = (size_t)RS_MAX_BINS * tiles;
    uint32_t *hist = (uint32_t *)temp;
    uint32_t *offs = hist + hist_cap;
    const size_t a = ((hist_cap * 4 + (hist_cap + 1) * 4) + 15) & ~(size_t)15;
    unsigned long long *total = (unsigned long long *)((char *)temp + a);
    if (bits < 1) bits = 1;
    int passes = (bits + RS_MAX_BITS - 1) / RS_MAX_BITS;
    // the narrower digit first: the first pass moves two arrays (keys, entries) and the second three,
    // and the 9-bit downsweep is the slower one (config 2, 17-bit keys: 8 + 9 bits sorts in 0.212 ms
    // against 0.224 for 9 + 8, profiles/r04_b/sort_ab.txt; 3 passes of fewer bits: 0.244 ms)
    const bool low_first = true;
    // ping-pong so that the last pass lands in *_out; vals_in == nullptr means identity values
    const uint32_t *ki = keys_in, *vi = vals_in, *ei = ents_in;
    int shift = 0;
    for (int p = 0; p < passes; ++p) {
        const int pb = low_first ? (bits - shift) / (passes - p)                  // split bits evenly
                                 : (bits - shift + (passes - p) - 1) / (passes - p);
        const uint32_t mask = (1u << pb) - 1;
        const bool to_out = ((passes - 1 - p) % 2) == 0;
        uint32_t *ko = to_out ? keys_out : keys_tmp;
        uint32_t *vo = to_out ? vals_out : vals_tmp;
        uint32_t *eo = ents_in ? (to_out ? ents_out : ents_tmp) : nullptr;
        const size_t hist_n = (size_t)(mask + 1) * tiles;
        if (small) hipLaunchKernelGGL(rs_upsweep<4>, dim3(tiles), dim3(RS_THREADS), 0, s, ki, n, shift, mask, hist, tiles);
        else hipLaunchKernelGGL(rs_upsweep<RS_ITEMS_MAX>, dim3(tiles), dim3(RS_THREADS), 0, s, ki, n, shift, mask, hist, tiles);
        exclusive_scan_u32(hist, offs, (uint32_t)hist_n, total, scan_state, s);
        if (pb > 8) {
            if (small)
                hipLaunchKernelGGL((rs_downsweep<9, 4>), dim3(tiles), dim3(RS_THREADS), 0, s, ki, vi, ko, vo, ei, eo, n, shift, mask, offs, tiles);
            else
                hipLaunchKernelGGL((rs_downsweep<9, RS_ITEMS_MAX>), dim3(tiles), dim3(RS_THREADS), 0, s, ki, vi, ko, vo, ei, eo, n, shift, mask, offs, tiles);
        } else {
            if (small)
                hipLaunchKernelGGL((rs_downsweep<8, 4>), dim3(tiles), dim3(RS_THREADS), 0, s, ki, vi, ko, vo, ei, eo, n, shift, mask, offs, tiles);
            else
                hipLaunchKernelGGL((rs_downsweep<8, RS_ITEMS_MAX>), dim3(tiles), dim3(RS_THREADS), 0, s, ki, vi, ko, vo, ei, eo, n, shift, mask, offs, tiles);
        }
        ki = ko; vi = vo; ei = eo;
        shift += pb;
    }
}

} // namespace accord
