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
// ---- a resident store's batch joining its carried history: sort the batch, merge ----
// The carry is key-major already (TxnId order inside a key) and the batch's pairs are in TxnId
// order, so a batch of up to 16 Ki pairs is sorted apart and merged instead of re-sorting [carry |
// batch] (six launches over C + P entries).  Every workgroup sorts one chunk of 1024 pairs as
// (key << ib | pair index) composites -- a thread per pair, LSD passes of <= 9 key bits ranked with
// wave ballots, re-ordered through LDS -- and every entry of the carry and of the chunks then finds
// its place by counting, in each other run, the entries that precede it: carry entry i of key k goes
// to i + #(batch keys < k); a batch pair of composite c and key k at position t of its chunk to
// t + #(carry keys <= k) + #(other chunks' composites < c) -- the carry's entries of a key first, then
// the batch's in TxnId order, as the stable sort of [carry | batch] put them.  The searches of one
// entry run in lockstep (one load per run per step in flight).  (One workgroup sorting the whole
// batch took 22 us for 8 Ki pairs: the ballot ranking is VALU-bound on one CU,
// scripts/micro/batch_sort.hip.)
constexpr uint32_t MS_CHUNK = 1024, MS_RUNS = 16, MS_MAX = MS_CHUNK * MS_RUNS;
constexpr int MS_WAVES = MS_CHUNK / 64, MS_BITS = 9, MS_BINS = 1 << MS_BITS;

__global__ __launch_bounds__(MS_CHUNK) void ms_chunk_sort_kernel(uint32_t P, uint32_t ib, int kbits,
                                                                 const uint32_t *__restrict__ bkey,
                                                                 uint32_t *__restrict__ comp)
{
    __shared__ uint32_t sh[MS_CHUNK];
    __shared__ uint32_t wcnt[MS_WAVES][MS_BINS];     // per wave and digit: count, then wave offset
    __shared__ uint32_t run[MS_BINS];
    __shared__ uint32_t wsum[MS_WAVES];
    const uint32_t tid = threadIdx.x, w = tid >> 6, lane = lane_id();
    const uint32_t base = blockIdx.x * MS_CHUNK, n = min(MS_CHUNK, P - base);
    const bool valid = tid < n;
    const uint64_t lt = lanemask_lt();
    uint32_t v = valid ? (bkey[base + tid] << ib) | (base + tid) : 0u;
    const int passes = (kbits + MS_BITS - 1) / MS_BITS;
    int shift = (int)ib, left = kbits;
    for (int p = 0; p < passes; ++p) {
        const int pb = left / (passes - p);
        const uint32_t mask = (1u << pb) - 1u, bins = mask + 1u;
        for (uint32_t b = lane; b < bins; b += 64) wcnt[w][b] = 0;
        const uint32_t d = (v >> shift) & mask;
        uint64_t peers = __ballot(valid);
        for (int b = 0; b < pb; ++b) {
            const uint64_t bb = __ballot(valid && ((d >> b) & 1u));
            peers &= ((d >> b) & 1u) ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        wave_lds_sync();
        if (valid && rank == 0) wcnt[w][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        {   // per digit: wave offsets (exclusive over waves), then the digits' exclusive scan
            uint32_t tot = 0;
            if (tid < bins)
#pragma unroll
                for (int ww = 0; ww < MS_WAVES; ++ww) { const uint32_t x = wcnt[ww][tid]; wcnt[ww][tid] = tot; tot += x; }
            const uint32_t inc = wave_incl_scan(tot);
            if (lane == 63) wsum[w] = inc;
            __syncthreads();
            uint32_t ex = inc - tot;
            for (uint32_t ww = 0; ww < w; ++ww) ex += wsum[ww];
            if (tid < bins) run[tid] = ex;
        }
        __syncthreads();
        if (valid) sh[run[d] + wcnt[w][d] + rank] = v;
        __syncthreads();
        v = valid ? sh[tid] : 0u;
        __syncthreads();
        shift += pb;
        left -= pb;
    }
    if (valid) comp[base + tid] = v;
}

// the chunks merged into one sorted run: every chunk in the LDS of each workgroup of 256 pairs; the
// pair goes to #(composites below it) summed over the chunks, the chunks
// searched in lockstep (one LDS read per chunk per step; 256-thread workgroups spread the searches'
// VALU work over P / 256 CUs -- a workgroup per 1024-pair chunk took 15 us for 8 Ki pairs)
constexpr uint32_t MS_MT = 256;
__global__ __launch_bounds__(MS_MT) void ms_chunk_merge_kernel(uint32_t P, const uint32_t *__restrict__ comp,
                                                               uint32_t *__restrict__ sorted)
{
    __shared__ uint32_t sh[MS_MAX];
    const uint32_t tid = threadIdx.x, nb = (P + MS_CHUNK - 1) / MS_CHUNK;
    for (uint32_t i0 = 0; i0 < P; i0 += MS_MT * 16) {     // 16 loads in flight per thread
        uint32_t t[16];
#pragma unroll
        for (uint32_t u = 0; u < 16; ++u) {
            const uint32_t i = i0 + u * MS_MT + tid;
            t[u] = i < P ? comp[i] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < 16; ++u) {
            const uint32_t i = i0 + u * MS_MT + tid;
            if (i < P) sh[i] = t[u];
        }
    }
    __syncthreads();
    const uint32_t g = blockIdx.x * MS_MT + tid;
    if (g >= P) return;
    const uint32_t c = sh[g];
    // every run counted, its own included (composites are distinct: there it counts t itself);
    // four runs searched together, branch-free steps (a fully unrolled 16-run search was 20 KB of
    // code and took 21 us, instruction fetch on cold CUs)
    uint32_t t = 0;
    for (uint32_t r0 = 0; r0 < nb; r0 += 4) {
        uint32_t pos[4], len[4];
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
            pos[u] = 0;
            len[u] = r0 + u < nb ? min(MS_CHUNK, P - (r0 + u) * MS_CHUNK) : 0u;
        }
#pragma unroll
        for (uint32_t step = MS_CHUNK; step >= 1; step >>= 1) {
            uint32_t v[4];
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u)
                v[u] = sh[min((r0 + u) * MS_CHUNK + min(pos[u] + step, max(len[u], 1u)) - 1, MS_MAX - 1)];
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u)
                if (pos[u] + step <= len[u] && v[u] < c) pos[u] += step;
        }
        t += pos[0] + pos[1] + pos[2] + pos[3];
    }
    sorted[t] = c;
}

// carry entry i of key k to i + #(batch keys < k), batch pair at position j of the sorted batch to
// j + #(carry keys <= k); branch-free searches (ctop, btop: the highest powers of two <= C, P)
__global__ __launch_bounds__(256) void ms_merge_kernel(uint32_t C, uint32_t P, uint32_t ib, uint32_t ctop, uint32_t btop,
                                                       const uint32_t *__restrict__ ckey, const uint32_t *__restrict__ cent,
                                                       const uint32_t *__restrict__ comp, const uint32_t *__restrict__ bent,
                                                       uint32_t *__restrict__ sort_key, uint32_t *__restrict__ sort_pair,
                                                       uint32_t *__restrict__ hist)
{
    const uint32_t mask = (1u << ib) - 1u;
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < C + P; x += gridDim.x * blockDim.x) {
        uint32_t k, pair, ent, pos;
        if (x < C) {
            k = ckey[x];
            const uint32_t c0 = k << ib;
            uint32_t lo = 0;
            for (uint32_t step = btop; step >= 1; step >>= 1)
                if (lo + step <= P && comp[lo + step - 1] < c0) lo += step;
            pos = x + lo; pair = x; ent = cent[x];
        } else {
            const uint32_t j = x - C, c = comp[j], q = c & mask;
            k = c >> ib;
            uint32_t lo = 0;
            for (uint32_t step = ctop; step >= 1; step >>= 1)
                if (lo + step <= C && ckey[lo + step - 1] <= k) lo += step;
            pos = j + lo; pair = C + q; ent = bent[q];
        }
        sort_key[pos] = k;
        sort_pair[pos] = pair;
        hist[pos] = ent;
    }
}
} // namespace

inline uint32_t ms_index_bits(uint32_t P)
{
    uint32_t ib = 0;
    while ((1u << ib) < P) ++ib;
    return ib;
}

bool merge_join_fits(uint32_t P, int bits)
{
    return P >= 1 && P <= MS_MAX && std::max(bits, 1) + (int)ms_index_bits(P) <= 31;
}

void merge_join_batch(const uint32_t *ckey, const uint32_t *cent, uint32_t C, const uint32_t *bkey,
                      const uint32_t *bent, uint32_t P, int bits, uint32_t *comp_tmp, uint32_t *sorted_tmp,
                      uint32_t *sort_key, uint32_t *sort_pair, uint32_t *hist, hipStream_t s)
{
    const uint32_t ib = ms_index_bits(P), nb = (P + MS_CHUNK - 1) / MS_CHUNK;
    hipLaunchKernelGGL(ms_chunk_sort_kernel, dim3(nb), dim3(MS_CHUNK), 0, s, P, ib, std::max(bits, 1), bkey, comp_tmp);
    hipLaunchKernelGGL(ms_chunk_merge_kernel, dim3((P + MS_MT - 1) / MS_MT), dim3(MS_MT), 0, s, P, comp_tmp, sorted_tmp);
    uint32_t ctop = 1, btop = 1;
    while (ctop * 2 <= C) ctop *= 2;
    while (btop * 2 <= P) btop *= 2;
    const uint32_t total = C + P;
    const uint32_t b = std::min<uint32_t>((total + 255) / 256, 8192u);
    hipLaunchKernelGGL(ms_merge_kernel, dim3(b), dim3(256), 0, s, C, P, ib, ctop, btop, ckey, cent, sorted_tmp, bent, sort_key,
                       sort_pair, hist);
}

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
