// KeyDeps construction for a PreAccept batch (SURVEY.md §8a rows a3 + a8, kernels K2-K4).
//
// Reference semantics (paths relative to accord-core/src/main/java/accord/):
//   CommandsForKey.mapReduceActive          local/CommandsForKey.java:614-650
//   PreAccept.calculatePartialDeps          messages/PreAccept.java:245-265
//   RelationMultiMap.AbstractBuilder.build  utils/RelationMultiMap.java:201-260
//   KeyDeps layout                          primitives/KeyDeps.java:150-187
// Under the status-at-time model the deps of (txn i, key) are the entries of
// the key's history (all (key, txn) pairs of the batch sorted by TxnId) in [lcw, i) whose kind
// is witnessed by kind(i), where lcw is the last Write entry j < i-W (APPLIED, so it bounds
// PRUNE_TRANSITIVE_DEPENDENCIES at :620-645) or the start of the history.
//
// One wave builds one txn's KeyDeps:
//   slots   : lanes < k locate each key's segment [lo, pos) by binary search (+ walk back to lcw)
//   phase 1 : the wave streams the raw entries of all slots; witnessed ones set a bit in an LDS
//             bitmap over [i-SPAN, i) ("near") or go to an LDS list ("far")
//   union   : |txnIds| = #distinct far + popcount(bitmap); ranks = prefix popcounts
//   fill    : txnIds (ascending == TxnId order), keysToTxnIds header (end offsets starting at
//             keyCount) and body (rank of every witnessed entry, in key order)
// The count pass writes per-txn sizes; an exclusive scan gives the CSR offsets; the fill pass
// recomputes and writes.
#include "device_common.h"
#include "kernels.h"

#include <cstdlib>
#include "../../include/accord_deps.h"

namespace accord {

namespace {

constexpr int KD_WAVES = 4;
constexpr int KD_THREADS = KD_WAVES * 64;
constexpr uint32_t KD_KCAP = 64;
constexpr uint32_t KD_FARCAP = 256;

__device__ __forceinline__ void record_error(DevStatus *st, uint32_t i, int32_t code)
{
    unsigned long long v = ((unsigned long long)i << 32) | (uint32_t)(-code);
    atomicMin(&st->first, v);
}

// Txn-major validation and pair packing.  One wave owns 64 consecutive txns; the pairs of those
// txns are then streamed 64 at a time (coalesced) and each lane finds its owner txn with a
// shuffle binary search over the wave's key offsets.
__global__ __launch_bounds__(256) void validate_pack_kernel(
    uint32_t n, const uint64_t *__restrict__ msb, const uint64_t *__restrict__ lsb, const int32_t *__restrict__ node,
    const uint32_t *__restrict__ key_off, const uint32_t *__restrict__ key_ord, const uint32_t *__restrict__ rng_off,
    const uint32_t *__restrict__ rng_start, const uint32_t *__restrict__ rng_end, uint32_t key_lo, uint32_t key_hi,
    uint32_t *__restrict__ pair_key, uint32_t *__restrict__ pair_ent, uint32_t *__restrict__ rng_owner,
    uint32_t *__restrict__ is_range, const uint32_t *__restrict__ txn_index, StreamPos sp, DevStatus *st)
{
    const uint32_t lane = lane_id();
    const uint32_t gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t t0 = gw * 64; t0 < n; t0 += nw * 64) {
        const uint32_t t = t0 + lane;
        const bool valid = t < n;
        const uint32_t cnt = min(64u, n - t0);
        uint32_t ko = key_off[min(t, n)];
        uint32_t ent = 0;
        if (valid) {
            const uint64_t l = lsb[t];
            const uint32_t kind = (uint32_t)(l >> 1) & 7, domain = (uint32_t)l & 1;
            const uint32_t gi = txn_index ? txn_index[t] : t;      // global stream position
            ent = (kind << ENT_KIND_SHIFT) | (gi & ENT_TXN_MASK);
            if (gi > ENT_TXN_MASK || (txn_index && t > 0 && txn_index[t - 1] >= gi) || gi < sp.min_gi)
                record_error(st, t, ACCORD_ERR_UNSORTED);
            // a resident store continues its stream: the batch starts after the last TxnId it holds
            if (t == 0 && sp.has_prev && ts_cmp(sp.prev_msb, sp.prev_lsb, sp.prev_node, msb[0], l, node[0]) >= 0)
                record_error(st, t, ACCORD_ERR_UNSORTED);
            if (witness_mask(kind) == 0) record_error(st, t, ACCORD_ERR_KIND);
            if (t > 0 && ts_cmp(msb[t - 1], lsb[t - 1], node[t - 1], msb[t], l, node[t]) >= 0)
                record_error(st, t, ACCORD_ERR_UNSORTED);
            const uint32_t k1 = key_off[t + 1];
            const uint32_t r0 = rng_off ? rng_off[t] : 0, r1 = rng_off ? rng_off[t + 1] : 0;
            if ((domain == 1 && k1 != ko) || (domain == 0 && r1 != r0)) record_error(st, t, ACCORD_ERR_DOMAIN);
            if (rng_start)
                for (uint32_t r = r0; r < r1; ++r)
                    if (rng_start[r] >= rng_end[r] || (r > r0 && rng_end[r - 1] > rng_start[r]))
                        record_error(st, t, ACCORD_ERR_RANGES);
        }
        if (valid) is_range[t] = (uint32_t)(lsb[t] & 1);
        if (rng_owner) {                             // owner txn of every range of the batch
            const uint32_t ro = rng_off[min(t, n)];
            const uint32_t rbase = __shfl(ro, 0, 64), rend = rng_off[t0 + cnt];
            for (uint32_t q0 = rbase; q0 < rend; q0 += 64) {
                const uint32_t q = q0 + lane;
                uint32_t j = 0;
#pragma unroll
                for (uint32_t step = 32; step >= 1; step >>= 1) {
                    const uint32_t c = j + step;
                    const uint32_t rc = __shfl(ro, (int)(c & 63), 64);
                    if (c < cnt && rc <= q) j = c;
                }
                if (q < rend) rng_owner[q] = t0 + j;
            }
        }
        const uint32_t pbase = __shfl(ko, 0, 64);
        const uint32_t pend = key_off[t0 + cnt];
        // the pairs in rounds of VP x 64: every key of a round is loaded before any is used (one
        // memory round trip per round), its predecessor comes from the lane below
        constexpr int VP = 8;
        uint32_t carry = pbase > 0 ? key_ord[pbase - 1] : 0u;   // the key before the round's first pair
        for (uint32_t r0 = pbase; r0 < pend; r0 += VP * 64) {
            uint32_t kv[VP];
#pragma unroll
            for (int v = 0; v < VP; ++v) {
                const uint32_t p = r0 + v * 64 + lane;
                kv[v] = p < pend ? key_ord[p] : 0u;
            }
#pragma unroll
            for (int v = 0; v < VP; ++v) {
                const uint32_t p0 = r0 + v * 64;
                if (p0 >= pend) break;                   // wave-uniform
                const uint32_t p = p0 + lane;
                uint32_t j = 0;                          // largest lane j < cnt with ko_j <= p
#pragma unroll
                for (uint32_t step = 32; step >= 1; step >>= 1) {
                    const uint32_t c = j + step;
                    const uint32_t kc = __shfl(ko, (int)(c & 63), 64);
                    if (c < cnt && kc <= p) j = c;
                }
                const uint32_t e = __shfl(ent, (int)j, 64);
                const uint32_t kj = __shfl(ko, (int)j, 64);
                const uint32_t key = kv[v];
                uint32_t prev = __shfl_up(key, 1, 64);
                if (lane == 0) prev = carry;
                carry = __shfl(key, 63, 64);
                if (p < pend) {
                    const bool in_range = key >= key_lo && key < key_hi;
                    if (!in_range || (p > kj && prev >= key)) record_error(st, t0 + j, ACCORD_ERR_KEYS);
                    pair_key[p] = in_range ? key - key_lo : 0u;      // keep the pipeline in bounds on error
                    pair_ent[p] = e;
                }
            }
        }
    }
}

// Accept batches (Accept.calculatePartialDeps, messages/Accept.java:113-117): the candidates of txn
// t are the registered txns with txnId < executeAt[t] (CommandsForKey.insertPos :1698-1703), i.e.
// the batch prefix [0, bound_l[t]) -- found by a binary search over the sorted batch TxnIds.
// bound_g is that bound in global stream positions (store subsets), pair_bound the same per pair.
__global__ __launch_bounds__(256) void accept_bounds_kernel(
    uint32_t n, const uint64_t *__restrict__ msb, const uint64_t *__restrict__ lsb, const int32_t *__restrict__ node,
    const uint64_t *__restrict__ emsb, const uint64_t *__restrict__ elsb, const int32_t *__restrict__ enode,
    const uint32_t *__restrict__ key_off, const uint32_t *__restrict__ txn_index, uint32_t *__restrict__ bound_l,
    uint32_t *__restrict__ bound_g, uint32_t *__restrict__ pair_bound, DevStatus *st)
{
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        const uint64_t em = emsb[t], el = elsb[t];
        const int32_t en = enode[t];
        if (ts_cmp(em, el, en, msb[t], lsb[t], node[t]) < 0) record_error(st, t, ACCORD_ERR_ARG);
        uint32_t lo = t, hi = n;                     // txnId[t] <= executeAt: the bound is past t
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (ts_cmp(msb[m], lsb[m], node[m], em, el, en) < 0) lo = m + 1; else hi = m;
        }
        const uint32_t g = !txn_index ? lo : (lo < n ? txn_index[lo] : txn_index[n - 1] + 1u);
        bound_l[t] = lo;
        bound_g[t] = g;
        for (uint32_t q = key_off[t]; q < key_off[t + 1]; ++q) pair_bound[q] = g;
    }
}

// ---- history annotation (key-major) ----
constexpr int HS_THREADS = 1024;
constexpr int HS_ITEMS = 4;
constexpr uint32_t HS_TILE = HS_THREADS * HS_ITEMS;
static_assert(HS_TILE == HISTORY_TILE, "history tile");

// Segment bounds per key; tile-local inclusive max-scan of (p+1 if entry p is a Write) -> the last
// Write at or before p, and tile-local inclusive class counts; both completed by tile carries.
// hist (key-major entries) comes out of the radix sort.  Every wave owns a contiguous sixteenth of
// the tile and scans it in 4 coalesced rounds with wave scans and a running carry held in
// registers; one block step adds the preceding waves' totals (16 waves of 4 rows: 50 VGPRs, 8 waves
// per SIMD; 4 waves of 16 rows held 108 VGPRs, measured 6 us slower on config 2, r03_hs).
__global__ __launch_bounds__(HS_THREADS) void history1_kernel(uint32_t P, const uint32_t *__restrict__ sorted_key,
                                                              const uint32_t *__restrict__ hist,
                                                              uint32_t *__restrict__ seg_start,
                                                              uint32_t *__restrict__ seg_end, uint32_t *__restrict__ pw_local,
                                                              uint32_t *__restrict__ tile_max, uint64_t *__restrict__ c_local,
                                                              uint64_t *__restrict__ tile_cnt)
{
    __shared__ uint32_t wmax[HS_THREADS / 64];
    __shared__ uint64_t wcnt[HS_THREADS / 64];
    const uint32_t w = wave_id(), lane = lane_id();
    const uint32_t wb = blockIdx.x * HS_TILE + w * (HS_ITEMS * 64);
    uint32_t e[HS_ITEMS], k[HS_ITEMS];
#pragma unroll
    for (int r = 0; r < HS_ITEMS; ++r) {
        const uint32_t p = wb + r * 64 + lane;
        e[r] = p < P ? hist[p] : 0u;
        k[r] = p < P ? sorted_key[p] : 0xFFFFFFFFu;
    }
    uint32_t run = 0;
    uint64_t crun = 0;
    uint64_t cc[HS_ITEMS];
#pragma unroll
    for (int r = 0; r < HS_ITEMS; ++r) {
        const uint32_t p = wb + r * 64 + lane;
        constexpr uint32_t EDGE = 0xFFFFFFFEu;       // neighbour outside the register rows: load it
        uint32_t kp = __shfl_up(k[r], 1, 64), kn = __shfl_down(k[r], 1, 64);
        const uint32_t kprev_row = __shfl(k[r > 0 ? r - 1 : 0], 63, 64);
        const uint32_t knext_row = __shfl(k[r + 1 < HS_ITEMS ? r + 1 : r], 0, 64);
        if (lane == 0) kp = r > 0 ? kprev_row : EDGE;
        if (lane == 63) kn = r + 1 < HS_ITEMS ? knext_row : EDGE;
        uint32_t v = 0;
        uint64_t c = 0;
        if (p < P) {
            if (kp == EDGE) kp = p > 0 ? sorted_key[p - 1] : 0xFFFFFFFFu;
            if (kn == EDGE) kn = p + 1 < P ? sorted_key[p + 1] : 0xFFFFFFFFu;
            if (kp != k[r]) seg_start[k[r]] = p;
            if (kn != k[r]) seg_end[k[r]] = p + 1;
            v = (e[r] >> ENT_KIND_SHIFT) == 1u ? p + 1 : 0u;
            c = class_bits(e[r] >> ENT_KIND_SHIFT);
        }
        v = max(run, wave_incl_max(v));
        c = crun + wave_incl_scan64(c);
        run = readlane(v, 63);
        crun = (uint64_t)readlane((uint32_t)c, 63) | ((uint64_t)readlane((uint32_t)(c >> 32), 63) << 32);
        e[r] = v;                                    // wave-local running values
        cc[r] = c;
    }
    if (lane == 0) { wmax[w] = run; wcnt[w] = crun; }
    __syncthreads();
    uint32_t ex = 0;
    uint64_t cex = 0;
    for (uint32_t u = 0; u < w; ++u) { ex = max(ex, wmax[u]); cex += wcnt[u]; }
#pragma unroll
    for (int r = 0; r < HS_ITEMS; ++r) {
        const uint32_t p = wb + r * 64 + lane;
        if (p < P) {
            pw_local[p] = max(e[r], ex);
            c_local[p] = cc[r] + cex;
        }
    }
    if (threadIdx.x == 0) {
        uint32_t m = 0;
        uint64_t c = 0;
        for (uint32_t u = 0; u < HS_THREADS / 64; ++u) { m = max(m, wmax[u]); c += wcnt[u]; }
        tile_max[blockIdx.x] = m;
        tile_cnt[blockIdx.x] = c;
    }
}

// exclusive max-scan of the tile maxima and exclusive sum-scan of the tile class counts (one block)
__global__ __launch_bounds__(256) void history_carry_kernel(uint32_t *__restrict__ tile_max,
                                                            const uint64_t *__restrict__ tile_cnt,
                                                            ClassCarry *__restrict__ ccarry, uint32_t tiles)
{
    __shared__ uint32_t wmax[4];
    __shared__ uint32_t wsum[3][4];
    uint32_t carry = 0, cw = 0, cr = 0, ce = 0;
    for (uint32_t base = 0; base < tiles; base += 256) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < tiles ? tile_max[i] : 0u;
        const uint64_t c = i < tiles ? tile_cnt[i] : 0ull;
        const uint32_t vw = (uint32_t)(c & 0xFFFFu), vr = (uint32_t)((c >> 16) & 0xFFFFu), ve = (uint32_t)((c >> 32) & 0xFFFFu);
        const uint32_t incl = wave_incl_max(v);
        const uint32_t iw = wave_incl_scan(vw), ir = wave_incl_scan(vr), ie = wave_incl_scan(ve);
        const uint32_t wv = threadIdx.x >> 6;
        if (lane_id() == 63) { wmax[wv] = incl; wsum[0][wv] = iw; wsum[1][wv] = ir; wsum[2][wv] = ie; }
        __syncthreads();
        uint32_t ex = __shfl_up(incl, 1, 64);
        if (lane_id() == 0) ex = 0;
        uint32_t xw = iw - vw, xr = ir - vr, xe = ie - ve;
        uint32_t blk = 0, bw = 0, br = 0, be = 0;
        for (uint32_t w = 0; w < 4; ++w) {
            if (w < wv) { ex = max(ex, wmax[w]); xw += wsum[0][w]; xr += wsum[1][w]; xe += wsum[2][w]; }
            blk = max(blk, wmax[w]);
            bw += wsum[0][w]; br += wsum[1][w]; be += wsum[2][w];
        }
        if (i < tiles) {
            tile_max[i] = max(carry, ex);
            ccarry[i] = ClassCarry{cw + xw, cr + xr, ce + xe, 0u};
        }
        carry = max(carry, blk);
        cw += bw; cr += br; ce += be;
        __syncthreads();
    }
}

// Per history entry p (txn i on key k): the deps slice [lo, p) of (i, k) under the status-at-time
// model.  lo = the last Write entry j < i-W of the segment (committed[] bound of
// CommandsForKey.mapReduceActive :620-645), else the segment start.  Written txn-major, with the
// number of slice entries kind(i) witnesses (the pair's share of keysToTxnIds).
// Block per tile of H2_TILE positions; the entries of the tile and of H2_HALO positions before it
// are staged in LDS, so the backward search for the window bound runs on LDS (a global search only
// when a segment's window reaches past the halo: keys hotter than H2_HALO entries per W txns).
// Each thread handles H2_ITEMS positions in stages (loads of every item issued before any is
// consumed), so the dependent round trips are paid once per stage, not once per item.
constexpr uint32_t H2_THREADS = 256, H2_TILE = 512, H2_HALO = 2048, H2_ITEMS = H2_TILE / H2_THREADS;

__global__ __launch_bounds__(H2_THREADS) void history2_kernel(uint32_t P, uint32_t window, const uint32_t *__restrict__ sorted_key,
                                                              const uint32_t *__restrict__ sorted_pair,
                                                              const uint32_t *__restrict__ hist,
                                                              const uint32_t *__restrict__ seg_start,
                                                              const uint32_t *__restrict__ pw_local,
                                                              const uint32_t *__restrict__ carry,
                                                              const uint64_t *__restrict__ c_local,
                                                              const ClassCarry *__restrict__ ccarry,
                                                              const uint32_t *__restrict__ seg_end,
                                                              const uint32_t *__restrict__ pair_bound,
                                                              PairSlice *__restrict__ slice, uint32_t ncarry)
{
    __shared__ uint32_t tx[H2_HALO + H2_TILE];
    const uint32_t base = blockIdx.x * H2_TILE;
    const uint32_t lds_lo = base > H2_HALO ? base - H2_HALO : 0u;
    const uint32_t end = min(P, base + H2_TILE);
    uint32_t key[H2_ITEMS], q[H2_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) {
        const uint32_t p = base + j * H2_THREADS + threadIdx.x;
        key[j] = p < end ? sorted_key[p] : 0u;
        // combined history of a resident store: [carried entries | batch pairs]; carried entries
        // (index < ncarry) are history only and get no slice (q = ~0)
        const uint32_t v = p < end ? sorted_pair[p] : 0u;
        q[j] = v >= ncarry ? v - ncarry : 0xFFFFFFFFu;
    }
    for (uint32_t x = lds_lo + threadIdx.x; x < end; x += H2_THREADS) tx[x - lds_lo] = hist[x];
    uint32_t a[H2_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) {
        const uint32_t p = base + j * H2_THREADS + threadIdx.x;
        a[j] = p < end ? seg_start[key[j]] : 0u;
    }
    __syncthreads();
    // window bound: l = first position in [a, p] whose txn >= i - W (only when i > W)
    uint32_t ent[H2_ITEMS], l[H2_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) {
        const uint32_t p = base + j * H2_THREADS + threadIdx.x;
        ent[j] = p < end ? tx[p - lds_lo] : 0u;
        const uint32_t i = ent[j] & ENT_TXN_MASK;
        l[j] = a[j];
        if (p < end && i > window) {
            const uint32_t thr = i - window;
            // exponential search backwards, on LDS down to lb
            const uint32_t lb = max(a[j], lds_lo);
            uint32_t hi = p, lo = lb, step = 1;
            bool found = false;
            while (hi > lb) {
                const uint32_t probe = (hi - lb > step) ? hi - step : lb;
                if ((tx[probe - lds_lo] & ENT_TXN_MASK) < thr) { lo = probe + 1; found = true; break; }
                hi = probe;
                step <<= 1;
            }
            if (found || lb == a[j]) {
                uint32_t h = hi;
                while (lo < h) {
                    const uint32_t m = (lo + h) >> 1;
                    if ((tx[m - lds_lo] & ENT_TXN_MASK) < thr) lo = m + 1; else h = m;
                }
                if (!found) lo = hi;                    // every entry of [lb, p] is inside the window
            } else {                                    // window reaches past the halo: global search
                uint32_t gh = lb, gl = a[j];
                uint32_t st = 1;
                while (gh > a[j]) {
                    const uint32_t probe = (gh - a[j] > st) ? gh - st : a[j];
                    if ((hist[probe] & ENT_TXN_MASK) < thr) { gl = probe + 1; break; }
                    gh = probe;
                    st <<= 1;
                }
                while (gl < gh) {
                    const uint32_t m = (gl + gh) >> 1;
                    if ((hist[m] & ENT_TXN_MASK) < thr) gl = m + 1; else gh = m;
                }
                lo = gl;
            }
            l[j] = lo;
        }
    }
    // lo = the last Write before l (if any, inside the segment), else the segment start
    uint32_t pw[H2_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) {
        pw[j] = 0;
        if (l[j] > a[j]) {
            const uint32_t x = l[j] - 1;
            pw[j] = max(pw_local[x], carry[x / HS_TILE]);   // (last Write <= x) + 1
        }
    }
    // upper bound: the pair's own position (PreAccept), or for an Accept the first entry whose txn
    // is not started before executeAt (pair_bound); the txn itself is then inside and not counted
    uint32_t hi[H2_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) {
        const uint32_t p = base + j * H2_THREADS + threadIdx.x;
        hi[j] = p;
        if (pair_bound && p < end && q[j] != 0xFFFFFFFFu) {
            const uint32_t b = pair_bound[q[j]], c = seg_end[key[j]];
            uint32_t x = p + 1, step = 1;
            while (x < c && (hist[x] & ENT_TXN_MASK) < b) {   // gallop, then bisect
                const uint32_t probe = x + step;
                if (probe >= c || (hist[probe] & ENT_TXN_MASK) >= b) {
                    uint32_t l2 = x + 1, h2 = min(probe, c);
                    while (l2 < h2) {
                        const uint32_t m = (l2 + h2) >> 1;
                        if ((hist[m] & ENT_TXN_MASK) < b) l2 = m + 1; else h2 = m;
                    }
                    x = l2;
                    break;
                }
                x = probe + 1;
                step <<= 1;
            }
            hi[j] = (b > (ent[j] & ENT_TXN_MASK)) ? x : p;
        }
    }
    uint32_t cnt[H2_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) {
        const uint32_t p = base + j * H2_THREADS + threadIdx.x;
        l[j] = pw[j] > a[j] ? pw[j] - 1 : a[j];         // now: lo
        cnt[j] = 0;
        if (p < end && hi[j] > l[j]) {
            const uint32_t kind = ent[j] >> ENT_KIND_SHIFT, wmask = witness_mask(kind);
            cnt[j] = witnessed_upto(c_local, ccarry, hi[j] - 1, wmask) -
                     (l[j] ? witnessed_upto(c_local, ccarry, l[j] - 1, wmask) : 0u);
            if (hi[j] > p) cnt[j] -= (wmask >> kind) & 1u;   // p1: the txn itself
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) {
        const uint32_t p = base + j * H2_THREADS + threadIdx.x;
        if (p < end && q[j] != 0xFFFFFFFFu) slice[q[j]] = PairSlice{l[j], hi[j], cnt[j], key[j]};
    }
}

// The same for windows W <= H2_HALO, with the window bound found by a fixed-step binary search run
// in lockstep over the thread's items (every step issues all items' LDS reads before any is
// consumed).  Each txn holds a key at most once, so the entries of the pair's key with txn >= i - W
// number at most W + 1 and the bound lies in [p - W, p]: the predicate "same key and txn >= i - W"
// is monotone over that range of the key-major history, and the search needs neither the segment
// start nor a global fallback.
template <uint32_t HALO>
__global__ __launch_bounds__(H2_THREADS) void history2_lockstep_kernel(
    uint32_t P, uint32_t window, uint32_t steps, const uint32_t *__restrict__ sorted_key,
    const uint32_t *__restrict__ sorted_pair, const uint32_t *__restrict__ hist, const uint32_t *__restrict__ seg_start,
    const uint32_t *__restrict__ pw_local, const uint32_t *__restrict__ carry, const uint64_t *__restrict__ c_local,
    const ClassCarry *__restrict__ ccarry, const uint32_t *__restrict__ seg_end, const uint32_t *__restrict__ pair_bound,
    PairSlice *__restrict__ slice, uint32_t ncarry)
{
    __shared__ uint32_t tx[HALO + H2_TILE];
    __shared__ uint32_t tk[HALO + H2_TILE];
    const uint32_t base = blockIdx.x * H2_TILE;
    const uint32_t lds_lo = base > HALO ? base - HALO : 0u;
    const uint32_t end = min(P, base + H2_TILE);
    uint32_t key[H2_ITEMS], q[H2_ITEMS], a[H2_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) {
        const uint32_t p = base + j * H2_THREADS + threadIdx.x;
        key[j] = p < end ? sorted_key[p] : 0u;
        const uint32_t v = p < end ? sorted_pair[p] : 0u;
        q[j] = v >= ncarry ? v - ncarry : 0xFFFFFFFFu;       // carried entries get no slice
    }
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) a[j] = seg_start[key[j]];   // issued early, used late
    for (uint32_t x = lds_lo + threadIdx.x; x < end; x += H2_THREADS) {
        tx[x - lds_lo] = hist[x];
        tk[x - lds_lo] = sorted_key[x];
    }
    __syncthreads();
    uint32_t ent[H2_ITEMS], lo[H2_ITEMS], len[H2_ITEMS], thr[H2_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) {
        const uint32_t p = base + j * H2_THREADS + threadIdx.x;
        ent[j] = p < end ? tx[p - lds_lo] : 0u;
        const uint32_t i = ent[j] & ENT_TXN_MASK;
        thr[j] = i > window ? i - window : 0u;
        const uint32_t lb = p > window ? max(p - window, lds_lo) : lds_lo;
        lo[j] = lb;
        len[j] = p < end ? p - lb : 0u;               // search [lb, p): p itself always qualifies
    }
    for (uint32_t st = 0; st < steps; ++st) {
        uint32_t probe[H2_ITEMS];
#pragma unroll
        for (uint32_t j = 0; j < H2_ITEMS; ++j) {
            const uint32_t half = len[j] >> 1;
            const uint32_t m = lo[j] + half;
            probe[j] = len[j] ? (tk[m - lds_lo] == key[j] && (tx[m - lds_lo] & ENT_TXN_MASK) >= thr[j] ? 1u : 0u) : 1u;
        }
#pragma unroll
        for (uint32_t j = 0; j < H2_ITEMS; ++j) {
            const uint32_t half = len[j] >> 1;
            if (!probe[j]) { lo[j] += half + 1; len[j] -= half + 1; }
            else len[j] = half;
        }
    }
    // lo = the window bound l; then the last Write before l inside the segment, else the segment start
    uint32_t pw[H2_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) {
        if (thr[j] == 0) lo[j] = a[j];                // txn <= W: nothing has left the window
        pw[j] = 0;
        if (lo[j] > a[j]) {
            const uint32_t x = lo[j] - 1;
            pw[j] = max(pw_local[x], carry[x / HS_TILE]);   // (last Write <= x) + 1
        }
    }
    uint32_t hi[H2_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) {
        const uint32_t p = base + j * H2_THREADS + threadIdx.x;
        hi[j] = p;
        if (pair_bound && p < end && q[j] != 0xFFFFFFFFu) {
            const uint32_t b = pair_bound[q[j]], c = seg_end[key[j]];
            uint32_t x = p + 1, step = 1;
            while (x < c && (hist[x] & ENT_TXN_MASK) < b) {   // gallop, then bisect
                const uint32_t probe = x + step;
                if (probe >= c || (hist[probe] & ENT_TXN_MASK) >= b) {
                    uint32_t l2 = x + 1, h2 = min(probe, c);
                    while (l2 < h2) {
                        const uint32_t m = (l2 + h2) >> 1;
                        if ((hist[m] & ENT_TXN_MASK) < b) l2 = m + 1; else h2 = m;
                    }
                    x = l2;
                    break;
                }
                x = probe + 1;
                step <<= 1;
            }
            hi[j] = (b > (ent[j] & ENT_TXN_MASK)) ? x : p;
        }
    }
#pragma unroll
    for (uint32_t j = 0; j < H2_ITEMS; ++j) {
        const uint32_t p = base + j * H2_THREADS + threadIdx.x;
        const uint32_t l = pw[j] > a[j] ? pw[j] - 1 : a[j];
        uint32_t cnt = 0;
        if (p < end && hi[j] > l) {
            const uint32_t kind = ent[j] >> ENT_KIND_SHIFT, wmask = witness_mask(kind);
            cnt = witnessed_upto(c_local, ccarry, hi[j] - 1, wmask) - (l ? witnessed_upto(c_local, ccarry, l - 1, wmask) : 0u);
            if (hi[j] > p) cnt -= (wmask >> kind) & 1u;   // p1: the txn itself
        }
        if (p < end && q[j] != 0xFFFFFFFFu) slice[q[j]] = PairSlice{l, hi[j], cnt, key[j]};
    }
}

// Per key txn: KeyDeps sizes from the per-pair witnessed counts.  keys = pairs with >= 1
// witnessed entry, keysToTxnIds = keys + body; txnIds <= body (an upper bound: the fill pass
// writes the exact count and the values are compacted afterwards).
// A wave per 64 consecutive txns: their pairs are one contiguous run, read coalesced (a lane per
// pair, its wcnt word), and summed per txn in LDS.
__global__ __launch_bounds__(256) void keydeps_sizes_kernel(uint32_t n, const uint32_t *__restrict__ key_off,
                                                            const PairSlice *__restrict__ slice,
                                                            uint32_t *__restrict__ cnt_keys,
                                                            uint32_t *__restrict__ cnt_vub,
                                                            uint32_t *__restrict__ cnt_k2v, DevStatus *status)
{
    __shared__ uint32_t s_kc[4][64], s_body[4][64];
    const uint32_t lane = lane_id(), w = wave_id();
    const uint32_t gw = blockIdx.x * 4u + w, nwv = gridDim.x * 4u;
    for (uint32_t t0 = gw * 64u; t0 < n; t0 += nwv * 64u) {
        const uint32_t cnt = min(64u, n - t0);
        const uint32_t ko = key_off[t0 + min(lane, cnt)];        // lanes >= cnt: the end
        s_kc[w][lane] = 0u;
        s_body[w][lane] = 0u;
        const uint32_t pbase = readlane(ko, 0), pend = key_off[t0 + cnt];   // (no lane holds it at cnt = 64)
        wave_lds_sync();
        for (uint32_t p0 = pbase; p0 < pend; p0 += 64u) {
            const uint32_t p = p0 + lane;
            uint32_t j = 0;                          // largest lane j < cnt with ko_j <= p
#pragma unroll
            for (uint32_t step = 32; step >= 1; step >>= 1) {
                const uint32_t c = j + step;
                const uint32_t kc = __shfl(ko, (int)(c & 63), 64);
                if (c < cnt && kc <= p) j = c;
            }
            if (p < pend) {
                const uint32_t c = slice[p].wcnt;
                if (c) {
                    atomicAdd(&s_kc[w][j], 1u);
                    atomicAdd(&s_body[w][j], c);
                }
            }
        }
        wave_lds_sync();
        if (lane < cnt) {
            const uint32_t kc = s_kc[w][lane], body = s_body[w][lane];
            cnt_keys[t0 + lane] = kc;
            cnt_vub[t0 + lane] = body;
            cnt_k2v[t0 + lane] = kc + body;
        }
        wave_lds_sync();
    }
}


template <int WPL>
struct WaveLds {
    unsigned long long bitmap[64 * WPL];
    uint32_t wprefix[64 * WPL];
    uint32_t far[KD_FARCAP];          // value | (owner << 31)
    uint32_t far_rank[KD_FARCAP];     // rank of far[f]'s value among the txn's unique txnIds
    uint32_t far_count;
    uint32_t pad[3];
};

// Candidates per lane per batch: one batch covers 64*KD_CB raw history entries with a single
// round trip to memory (loads are issued before any is consumed).
constexpr int KD_CB = 4;
constexpr uint32_t KD_NONE = 0xFFFFFFFFu;     // candidate not witnessed (also: no candidate)
constexpr uint32_t KD_FAR = 0x80000000u;      // witnessed far candidate: KD_FAR | far-list index

// Global accesses with a 32-bit byte offset from a uniform base, so they compile to the
// saddr + voffset form (no 64-bit address arithmetic per access).  Callers keep every array
// below 4 GiB (checked by the store before launching).
template <typename T> __device__ __forceinline__ T ldg(const T *base, uint32_t idx)
{
    return *(const T *)((const char *)base + (size_t)(uint32_t)(idx * (uint32_t)sizeof(T)));
}
template <typename T> __device__ __forceinline__ void stg(T *base, uint32_t idx, T v)
{
#ifdef ACCORD_NT_STORES
    __builtin_nontemporal_store(v, (T *)((char *)base + (size_t)(uint32_t)(idx * (uint32_t)sizeof(T))));
#else
    *(T *)((char *)base + (size_t)(uint32_t)(idx * (uint32_t)sizeof(T))) = v;
#endif
}

struct TxnMeta {
    uint32_t k0, k1;
    uint64_t lsb;
};

__device__ __forceinline__ TxnMeta load_meta(const KeyDepsParams &p, uint32_t t, uint32_t limit)
{
    TxnMeta m{0u, 0u, 0ull};
    if (t < limit) {
        const uint32_t i = p.fb_list ? p.fb_list[t] : t;
        m.k0 = ldg(p.key_off, i); m.k1 = ldg(p.key_off, i + 1); m.lsb = ldg(p.lsb, i);
    }
    return m;
}

__device__ __forceinline__ void load_slice(const KeyDepsParams &p, const TxnMeta &m, bool valid, uint32_t lane,
                                           uint32_t &lo, uint32_t &pos, uint32_t &wc)
{
    lo = pos = wc = 0;
    if (valid && lane < m.k1 - m.k0 && lane < KD_KCAP) {
        const PairSlice ps = ldg(p.slice, m.k0 + lane);
        lo = ps.lo; pos = ps.pos; wc = ps.wcnt;
    }
}

// Raw candidate r (slot-major concatenation of the k slices) lives at hist[r + delta_s] where s is
// its slot: s = #{q < k : end_q <= r}.  end/delta are per-lane registers of lanes q < k.  The
// slot of the window's first candidate is carried across windows; inside a 64-candidate window
// only the slot boundaries that fall in it are compared (scalar reads of end), then one lane
// permute fetches the slot's delta.
__device__ __forceinline__ void load_batch(const KeyDepsParams &p, uint32_t r0, uint32_t raw_total, uint32_t k,
                                           uint32_t end, int32_t delta, uint32_t (&e)[KD_CB], uint32_t lane)
{
    if (k <= 8) {
        // few slots: the boundaries and deltas sit in SGPRs; a candidate picks its delta by a
        // compare/select chain (lanes >= k hold end = raw_total, never <= a valid candidate)
        uint32_t eq[7];
        int32_t dq[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) dq[q] = (int32_t)readlane((uint32_t)delta, q);
#pragma unroll
        for (int q = 0; q < 7; ++q) eq[q] = readlane(end, q);
#pragma unroll
        for (int c = 0; c < KD_CB; ++c) {
            e[c] = KD_NONE;
            const uint32_t r = r0 + c * 64 + lane;
            int32_t d = dq[0];
#pragma unroll
            for (int q = 0; q < 7; ++q) d = r >= eq[q] ? dq[q + 1] : d;
            if (r < raw_total) e[c] = ldg(p.hist, (uint32_t)((int32_t)r + d));
        }
        return;
    }
    uint32_t q = 0;                                   // uniform: slot of the window's first candidate
#pragma unroll
    for (int c = 0; c < KD_CB; ++c) {
        e[c] = KD_NONE;
        const uint32_t w0 = r0 + c * 64;
        if (w0 >= raw_total) continue;                // wave-uniform: no candidates left
        const uint32_t r = w0 + lane;
        while (q < k && readlane(end, (int)q) <= w0) ++q;
        uint32_t s = q;
        for (uint32_t qq = q; qq < k; ++qq) {
            const uint32_t eq = readlane(end, (int)qq);
            if (eq >= w0 + 64) break;
            s += r >= eq ? 1u : 0u;
        }
        const int32_t d = __shfl(delta, (int)min(s, 63u), 64);
        if (r < raw_total) e[c] = ldg(p.hist, (uint32_t)((int32_t)r + d));
    }
}

// The slots of a txn: lane q < k holds end_q (inclusive scan of the slice lengths) and
// delta_q = slice start - exclusive scan; raw_total = all candidates.
__device__ __forceinline__ void slot_setup(uint32_t lo, uint32_t pos, uint32_t k, uint32_t lane, uint32_t &incl,
                                           int32_t &delta, uint32_t &raw_total)
{
    const uint32_t raw = lane < k ? pos - lo : 0u;
    incl = wave_incl_scan(raw);
    delta = lane < k ? (int32_t)lo - (int32_t)(incl - raw) : 0;
    raw_total = readlane(incl, 63);
}

// One wave builds one txn's KeyDeps.  keys and the keysToTxnIds header come straight from the
// per-pair witnessed counts (PairSlice.wcnt); the body position of a witnessed entry is its
// running ballot count; its value is its rank in the txn's sorted unique txnIds (LDS bitmap over
// [i-SPAN, i) + far list).
// Software pipeline over the wave's txns i, i+S, i+2S, ...: offsets three txns ahead, slices two
// ahead, and the first batch of history candidates one ahead, so the candidate round trip of the
// next txn overlaps this txn's LDS work.
template <int WPL, int MINW = (WPL == 1 ? 8 : 4)>
__global__ __launch_bounds__(KD_THREADS) __attribute__((amdgpu_waves_per_eu(MINW, 8))) void keydeps_kernel(KeyDepsParams p)
{
    if (p.abort && *p.abort) return;           // speculative fill: outputs too small
    __shared__ WaveLds<WPL> lds_all[KD_WAVES];
    const uint32_t w = wave_id(), lane = lane_id();
    WaveLds<WPL> &L = lds_all[w];
    const uint64_t lt = lanemask_lt();
    constexpr uint32_t SPAN = 64u * 64u * WPL;
    const uint32_t S = gridDim.x * KD_WAVES;

    // positions t of the txns to process: every txn, or (fallback after the fast kernel) a list
    const uint32_t limit = p.fb_list ? *p.fb_count : p.n;
    uint32_t t = blockIdx.x * KD_WAVES + w;
    TxnMeta m0 = load_meta(p, t, limit), m1 = load_meta(p, t + S, limit), m2 = load_meta(p, t + 2 * S, limit);
    uint32_t lo0, pos0, wc0, lo1, pos1, wc1;
    load_slice(p, m0, t < limit, lane, lo0, pos0, wc0);
    load_slice(p, m1, t + S < limit, lane, lo1, pos1, wc1);
    uint32_t incl0, raw_total0;
    int32_t delta0;
    uint32_t e0[KD_CB];
    {
        const uint32_t k = m0.k1 - m0.k0;
        slot_setup(lo0, pos0, (t < limit && k <= KD_KCAP) ? k : 0u, lane, incl0, delta0, raw_total0);
        load_batch(p, 0, raw_total0, k, incl0, delta0, e0, lane);
    }

    for (; t < limit; t += S) {
        const uint32_t i = p.fb_list ? p.fb_list[t] : t;
        // ---- prefetch ----
        const TxnMeta m3 = load_meta(p, t + 3 * S, limit);
        uint32_t lo2, pos2, wc2;
        load_slice(p, m2, t + 2 * S < limit, lane, lo2, pos2, wc2);
        uint32_t incl1, raw_total1;
        int32_t delta1;
        uint32_t e1[KD_CB];
        {
            const uint32_t kn = m1.k1 - m1.k0;
            slot_setup(lo1, pos1, (t + S < limit && kn <= KD_KCAP) ? kn : 0u, lane, incl1, delta1, raw_total1);
            load_batch(p, 0, raw_total1, kn, incl1, delta1, e1, lane);
        }

        // ---- this txn ----
        const uint32_t k0 = m0.k0, k = m0.k1 - m0.k0;
        const uint32_t wmask = witness_mask((uint32_t)(m0.lsb >> 1) & 7);
        const uint32_t wc = wc0, incl = incl0, raw_total = raw_total0;
        const int32_t delta = delta0;
        uint32_t e[KD_CB];
#pragma unroll
        for (int c = 0; c < KD_CB; ++c) { e[c] = e0[c]; e0[c] = e1[c]; }
        m0 = m1; m1 = m2; m2 = m3;
        lo0 = lo1; pos0 = pos1; wc0 = wc1; lo1 = lo2; pos1 = pos2; wc1 = wc2;
        incl0 = incl1; delta0 = delta1; raw_total0 = raw_total1;

        if (k > KD_KCAP) {                              // more keys than lanes: the big-txn kernel
            if (lane == 0) p.big_list[atomicAdd(p.big_count, 1u)] = i;
            continue;
        }
        if (k == 0) {                                   // range txn (sized by rangekeys) / no key here
            if (lane == 0) stg(p.cnt_vals, i, ldg(p.cnt_vub, i));
            continue;
        }
        uint32_t my_key = 0;
        if (lane < k) my_key = ldg(p.key_ord, k0 + lane);
        const uint32_t gi = p.txn_index ? ldg(p.txn_index, i) : i;   // global stream position
        const uint32_t key_base = ldg(p.kd_key_off, i), val_base = ldg(p.vub_off, i), k2v_base = ldg(p.kd_k2v_off, i);
        // near bit of txn j: j + nb (< SPAN iff near); candidates precede the bound (Accept: executeAt)
        const uint32_t nb = SPAN - (p.bound_g ? ldg(p.bound_g, i) : gi);

        // ---- keys and keysToTxnIds header from the witnessed counts ----
        const bool ne = lane < k && wc != 0;
        const uint64_t ne_bal = __ballot(ne);
        const uint32_t kc = (uint32_t)__popcll(ne_bal);
        const uint32_t wincl = wave_incl_scan(lane < k ? wc : 0u);
        if (ne) {
            const uint32_t ns = (uint32_t)__popcll(ne_bal & lt);
            stg(p.kd_keys, key_base + ns, my_key);
            stg(p.kd_k2v, k2v_base + ns, (int32_t)(kc + wincl));
        }

#pragma unroll
        for (int q = 0; q < WPL; ++q) L.bitmap[lane * WPL + q] = 0ull;
        if (lane == 0) L.far_count = 0;
        wave_lds_sync();

        // ---- phase 1: witness filter -> near bitmap / far list; e[] becomes j / KD_FAR|f / KD_NONE ----
        const bool one_batch = raw_total <= 64u * KD_CB;
        for (uint32_t r0 = 0; r0 < raw_total; r0 += 64u * KD_CB) {
            if (r0) load_batch(p, r0, raw_total, k, incl, delta, e, lane);
#pragma unroll
            for (int c = 0; c < KD_CB; ++c) {
                if (r0 + c * 64 >= raw_total) break;    // wave-uniform early exit
                const uint32_t ev = e[c];
                uint32_t out = KD_NONE;
                if (((wmask >> (ev >> ENT_KIND_SHIFT)) & 1u) && (ev & ENT_TXN_MASK) != gi) {   // p1
                    const uint32_t j = ev & ENT_TXN_MASK;
                    const uint32_t b = j + nb;
                    if (b < SPAN) {
                        atomicOr(&L.bitmap[b >> 6], 1ull << (b & 63));
                        out = j;
                    } else {
                        const uint32_t f = atomicAdd(&L.far_count, 1u);
                        if (f < KD_FARCAP) L.far[f] = j;
                        out = KD_FAR | f;
                    }
                }
                e[c] = out;
            }
        }
        wave_lds_sync();
        const uint32_t F = L.far_count;
        if (F > KD_FARCAP) {                            // more far deps than the list holds: big-txn kernel
            if (lane == 0) p.big_list[atomicAdd(p.big_count, 1u)] = i;
            continue;
        }

        // ---- union: near popcounts, far owners and ranks ----
        uint32_t pc[WPL];
        uint32_t mysum = 0;
#pragma unroll
        for (int q = 0; q < WPL; ++q) { pc[q] = (uint32_t)__popcll(L.bitmap[lane * WPL + q]); mysum += pc[q]; }
        const uint32_t incl2 = wave_incl_scan(mysum);
        const uint32_t near_u = readlane(incl2, 63);
        uint32_t far_u = 0;
        if (F) {                                        // wave-uniform
            constexpr uint32_t OWN = 0x80000000u;       // first occurrence of its value
            for (uint32_t f = lane; f < F; f += 64) {
                const uint32_t x = L.far[f] & ENT_TXN_MASK;
                bool owner = true;
                for (uint32_t g = 0; g < f; ++g)
                    if ((L.far[g] & ENT_TXN_MASK) == x) { owner = false; break; }
                far_u += owner ? 1u : 0u;
                if (owner) L.far[f] = x | OWN;
            }
            wave_lds_sync();
            for (uint32_t f = lane; f < F; f += 64) {   // far values all precede the near ones
                const uint32_t x = L.far[f] & ENT_TXN_MASK;
                uint32_t rk = 0;
                for (uint32_t g = 0; g < F; ++g) {
                    const uint32_t y = L.far[g];
                    rk += ((y & OWN) && (y & ENT_TXN_MASK) < x) ? 1u : 0u;
                }
                L.far_rank[f] = rk;
            }
            far_u = wave_sum(far_u);
        }
        if (lane == 0) stg(p.cnt_vals, i, far_u + near_u);

        // ---- fill: per witnessed entry its rank -> keysToTxnIds body and txnIds ----
        {
            uint32_t ex = incl2 - mysum + far_u;
#pragma unroll
            for (int q = 0; q < WPL; ++q) { L.wprefix[lane * WPL + q] = ex; ex += pc[q]; }
        }
        wave_lds_sync();
        uint32_t running = 0;
        for (uint32_t r0 = 0; r0 < raw_total; r0 += 64u * KD_CB) {
            if (!one_batch) {                           // rare: re-load and re-filter this batch
                load_batch(p, r0, raw_total, k, incl, delta, e, lane);
#pragma unroll
                for (int c = 0; c < KD_CB; ++c) {
                    const uint32_t ev = e[c];
                    uint32_t out = KD_NONE;
                    if (((wmask >> (ev >> ENT_KIND_SHIFT)) & 1u) && (ev & ENT_TXN_MASK) != gi) {
                        const uint32_t j = ev & ENT_TXN_MASK;
                        if (j + nb < SPAN) {
                            out = j;
                        } else {
                            for (uint32_t g = 0; g < F; ++g)
                                if ((L.far[g] & ENT_TXN_MASK) == j) { out = KD_FAR | g; break; }
                        }
                    }
                    e[c] = out;
                }
            }
#pragma unroll
            for (int c = 0; c < KD_CB; ++c) {
                if (r0 + c * 64 >= raw_total) break;    // wave-uniform early exit
                const uint32_t ev = e[c];
                const bool wit = ev != KD_NONE;
                uint32_t rank = 0, j = ev;
                if (wit) {
                    if (ev & KD_FAR) {
                        const uint32_t f = ev & ~KD_FAR;
                        rank = L.far_rank[f];
                        j = L.far[f] & ENT_TXN_MASK;
                    } else {
                        const uint32_t b = ev + nb;
                        rank = L.wprefix[b >> 6] + (uint32_t)__popcll(L.bitmap[b >> 6] & ((1ull << (b & 63)) - 1ull));
                    }
                }
                const uint64_t bal = __ballot(wit);
                const uint32_t pos = running + (uint32_t)__popcll(bal & lt);
                if (wit) {
                    stg(p.kd_k2v, k2v_base + kc + pos, (int32_t)rank);
                    stg(p.vgap, val_base + rank, j);    // every holder of j writes the same word
                }
                running += (uint32_t)__popcll(bal);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Fast fill: the common txn of a key batch -- k <= 8 keys, <= 256 raw candidates, <= 64 deps older
// than the near span -- with nothing else on its path: a 32-byte per-txn record (one load), the pair
// slices, one batch of candidates located by a compare/select chain, LDS bitmap union, ranks.
// Anything else (more keys or candidates, more far deps) is appended to a list the
// general keydeps_kernel processes afterwards; its outputs are identical, so a txn abandoned
// half-way (after its keys were written) is simply redone.
// ---------------------------------------------------------------------------------------------
struct alignas(32) TxnRec {
    uint32_t k0, k, kind, gi, key_base, val_base, k2v_base, bound;
};

__global__ __launch_bounds__(256) void txnrec_kernel(KeyDepsParams p, TxnRec *__restrict__ out)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.n; i += gridDim.x * blockDim.x) {
        TxnRec r;
        r.k0 = p.key_off[i];
        r.k = p.key_off[i + 1] - r.k0;
        r.kind = (uint32_t)(p.lsb[i] >> 1) & 7;
        r.gi = p.txn_index ? p.txn_index[i] : i;
        r.key_base = p.kd_key_off[i];
        r.val_base = p.vub_off[i];
        r.k2v_base = p.kd_k2v_off[i];
        r.bound = p.bound_g ? p.bound_g[i] : r.gi;   // candidates precede it (Accept: executeAt)
        out[i] = r;
    }
}

// tiny txns (keydeps_tiny_kernel below): k <= TN_K keys and <= TN_RAW raw candidates
constexpr uint32_t TN_K = 4, TN_RAW = 16;
constexpr uint32_t TN_END = 0xFFFFFFFFu;

__device__ __forceinline__ bool tn_take(uint32_t k, uint32_t raw) { return k > 0 && k <= TN_K && raw <= TN_RAW; }

constexpr int FK_CB = 6;                      // candidate batches of 64 a fast-path txn may use
constexpr uint32_t FK_RAW = 64u * FK_CB;      // raw candidates the fast path takes

// inclusive scan over lanes 0..7 (row 0 of the wave; lanes >= 8 get partial sums)
__device__ __forceinline__ uint32_t scan8(uint32_t v)
{
    v += dpp_row_shr<1>(v);
    v += dpp_row_shr<2>(v);
    v += dpp_row_shr<4>(v);
    return v;
}

struct FkTxn {
    uint32_t rec;                     // lane f < 8: TxnRec field f
    uint32_t lo, pos, wc, key;        // lane q < k: its pair slice and key ordinal
};

__device__ __forceinline__ uint32_t fk_rec(const TxnRec *__restrict__ recs, uint32_t t, uint32_t n, uint32_t lane)
{
    return (t < n && lane < 8) ? ldg((const uint32_t *)recs, t * 8u + lane) : 0u;
}

__device__ __forceinline__ void fk_slices(const KeyDepsParams &p, FkTxn &x, uint32_t lane)
{
    const uint32_t k0 = readlane(x.rec, 0), k = readlane(x.rec, 1);
    x.lo = x.pos = x.wc = x.key = 0;
    if (k <= 8 && lane < k) {
        const PairSlice ps = ldg(p.slice, k0 + lane);
        x.lo = ps.lo; x.pos = ps.pos; x.wc = ps.wcnt;
        // the key from key_ord (an own load): measured 0.05 ms faster than taking ps.key with the slice
        x.key = ldg(p.key_ord, k0 + lane);
    }
}

// The raw candidates of a txn with k <= 8 and <= FK_RAW of them (else e[] stays empty): candidate r
// lies in slot q = #{q' >= 1 : excl_q' <= r} (empty slots fall out: their boundary equals the next
// slot's), and sits at hist[r + lo_q - excl_q]; the slot's delta comes from lane q by bpermute.
__device__ __forceinline__ uint32_t fk_cands(const KeyDepsParams &p, const FkTxn &x, uint32_t lane,
                                             uint32_t (&e)[FK_CB])
{
    const uint32_t k = readlane(x.rec, 1);
    const uint32_t raw = (k <= 8 && lane < k) ? x.pos - x.lo : 0u;
    const uint32_t incl = scan8(raw);
    const uint32_t excl = incl - raw;
    const int32_t delta = (int32_t)x.lo - (int32_t)excl;
    const uint32_t rt = readlane(incl, 7);
    uint32_t eq[7];
#pragma unroll
    for (int q = 0; q < 7; ++q) eq[q] = readlane(excl, q + 1);
    const bool take = k <= 8 && rt <= FK_RAW && !(p.tiny && tn_take(k, rt));   // tiny txns: not this kernel's
#pragma unroll
    for (int c = 0; c < FK_CB; ++c) e[c] = KD_NONE;
#pragma unroll
    for (int c = 0; c < FK_CB; ++c) {
        if (!take || (uint32_t)c * 64u >= rt) break;   // wave-uniform
        const uint32_t r = c * 64 + lane;
        uint32_t slot = 0;
#pragma unroll
        for (int q = 0; q < 7; ++q) slot += r >= eq[q] ? 1u : 0u;
        const int32_t d = __builtin_amdgcn_ds_bpermute((int)(slot << 2), delta);
        if (r < rt) e[c] = ldg(p.hist, (uint32_t)((int32_t)r + d));
    }
    return rt;
}

// Near map: one byte per txn of the near span [bound - SPAN, bound), set by plain byte stores
// (measured, scripts/micro/lds_patterns.hip: lanes storing to one word cost nothing extra, while
// same-word LDS atomics serialize -- 8 lanes on a word = 8x), then packed into bits: lane L owns
// the BPL bytes [L*BPL, (L+1)*BPL) of the map, packs them into its bit word and zeroes them for the
// next txn.  A candidate's rank comes from its word owner by one lane permute (no LDS traffic).
// 4 map bytes (0 / 1 each) -> 4 bits, byte b at bit b: the bytes land on bits 24..27 of the product
// (M = 2^24 + 2^17 + 2^10 + 2^3; the cross terms stay below bit 20 or above bit 31)
__device__ __forceinline__ uint32_t pack4(uint32_t x) { return ((x & 0x01010101u) * 0x01020408u) >> 24; }

template <int BPL>
__device__ __forceinline__ uint32_t near_take(uint8_t *map, uint32_t lane)
{
    uint32_t bits = 0;
#pragma unroll
    for (int h = 0; h < BPL / 16; ++h) {
        uint4 *q = (uint4 *)(map + lane * BPL + h * 16);
        const uint4 v = *q;
        *q = make_uint4(0u, 0u, 0u, 0u);               // cleared for the next txn (in-order LDS)
        bits |= (pack4(v.x) | pack4(v.y) << 4 | pack4(v.z) << 8 | pack4(v.w) << 12) << (16 * h);
    }
    return bits;
}

// Diagnostic build only (-DACCORD_FK_STAMPS, scripts/fk_stamps.py): s_memtime stamps at the
// segment boundaries of the fast kernel's txn loop, summed per segment over every wave.  Read the
// SHARES, not the run time: each stamp drains the wave's LDS traffic.
#ifdef ACCORD_FK_STAMPS
__device__ unsigned long long g_fk_stamps[16];
#define FK_STAMP(seg)                                                                          \
    do {                                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        unsigned long long t_;                                                                 \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        fk_sum[seg] += t_ - fk_last;                                                           \
        fk_last = t_;                                                                          \
    } while (0)
#else
#define FK_STAMP(seg) do {} while (0)
#endif

// COPY (diagnostic, ACCORD_FILL_COPY=1, outputs meaningless): the same record / slice / candidate
// loads and the same output stores -- keys, keysToTxnIds header and body at their positions, one
// txnId store per witnessed candidate inside the txn's region -- without the union (near map, far
// list, ranks): the address-path floor of this kernel.
template <int BPL, bool COPY = false>
__global__ __launch_bounds__(KD_THREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) void keydeps_fast_kernel(
    KeyDepsParams p, const TxnRec *__restrict__ recs)
{
    if (p.abort && *p.abort) return;           // speculative fill: outputs too small
    constexpr uint32_t SPAN = 64u * BPL;
    __shared__ __attribute__((aligned(16))) uint8_t map_all[KD_WAVES][SPAN];   // near map (bytes)
    __shared__ uint32_t fr_all[KD_WAVES][64];       // far deps: value, then its rank
    const uint32_t w = wave_id(), lane = lane_id();
    uint8_t *map = map_all[w];
    uint32_t *fr = fr_all[w];
    const uint64_t lt = lanemask_lt();
#pragma unroll
    for (int h = 0; h < BPL / 16; ++h) *(uint4 *)(map + lane * BPL + h * 16) = make_uint4(0u, 0u, 0u, 0u);
    // XCD-aware order: blocks b and b + 8 share an XCD (round-robin placement, MI355X_MICROARCH.md),
    // so the 8 block classes take contiguous eighths of the batch and each XCD's waves sweep theirs
    // in step: consecutive txns read the same hot keys' history slices, which then stay in that
    // XCD's L2 instead of being fetched into all eight
    const uint32_t xg = blockIdx.x & 7u, B = gridDim.x >> 3;
    const uint32_t n = (uint32_t)(((uint64_t)p.n * (xg + 1)) >> 3), S = B * KD_WAVES;
    uint32_t t = (uint32_t)(((uint64_t)p.n * xg) >> 3) + (blockIdx.x >> 3) * KD_WAVES + w;

    // software pipeline: records three txns ahead, slices two ahead, candidates one ahead
    FkTxn a, b, c;
    a.rec = fk_rec(recs, t, n, lane);
    b.rec = fk_rec(recs, t + S, n, lane);
    c.rec = fk_rec(recs, t + 2 * S, n, lane);
    fk_slices(p, a, lane);
    fk_slices(p, b, lane);
    uint32_t ea[FK_CB];
    uint32_t rta = fk_cands(p, a, lane, ea);

#ifdef ACCORD_FK_STAMPS
    unsigned long long fk_sum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, fk_last = 0, fk_n = 0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(fk_last)::"memory");
#endif
    for (; t < n; t += S) {
        FkTxn d;
        d.rec = fk_rec(recs, t + 3 * S, n, lane);
        fk_slices(p, c, lane);
        uint32_t eb[FK_CB];
        const uint32_t rtb = fk_cands(p, b, lane, eb);
        FK_STAMP(0);                                  // prefetch issue (waits for c's record, b's slices)
#ifdef ACCORD_FK_STAMPS
        ++fk_n;
#endif

        do {   // ---- txn t (break = done with it) ----
            const uint32_t k = readlane(a.rec, 1);
            if (k == 0) {                             // range txn / no key in this store
                if (lane == 0) stg(p.cnt_vals, t, 0u);
                break;
            }
            if (p.tiny && tn_take(k, rta)) break;     // a tiny txn: keydeps_tiny_kernel builds it
            if (COPY) {
                if (k > 8 || rta > FK_RAW) break;
                const uint32_t kind = readlane(a.rec, 2), gi = readlane(a.rec, 3), wmask = witness_mask(kind);
                const uint32_t key_base = readlane(a.rec, 4), val_base = readlane(a.rec, 5), k2v_base = readlane(a.rec, 6);
                const bool ne = lane < k && a.wc != 0;
                const uint64_t hb = __ballot(ne);
                const uint32_t kc = (uint32_t)__popcll(hb);
                const uint32_t wincl = scan8(lane < k ? a.wc : 0u);
                if (ne) {
                    const uint32_t ns = (uint32_t)__popcll(hb & lt);
                    stg(p.kd_keys, key_base + ns, a.key);
                    stg(p.kd_k2v, k2v_base + ns, (int32_t)(kc + wincl));
                }
                uint32_t run = 0;
#pragma unroll
                for (int cc = 0; cc < FK_CB; ++cc) {
                    if ((uint32_t)cc * 64 >= rta) break;
                    const uint32_t ev = ea[cc], j = ev & ENT_TXN_MASK;
                    const bool wit = (uint32_t)cc * 64 + lane < rta && ((wmask >> (ev >> ENT_KIND_SHIFT)) & 1u) && j != gi;
                    const uint64_t wb = __ballot(wit);
                    if (wit) {
                        stg(p.kd_k2v, k2v_base + kc + run + (uint32_t)__popcll(wb & lt), (int32_t)j);
                        stg(p.vgap, val_base + (j & 63u), j);
                    }
                    run += (uint32_t)__popcll(wb);
                }
                if (lane == 0) stg(p.cnt_vals, t, run);
                break;
            }
            bool fallback = k > 8 || rta > FK_RAW;
            const uint32_t kind = readlane(a.rec, 2), gi = readlane(a.rec, 3);
            const uint32_t wmask = witness_mask(kind);
            const uint32_t nb = SPAN - readlane(a.rec, 7);   // map byte of txn j: j + nb (< SPAN iff near)
            uint32_t F = 0;                           // far deps (older than the near span)
            if (!fallback) {
                // each candidate's verdict replaces it in ea[]: KD_NONE (not witnessed), its near map
                // byte (< SPAN), or KD_FAR | its far-list index -- phase 2 reads it back
#pragma unroll
                for (int cc = 0; cc < FK_CB; ++cc) {
                    if ((uint32_t)cc * 64 >= rta) break;   // wave-uniform
                    const uint32_t ev = ea[cc];
                    const uint32_t j = ev & ENT_TXN_MASK;
                    const bool wit = ((wmask >> (ev >> ENT_KIND_SHIFT)) & 1u) && j != gi;   // p1
                    const uint32_t off = j + nb;
                    const bool nr = wit && off < SPAN;
                    if (nr) map[off] = 1;
                    uint32_t pv = nr ? off : KD_NONE;
                    const uint64_t fb = __ballot(wit && !nr);
                    if (fb) {                             // wave-uniform
                        const uint32_t f = F + (uint32_t)__popcll(fb & lt);
                        if (wit && !nr) {
                            if (f < 64) fr[f] = j;
                            pv = KD_FAR | f;
                        }
                        F += (uint32_t)__popcll(fb);
                    }
                    ea[cc] = pv;
                }
                fallback = F > 64;
            }
            if (fallback) {
                if (lane == 0) p.fb_list[atomicAdd(p.fb_count, 1u)] = t;
                if (rta <= FK_RAW && k <= 8) {        // its bytes went into the map: clear them
                    wave_lds_sync();
                    (void)near_take<BPL>(map, lane);
                }
                break;
            }
            wave_lds_sync();
            FK_STAMP(1);                              // phase 1 (waits for this txn's candidates)
            // far deps: de-duplicated ranks (all of them precede the near span in TxnId order)
            uint32_t far_u = 0;
            if (F) {                                      // wave-uniform
                // the first holder of every value owns it; rank = distinct values below it
                const uint32_t x = lane < F ? fr[lane] : 0xFFFFFFFFu;
                uint64_t om = 0;
                uint32_t rk = 0;
                for (uint32_t g = 0; g < F; ++g) {
                    const uint32_t xg = readlane(x, (int)g);
                    const uint64_t m = __ballot(x == xg);
                    if ((uint32_t)__builtin_ctzll(m) == g) {   // g is xg's first holder (uniform)
                        om |= 1ull << g;
                        rk += xg < x ? 1u : 0u;
                    }
                }
                far_u = (uint32_t)__popcll(om);
                wave_lds_sync();
                if (lane < F) fr[lane] = rk;
                if ((om >> lane) & 1ull) stg(p.vgap, readlane(a.rec, 5) + rk, x);
            }
            FK_STAMP(2);                              // far deps
            // union: the lane's map bytes -> bit word, popcount prefix (after the far deps); |txnIds|
            const uint32_t bits = near_take<BPL>(map, lane);
            const uint32_t pc = (uint32_t)__popc(bits);
            const uint32_t incl = wave_incl_scan(pc);
            const uint32_t pre = incl - pc + far_u;
            if (lane == 0) stg(p.cnt_vals, t, readlane(incl, 63) + far_u);
            FK_STAMP(3);                              // union
            // keys and keysToTxnIds header from the witnessed counts
            const uint32_t key_base = readlane(a.rec, 4), val_base = readlane(a.rec, 5), k2v_base = readlane(a.rec, 6);
            const bool ne = lane < k && a.wc != 0;
            const uint64_t hb = __ballot(ne);
            const uint32_t kc = (uint32_t)__popcll(hb);
            const uint32_t wincl = scan8(lane < k ? a.wc : 0u);
            if (ne) {
                const uint32_t ns = (uint32_t)__popcll(hb & lt);
                stg(p.kd_keys, key_base + ns, a.key);
                stg(p.kd_k2v, k2v_base + ns, (int32_t)(kc + wincl));
            }
            if (F) wave_lds_sync();                      // far ranks in fr[]
            FK_STAMP(4);                              // keys + header
            // body: rank of every witnessed entry; txnIds at their ranks
            uint32_t run = 0;
#pragma unroll
            for (int cc = 0; cc < FK_CB; ++cc) {
                if ((uint32_t)cc * 64 >= rta) break;
                const uint32_t pv = ea[cc];                            // phase 1's verdict
                const bool wit = pv != KD_NONE;
                const bool nr = pv < SPAN;
                const uint32_t off = pv, j = pv - nb;                  // (near only)
                const uint32_t src = (nr ? off : 0u) / BPL;            // the word owner of the byte
                const uint32_t ob = (nr ? off : 0u) % BPL;
                uint32_t rank;
                if (BPL == 16) {                           // 16 bits + a prefix below 2^16: one permute
                    const uint32_t v = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)(pre << 16 | bits));
                    rank = (v >> 16) + (uint32_t)__popc(v & ((1u << ob) - 1u));
                } else {
                    const uint32_t wbits = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)bits);
                    const uint32_t wpre = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)pre);
                    rank = wpre + (uint32_t)__popc(wbits & ((1u << ob) - 1u));
                }
                if (F && wit && !nr) rank = fr[pv & ~KD_FAR];
                const uint64_t wb = __ballot(wit);
                if (wit) {
                    stg(p.kd_k2v, k2v_base + kc + run + (uint32_t)__popcll(wb & lt), (int32_t)rank);
                    if (nr) stg(p.vgap, val_base + rank, j);           // every holder of j writes the same word
                }
                run += (uint32_t)__popcll(wb);
            }
            FK_STAMP(5);                              // phase 2 (body + txnIds stores)
        } while (0);

        // rotate the pipeline (after the txn: a register copy waits for the loads it copies)
        a = b; b = c; c = d;
        rta = rtb;
#pragma unroll
        for (int cc = 0; cc < FK_CB; ++cc) ea[cc] = eb[cc];
        FK_STAMP(6);                                  // rotation (+ skipped / fallback txns)
    }
#ifdef ACCORD_FK_STAMPS
    if (lane == 0) {
        for (int q = 0; q < 7; ++q) atomicAdd(&g_fk_stamps[q], fk_sum[q]);
        atomicAdd(&g_fk_stamps[7], fk_n);
        atomicAdd(&g_fk_stamps[8], 1ull);
    }
#endif
}


// ---------------------------------------------------------------------------------------------
// Big txns: more keys than a wave has lanes (k > KD_KCAP) or more distinct deps older than the
// near span than the general kernel's far list holds (> KD_FARCAP) -- no size limit besides the
// output arrays.  One workgroup per listed txn (the general kernel lists them):
//   keys / keysToTxnIds header : block scans over the pairs in chunks of 256 (same values as the
//                                other kernels: keys with >= 1 witnessed entry, end offsets)
//   union                      : windows of BK_SPAN txns, from the smallest witnessed dep up; per
//                                window an LDS bitmap (OR of the window's witnessed entries), word
//                                popcount prefixes, then every witnessed entry of the window writes
//                                its rank at its body position and the bitmap expands into txnIds
// A wave walks one pair's slice at a time (64 entries per step, ballot-counted body positions from
// the pair's witnessed prefix), so long slices and many keys both spread over the block.
// ---------------------------------------------------------------------------------------------
constexpr int BK_THREADS = 256;
constexpr uint32_t BK_WORDS = 8192;                 // 64 KiB of bitmap
constexpr uint32_t BK_SPAN = BK_WORDS * 64;         // txns per window
constexpr uint32_t BK_WPT = BK_WORDS / BK_THREADS;  // bitmap words per thread

// exclusive block scan of v (all threads of the block call it); total of the block in `tot`
__device__ __forceinline__ uint32_t bk_excl_scan(uint32_t v, uint32_t &tot, uint32_t *sh)
{
    const uint32_t incl = wave_incl_scan(v), w = wave_id();
    if (lane_id() == 63) sh[w] = incl;
    __syncthreads();
    uint32_t off = 0, t = 0;
#pragma unroll
    for (uint32_t q = 0; q < BK_THREADS / 64; ++q) { off += q < w ? sh[q] : 0u; t += sh[q]; }
    __syncthreads();
    tot = t;
    return off + incl - v;
}

__device__ __forceinline__ uint32_t bk_min(uint32_t v, uint32_t *sh)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, d, 64));
    if (lane_id() == 0) sh[wave_id()] = v;
    __syncthreads();
    uint32_t m = sh[0];
#pragma unroll
    for (uint32_t q = 1; q < BK_THREADS / 64; ++q) m = min(m, sh[q]);
    __syncthreads();
    return m;
}

__global__ __launch_bounds__(BK_THREADS) void keydeps_big_kernel(KeyDepsParams p)
{
    if (p.abort && *p.abort) return;           // speculative fill: outputs too small
    __shared__ unsigned long long bm[BK_WORDS];
    __shared__ uint32_t pre[BK_WORDS];
    __shared__ uint32_t sh[BK_THREADS / 64];
    const uint32_t tid = threadIdx.x, w = wave_id(), lane = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint32_t count = *p.big_count;
    for (uint32_t b = blockIdx.x; b < count; b += gridDim.x) {
        const uint32_t i = p.big_list[b];
        const uint32_t k0 = p.key_off[i], k = p.key_off[i + 1] - k0;
        const uint32_t kind = (uint32_t)(p.lsb[i] >> 1) & 7, wmask = witness_mask(kind);
        const uint32_t gi = p.txn_index ? p.txn_index[i] : i;
        const uint32_t key_base = p.kd_key_off[i], val_base = p.vub_off[i], k2v_base = p.kd_k2v_off[i];
        // ---- keys, header, each pair's witnessed prefix ----
        uint32_t kc = 0;
        for (uint32_t c = 0; c < k; c += BK_THREADS) {
            const uint32_t q = c + tid;
            uint32_t t;
            (void)bk_excl_scan(q < k && p.slice[k0 + q].wcnt ? 1u : 0u, t, sh);
            kc += t;
        }
        uint32_t run_kc = 0, run_wc = 0;
        for (uint32_t c = 0; c < k; c += BK_THREADS) {
            const uint32_t q = c + tid;
            const uint32_t wc = q < k ? p.slice[k0 + q].wcnt : 0u;
            uint32_t tk, tw;
            const uint32_t xk = bk_excl_scan(wc ? 1u : 0u, tk, sh) + run_kc;
            const uint32_t xw = bk_excl_scan(wc, tw, sh) + run_wc;
            if (q < k) {
                p.big_wex[k0 + q] = xw;
                if (wc) {
                    p.kd_keys[key_base + xk] = p.key_ord[k0 + q];
                    p.kd_k2v[k2v_base + xk] = (int32_t)(kc + xw + wc);
                }
            }
            run_kc += tk;
            run_wc += tw;
        }
        __syncthreads();
        // ---- the smallest witnessed dep ----
        uint32_t mn = 0xFFFFFFFFu;
        for (uint32_t q = w; q < k; q += BK_THREADS / 64) {
            const PairSlice ps = p.slice[k0 + q];
            for (uint32_t x = ps.lo + lane; x < ps.pos; x += 64) {
                const uint32_t ev = p.hist[x], j = ev & ENT_TXN_MASK;
                if (((wmask >> (ev >> ENT_KIND_SHIFT)) & 1u) && j != gi) mn = min(mn, j);
            }
        }
        uint32_t wlo = bk_min(mn, sh);
        uint32_t base = 0;                                  // distinct deps below the window
        while (wlo != 0xFFFFFFFFu) {
            // window [wlo, wlo + BK_SPAN)
            for (uint32_t x = tid; x < BK_WORDS; x += BK_THREADS) bm[x] = 0ull;
            __syncthreads();
            uint32_t nx = 0xFFFFFFFFu;                      // smallest witnessed dep past the window
            for (uint32_t q = w; q < k; q += BK_THREADS / 64) {
                const PairSlice ps = p.slice[k0 + q];
                for (uint32_t x = ps.lo + lane; x < ps.pos; x += 64) {
                    const uint32_t ev = p.hist[x], j = ev & ENT_TXN_MASK;
                    if (!(((wmask >> (ev >> ENT_KIND_SHIFT)) & 1u) && j != gi)) continue;
                    if (j >= wlo && j - wlo < BK_SPAN) atomicOr(&bm[(j - wlo) >> 6], 1ull << ((j - wlo) & 63));
                    else if (j >= wlo) nx = min(nx, j);     // past the window (earlier ones are done)
                }
            }
            __syncthreads();
            uint32_t pc[BK_WPT], mine = 0;
#pragma unroll
            for (uint32_t y = 0; y < BK_WPT; ++y) { pc[y] = (uint32_t)__popcll(bm[tid * BK_WPT + y]); mine += pc[y]; }
            uint32_t wtot;
            uint32_t ex = bk_excl_scan(mine, wtot, sh) + base;
#pragma unroll
            for (uint32_t y = 0; y < BK_WPT; ++y) {
                const uint32_t x = tid * BK_WPT + y;
                pre[x] = ex;
                unsigned long long bits = bm[x];
                uint32_t o = ex;
                while (bits) {                              // the window's txnIds, ascending
                    const uint32_t bit = (uint32_t)__builtin_ctzll(bits);
                    bits &= bits - 1ull;
                    stg(p.vgap, val_base + o++, wlo + x * 64 + bit);
                }
                ex += pc[y];
            }
            __syncthreads();
            // ranks of the window's witnessed entries at their body positions
            for (uint32_t q = w; q < k; q += BK_THREADS / 64) {
                const PairSlice ps = p.slice[k0 + q];
                uint32_t run = p.big_wex[k0 + q];
                for (uint32_t x0 = ps.lo; x0 < ps.pos; x0 += 64) {
                    const uint32_t x = x0 + lane;
                    uint32_t ev = 0, j = 0;
                    bool wit = false;
                    if (x < ps.pos) {
                        ev = p.hist[x];
                        j = ev & ENT_TXN_MASK;
                        wit = ((wmask >> (ev >> ENT_KIND_SHIFT)) & 1u) && j != gi;
                    }
                    const uint64_t bal = __ballot(wit);
                    if (wit && j >= wlo && j - wlo < BK_SPAN) {
                        const uint32_t d = j - wlo;
                        const uint32_t rank = pre[d >> 6] + (uint32_t)__popcll(bm[d >> 6] & ((1ull << (d & 63)) - 1ull));
                        stg(p.kd_k2v, k2v_base + kc + run + (uint32_t)__popcll(bal & lt), (int32_t)rank);
                    }
                    run += (uint32_t)__popcll(bal);
                }
            }
            base += wtot;
            wlo = bk_min(nx, sh);
            __syncthreads();
        }
        if (tid == 0) p.cnt_vals[i] = base;
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// Tiny txns: k <= TN_K keys and <= TN_RAW raw candidates -- most txns of a store that owns a slice
// of the keyspace (a rank of the multi-GPU bench sees ~1.5 keys per txn).  One THREAD per txn
// instead of a wave: its <= TN_RAW candidates (slot-major, as the fast kernel orders them) are
// loaded at once into registers, the union is ranked by pairwise compares (a value's rank =
// first occurrences below it), and txnIds / body are written from the registers.  The fast kernel
// skips exactly these txns.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void keydeps_tiny_kernel(KeyDepsParams p)
{
    if (p.abort && *p.abort) return;           // speculative fill: outputs too small
    // launched (and skipped by the fast kernel) only for batches of few keys per txn: with the
    // fast kernel's per-txn pipeline running over every txn anyway, a thread-per-txn pass pays off
    // only when tiny txns are the bulk (measured: config 5, 4 keys/txn, +0.26 ms; an 8-rank store
    // block, 1.5 keys/txn, -0.5 ms)
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < p.n; t += gridDim.x * blockDim.x) {
        const uint32_t k0 = p.key_off[t], k = p.key_off[t + 1] - k0;
        if (k == 0 || k > TN_K) continue;
        uint32_t lo[TN_K], ex[TN_K], wc[TN_K], raw = 0;
#pragma unroll
        for (uint32_t q = 0; q < TN_K; ++q) {
            lo[q] = wc[q] = 0;
            ex[q] = raw;
            if (q < k) {
                const PairSlice ps = p.slice[k0 + q];
                lo[q] = ps.lo; wc[q] = ps.wcnt;
                raw += ps.pos - ps.lo;
            }
        }
        if (!tn_take(k, raw)) continue;
        const uint32_t wmask = witness_mask((uint32_t)(p.lsb[t] >> 1) & 7);
        const uint32_t gi = p.txn_index ? p.txn_index[t] : t;
        // candidate r of slot q sits at hist[lo_q + r - ex_q]; later slots win the select chain
        uint32_t v[TN_RAW];
#pragma unroll
        for (uint32_t r = 0; r < TN_RAW; ++r) {
            uint32_t a = lo[0] + r;
#pragma unroll
            for (uint32_t q = 1; q < TN_K; ++q) a = (q < k && r >= ex[q]) ? lo[q] + (r - ex[q]) : a;
            v[r] = TN_END;
            if (r < raw) {
                const uint32_t e = p.hist[a], j = e & ENT_TXN_MASK;
                if (((wmask >> (e >> ENT_KIND_SHIFT)) & 1u) && j != gi) v[r] = j;
            }
        }
        bool first[TN_RAW];
        uint32_t U = 0;
#pragma unroll
        for (uint32_t r = 0; r < TN_RAW; ++r) {
            bool f = v[r] != TN_END;
#pragma unroll
            for (uint32_t x = 0; x < r; ++x) f = f && v[x] != v[r];
            first[r] = f;
            U += f ? 1u : 0u;
        }
        const uint32_t key_base = p.kd_key_off[t], val_base = p.vub_off[t], k2v_base = p.kd_k2v_off[t];
        uint32_t kc = 0;
#pragma unroll
        for (uint32_t q = 0; q < TN_K; ++q) kc += wc[q] ? 1u : 0u;
        uint32_t run = 0, ns = 0;
#pragma unroll
        for (uint32_t q = 0; q < TN_K; ++q)
            if (wc[q]) {
                run += wc[q];
                p.kd_keys[key_base + ns] = p.key_ord[k0 + q];
                p.kd_k2v[k2v_base + ns] = (int32_t)(kc + run);
                ++ns;
            }
        uint32_t pos = k2v_base + kc;                   // body: witnessed candidates in slot order
#pragma unroll
        for (uint32_t r = 0; r < TN_RAW; ++r) {
            if (v[r] == TN_END) continue;
            uint32_t rank = 0;
#pragma unroll
            for (uint32_t x = 0; x < TN_RAW; ++x) rank += (first[x] && v[x] < v[r]) ? 1u : 0u;
            p.kd_k2v[pos++] = (int32_t)rank;
            if (first[r]) p.vgap[val_base + rank] = v[r];
        }
        p.cnt_vals[t] = U;
    }
}

void launch_keydeps_fast(const KeyDepsParams &p, int wpl, void *recs, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t blocks = (p.n + KD_WAVES - 1) / KD_WAVES;
    const uint32_t cap = 256u * 16u;       // 4096 blocks: 2048 / 1024 measured 6 % / 32 % slower (r04_b)
    if (blocks > cap) blocks = cap;
    blocks = (blocks + 7u) & ~7u;                       // a multiple of 8: one block class per XCD
    (void)wpl;
    // near span: 1024 txns below the bound for windows up to 384 (config 2: 94 % of the distinct
    // deps, p99 16 far ones per txn), else 2048
    static const bool copy = getenv("ACCORD_FILL_COPY") && atoi(getenv("ACCORD_FILL_COPY")) == 1;
    if (copy && p.window <= 384u) {
        hipLaunchKernelGGL((keydeps_fast_kernel<16, true>), dim3(blocks), dim3(KD_THREADS), 0, s, p, (const TxnRec *)recs);
    } else if (p.window <= 384u) {
        hipLaunchKernelGGL((keydeps_fast_kernel<16>), dim3(blocks), dim3(KD_THREADS), 0, s, p, (const TxnRec *)recs);
    } else {
        hipLaunchKernelGGL((keydeps_fast_kernel<32>), dim3(blocks), dim3(KD_THREADS), 0, s, p, (const TxnRec *)recs);
    }
}

size_t fk_temp_bytes(uint32_t n) { return (size_t)n * sizeof(TxnRec) + 64; }

void launch_keydeps(const KeyDepsParams &p, int wpl, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t blocks = (p.n + KD_WAVES - 1) / KD_WAVES;
    if (blocks > 256u * 16u) blocks = 256u * 16u;
    switch (wpl) {
    // 8 waves/SIMD caps the kernel at 80 SGPRs (some spill to VGPR lanes); measured faster than
    // 7 or fewer waves without spills (latency-bound: occupancy wins)
    case 1: hipLaunchKernelGGL((keydeps_kernel<1>), dim3(blocks), dim3(KD_THREADS), 0, s, p); break;
    case 2: hipLaunchKernelGGL((keydeps_kernel<2>), dim3(blocks), dim3(KD_THREADS), 0, s, p); break;
    default: hipLaunchKernelGGL((keydeps_kernel<4>), dim3(blocks), dim3(KD_THREADS), 0, s, p); break;
    }
}

// txnIds: gapped (upper-bound offsets) -> dense CSR, flat over the output: a block owns CV_OUT
// consecutive outputs, takes its first txn from bstart (cv_bstart_kernel), stages windows of
// CV_WIN txns' offsets in LDS and maps every quad of outputs to its txn by an LDS search --
// 16-byte coalesced stores, mostly coalesced loads, and no idle lanes whatever the mix of small and
// large txnIds lists (measured against one output per lane with 4 searches in flight: config 2
// compact 209 -> 201 us, config 3 488 -> 468 us).
constexpr uint32_t CV_OUT = 8192, CV_WIN = 256;   // 8192: 0.194 ms vs 0.196 at 4096, 0.204 at 2048 (r04_b)
struct __attribute__((aligned(4))) CvU4 { uint32_t x, y, z, w; };
// bstart[b] = the last txn t with val_off[t] <= b * CV_OUT (thread per txn; the blocks whose first
// output lies in [val_off[t], val_off[t+1]) are t's)
__global__ __launch_bounds__(256) void cv_bstart_kernel(uint32_t n, const uint32_t *__restrict__ val_off,
                                                        uint32_t *__restrict__ bstart, uint32_t cvo)
{
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        const uint32_t a = val_off[t], e = val_off[t + 1];
        for (uint32_t b = (a + cvo - 1) / cvo; b * cvo < e; ++b) bstart[b] = t;
    }
}

__global__ __launch_bounds__(256) void compact_vals_kernel(uint32_t n, const uint32_t *__restrict__ vub_off,
                                                           const uint32_t *__restrict__ val_off,
                                                           const uint32_t *__restrict__ vgap,
                                                           const uint32_t *__restrict__ bstart,
                                                           uint32_t *__restrict__ vals, uint32_t cvo)
{
    __shared__ uint32_t s_off[CV_WIN + 1], s_src[CV_WIN];
    const uint32_t total = val_off[n];
    const uint32_t o0 = blockIdx.x * cvo;
    if (o0 >= total) return;                          // block-uniform
    const uint32_t o1 = min(total, o0 + cvo);
    uint32_t t0 = bstart[blockIdx.x], o = o0;         // last txn with val_off <= o0
    while (o < o1) {                                  // block-uniform
        const uint32_t tw = t0 + threadIdx.x;
        s_off[threadIdx.x] = tw <= n ? val_off[tw] : 0xFFFFFFFFu;
        s_src[threadIdx.x] = tw < n ? vub_off[tw] : 0u;
        if (threadIdx.x == 0) s_off[CV_WIN] = t0 + CV_WIN <= n ? val_off[t0 + CV_WIN] : 0xFFFFFFFFu;
        __syncthreads();
        const uint32_t oe = min(o1, s_off[CV_WIN]);   // outputs of this window's txns
        // a lane takes 4 consecutive outputs (one 16-byte store; quads aligned to 4): one search for
        // the quad's first output, then a step forward where a txn ends inside the quad
        for (uint32_t x0 = (o & ~3u) + 4u * threadIdx.x; x0 < oe; x0 += 1024u) {
            const uint32_t xs = max(x0, o);
            uint32_t l = 0, h = CV_WIN;               // last slot with s_off <= xs
#pragma unroll
            for (int it = 0; it < 8; ++it) {
                const uint32_t m = (l + h) >> 1;
                if (h - l > 1) { if (s_off[m] <= xs) l = m; else h = m; }
            }
            uint32_t v[4];
            if (x0 >= o && x0 + 4u <= oe && s_off[l + 1] >= x0 + 4u) {
                // the quad inside one txn's run (most quads): its 4 gapped values are contiguous too --
                // one 16-byte load (4-byte aligned; gfx950 takes unaligned dwordx4)
                const CvU4 q = *(const CvU4 *)(vgap + s_src[l] + (x0 - s_off[l]));
                v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t x = x0 + j;
                    v[j] = 0u;
                    if (x >= o && x < oe) {
                        while (s_off[l + 1] <= x) ++l;    // s_off[CV_WIN] >= oe ends it
                        v[j] = vgap[s_src[l] + (x - s_off[l])];
                    }
                }
            }
            if (x0 >= o && x0 + 4u <= oe) {
                *(uint4 *)(vals + x0) = make_uint4(v[0], v[1], v[2], v[3]);
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (x0 + j >= o && x0 + j < oe) vals[x0 + j] = v[j];
            }
        }
        __syncthreads();
        o = oe;
        t0 += CV_WIN;
    }
}

} // namespace


void launch_validate_pack(uint32_t n, const uint64_t *msb, const uint64_t *lsb, const int32_t *node,
                          const uint32_t *key_off, const uint32_t *key_ord, const uint32_t *rng_off,
                          const uint32_t *rng_start, const uint32_t *rng_end, uint32_t key_lo, uint32_t key_hi,
                          uint32_t *pair_key, uint32_t *pair_ent, uint32_t *rng_owner, uint32_t *is_range,
                          const uint32_t *txn_index, const StreamPos &sp, DevStatus *status, hipStream_t s)
{
    if (n == 0) return;
    uint32_t blocks = (n + 255) / 256;               // a wave per 64 txns
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(validate_pack_kernel, dim3(blocks), dim3(256), 0, s, n, msb, lsb, node, key_off, key_ord,
                       rng_off, rng_start, rng_end, key_lo, key_hi, pair_key, pair_ent, rng_owner, is_range,
                       txn_index, sp, status);
}

__global__ __launch_bounds__(256) void compact_flags_kernel(uint32_t n, const uint32_t *__restrict__ flags,
                                                            const uint32_t *__restrict__ excl, uint32_t *__restrict__ out)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        if (flags[i]) out[excl[i]] = i;
}

void launch_accept_bounds(uint32_t n, const uint64_t *msb, const uint64_t *lsb, const int32_t *node,
                          const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode, const uint32_t *key_off,
                          const uint32_t *txn_index, uint32_t *bound_l, uint32_t *bound_g, uint32_t *pair_bound,
                          DevStatus *status, hipStream_t s)
{
    if (n == 0) return;
    uint32_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(accept_bounds_kernel, dim3(blocks), dim3(256), 0, s, n, msb, lsb, node, emsb, elsb, enode, key_off,
                       txn_index, bound_l, bound_g, pair_bound, status);
}

void launch_compact_flags(uint32_t n, const uint32_t *flags, const uint32_t *excl, uint32_t *out, hipStream_t s)
{
    if (n == 0) return;
    uint32_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(compact_flags_kernel, dim3(blocks), dim3(256), 0, s, n, flags, excl, out);
}

size_t history_temp_bytes(uint32_t P)
{
    const size_t tiles = (P + HS_TILE - 1) / HS_TILE;
    // pw_local[P] u32 | tile_max[tiles] u32 | (align 16) c_local[P] u64 | tile_cnt[tiles] u64 |
    // ccarry[tiles] ClassCarry
    size_t b = ((size_t)P + tiles) * 4;
    b = (b + 15) & ~(size_t)15;
    b += ((size_t)P + tiles) * 8;
    b = (b + 15) & ~(size_t)15;
    b += tiles * sizeof(ClassCarry) + 64;
    return b;
}

HistoryViews history_views(void *temp, uint32_t P)
{
    const uint32_t tiles = (P + HS_TILE - 1) / HS_TILE;
    HistoryViews v;
    v.pw_local = (uint32_t *)temp;
    v.pw_carry = v.pw_local + P;
    size_t off = ((size_t)P + tiles) * 4;
    off = (off + 15) & ~(size_t)15;
    v.c_local = (uint64_t *)((char *)temp + off);
    off += ((size_t)P + tiles) * 8;
    off = (off + 15) & ~(size_t)15;
    v.ccarry = (ClassCarry *)((char *)temp + off);
    return v;
}

void launch_history(uint32_t P, uint32_t nkeys, uint32_t window, const uint32_t *sorted_key,
                    const uint32_t *sorted_pair, const uint32_t *hist, uint32_t *seg_start,
                    uint32_t *seg_end, PairSlice *slice, void *temp, const uint32_t *pair_bound, uint32_t carry,
                    hipStream_t s)
{
    (void)nkeys;
    if (P == 0) return;
    const uint32_t tiles = (P + HS_TILE - 1) / HS_TILE;
    uint32_t *pw_local = (uint32_t *)temp;
    uint32_t *tile_max = pw_local + P;
    size_t off = ((size_t)P + tiles) * 4;
    off = (off + 15) & ~(size_t)15;
    uint64_t *c_local = (uint64_t *)((char *)temp + off);
    uint64_t *tile_cnt = c_local + P;
    off += ((size_t)P + tiles) * 8;
    off = (off + 15) & ~(size_t)15;
    ClassCarry *ccarry = (ClassCarry *)((char *)temp + off);
    hipLaunchKernelGGL(history1_kernel, dim3(tiles), dim3(HS_THREADS), 0, s, P, sorted_key, hist, seg_start, seg_end, pw_local, tile_max, c_local, tile_cnt);
    hipLaunchKernelGGL(history_carry_kernel, dim3(1), dim3(256), 0, s, tile_max, tile_cnt, ccarry, tiles);
    if (window <= H2_HALO) {
        uint32_t steps = 0;
        while ((1u << steps) <= window) ++steps;     // ceil(log2(window + 1)) halvings of a <= window range
        // the halo only has to reach back W positions: the smallest that does keeps the block's LDS small
        // (one 64-bit LDS word per position, key << 32 | txn, and one compare per probe measured the
        // same: segment 0.254 vs 0.250 ms, profiles/r04_b/segment_compact_ab.txt -- the probes are
        // not what bounds it)
        auto h2 = window <= 256 ? history2_lockstep_kernel<256> : window <= 512 ? history2_lockstep_kernel<512>
                : window <= 1024 ? history2_lockstep_kernel<1024> : history2_lockstep_kernel<H2_HALO>;
        hipLaunchKernelGGL(h2, dim3((P + H2_TILE - 1) / H2_TILE), dim3(H2_THREADS), 0, s, P,
                           window, steps, sorted_key, sorted_pair, hist, seg_start, pw_local, tile_max, c_local, ccarry,
                           seg_end, pair_bound, slice, carry);
        return;
    }
    hipLaunchKernelGGL(history2_kernel, dim3((P + H2_TILE - 1) / H2_TILE), dim3(H2_THREADS), 0, s, P, window,
                       sorted_key, sorted_pair, hist,
                       seg_start, pw_local, tile_max, c_local, ccarry, seg_end, pair_bound, slice, carry);
}

void launch_keydeps_sizes(uint32_t n, const uint32_t *key_off, const PairSlice *slice, uint32_t *cnt_keys,
                          uint32_t *cnt_vub, uint32_t *cnt_k2v, DevStatus *status, hipStream_t s)
{
    if (n == 0) return;
    uint32_t blocks = (n + 255) / 256;               // a wave per 64 txns
    if (blocks > 16384) blocks = 16384;
    // (a thread per txn measured 0.046 ms against 0.036 for config 2, profiles/r04_b)
    hipLaunchKernelGGL(keydeps_sizes_kernel, dim3(blocks), dim3(256), 0, s, n, key_off, slice, cnt_keys, cnt_vub,
                       cnt_k2v, status);
}

size_t keydeps_fast_temp_bytes(uint32_t n) { return fk_temp_bytes(n); }

// one workgroup per listed big txn (the list is short: a fixed grid that loops over it)
void launch_keydeps_big(const KeyDepsParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    hipLaunchKernelGGL(keydeps_big_kernel, dim3(512), dim3(BK_THREADS), 0, s, p);
}

// The fast fill's per-txn records (offsets and kind only): launched before the host reads the
// output sizes, so it runs during that wait instead of after it.
void launch_keydeps_recs(const KeyDepsParams &p, void *recs, hipStream_t s)
{
    if (p.n == 0 || p.window > 512u) return;
    uint32_t rb = (p.n + 255) / 256;
    if (rb > 4096) rb = 4096;
    hipLaunchKernelGGL(txnrec_kernel, dim3(rb), dim3(256), 0, s, p, (TxnRec *)recs);
}

void launch_keydeps_fill(const KeyDepsParams &p, int wpl, void *recs, hipStream_t s)
{
    // fast path over every txn (its records from launch_keydeps_recs); the general kernel over the
    // fallback list (fb_count zeroed by the caller).  Windows past 512 txns put most txns over the fast path's 256 candidates: general only.
    if (p.window > 512u) {
        KeyDepsParams q = p;
        q.fb_list = nullptr;
        q.fb_count = nullptr;
        launch_keydeps(q, wpl, s);
        launch_keydeps_big(p, s);
        return;
    }
    launch_keydeps_fast(p, wpl, recs, s);
    if (p.tiny) {
        uint32_t b = (p.n + 255) / 256;
        if (b > 8192) b = 8192;
        hipLaunchKernelGGL(keydeps_tiny_kernel, dim3(b), dim3(256), 0, s, p);
    }
    launch_keydeps(p, wpl, s);
    launch_keydeps_big(p, s);
}

size_t compact_temp_bytes(uint64_t max_total) { return ((max_total + 1023) / 1024 + 1) * 4 + 64; }

void launch_compact_vals(uint32_t n, const uint32_t *vub_off, const uint32_t *val_off, const uint32_t *vgap,
                         uint32_t *vals, uint64_t max_total, void *temp, hipStream_t s)
{
    if (n == 0 || max_total == 0) return;
    const uint32_t cvo = CV_OUT;                        // outputs per block
    const uint64_t blocks = (max_total + cvo - 1) / cvo;   // blocks past the exact total exit
    uint32_t *bstart = (uint32_t *)temp;
    uint32_t sb = (n + 255) / 256;
    if (sb > 4096) sb = 4096;
    hipLaunchKernelGGL(cv_bstart_kernel, dim3(sb), dim3(256), 0, s, n, val_off, bstart, cvo);
    hipLaunchKernelGGL(compact_vals_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, n, vub_off, val_off, vgap, bstart,
                       vals, cvo);
}

} // namespace accord

#ifdef ACCORD_FK_STAMPS
extern "C" int accord_dbg_fk_stamps(unsigned long long *out)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(accord::g_fk_stamps), 16 * 8) != hipSuccess) return -1;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(accord::g_fk_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
