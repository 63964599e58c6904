// Range transactions: RangeDeps for every txn and the KeyDeps
// of range-domain txns.
//
// Reference semantics (paths relative to accord-core/src/main/java/accord/):
//   range-command scan       impl/InMemoryCommandStore.java:883-1016 (Erased skipped :891,
//                            txnId < startedBefore :901-902, witness :927, each range of the
//                            command intersecting the query -> (range, txnId) :950-959, collected
//                            in a TreeMap by Range.compare and replayed in that order)
//   range query over CFKs    impl/InMemoryCommandStore.java:274-289 (every CFK key in (start,end])
//   RangeDeps layout         primitives/RangeDeps.java:81-99 (RelationMultiMap with Range keys)
// Under the status-at-time model a range command j is live for txn i iff i-W <= j < i, so the
// candidate ranges of txn i are exactly the contiguous span rng[rng_off[max(0,i-W)], rng_off[i])
// of the batch's range CSR (the window bounds the live set; each wave stabs it directly).
#include "device_common.h"
#include "kernels.h"

#include <algorithm>
#include <cstdlib>
#include "../../include/accord_deps.h"

namespace accord {

namespace {

constexpr int RD_WAVES = 4;
constexpr uint32_t RD_HCAP = 256;            // hits per txn in the main pass (5 KiB of LDS per wave)
constexpr uint32_t RD_HCAP_BIG = 2048;       // txns with more hits: a one-wave-per-block pass over a list

__device__ __forceinline__ void rd_overflow(DevStatus *st, uint32_t i)
{
    atomicAdd(&st->overflow, 1u);
    atomicMin(&st->overflow_first, i);
}

template <uint32_t HCAP> struct RdLds {
    unsigned long long code[HCAP];      // start << 32 | end
    uint32_t j[HCAP];
    uint32_t jrank[HCAP];
    uint32_t first[HCAP];               // first hit (lowest txn) of its range
};

// Does (s, e] intersect the query of txn i?  Key query: some key k with s < k <= e.  Range query:
// some (qs, qe] with s < qe && qs < e (Range.compareIntersecting semantics, Range.java:296-308).
__device__ __forceinline__ bool rd_hits(const RangeDepsParams &p, uint32_t s, uint32_t e, bool key_query, uint32_t q0,
                                        uint32_t q1)
{
    if (key_query) {
        uint32_t lo = q0, hi = q1;                       // first key > s
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (p.key_ord[m] <= s) lo = m + 1; else hi = m;
        }
        return lo < q1 && p.key_ord[lo] <= e;
    }
    uint32_t lo = q0, hi = q1;                           // first query range with end > s
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (p.rng_end[m] <= s) lo = m + 1; else hi = m;
    }
    return lo < q1 && p.rng_start[lo] < e;
}

// Per-txn pass (LIST = false): the txns the tile pass handed on, hits up to HCAP; a txn with more
// is appended to a list in the count pass and skipped (by both passes).  Big pass (LIST = true):
// the listed txns with RD_HCAP_BIG hits of LDS; more than that is reported as overflow.
template <bool FILL, uint32_t HCAP, int WAVES, bool LIST>
__global__ __launch_bounds__(WAVES * 64) void rangedeps_kernel(RangeDepsParams p)
{
    __shared__ RdLds<HCAP> lds_all[WAVES];
    const uint32_t w = wave_id(), lane = lane_id();
    RdLds<HCAP> &L = lds_all[w];
    const uint64_t lt = lanemask_lt();
    // main pass: the txns the tile pass handed on (rd_fb_list); big pass: those with more hits
    const uint32_t limit = LIST ? *p.rd_big_count : *p.rd_fb_count;
    for (uint32_t it = blockIdx.x * WAVES + w; it < limit; it += gridDim.x * WAVES) {
        const uint32_t i = LIST ? p.rd_big_list[it] : p.rd_fb_list[it];
        const uint64_t lsb_i = p.lsb[i];
        const uint32_t wmask = witness_mask((uint32_t)(lsb_i >> 1) & 7);
        const bool key_query = (lsb_i & 1) == 0;
        const uint32_t q0 = key_query ? p.key_off[i] : p.rng_off[i];
        const uint32_t q1 = key_query ? p.key_off[i + 1] : p.rng_off[i + 1];
        // live range commands: started in the window and before the bound (i; Accept: executeAt).
        // Candidate index space: the ncr carried commands (resident stores), then the batch's.
        const uint32_t g = p.g0 + i;
        const uint32_t lo_g = g > p.window ? g - p.window : 0u;
        uint32_t r_lo;
        if (lo_g >= p.g0) {
            r_lo = p.ncr + p.rng_off[lo_g - p.g0];
        } else {
            uint32_t l = 0, h = p.ncr;                   // first carried command with owner >= lo_g
            while (l < h) {
                const uint32_t m = (l + h) >> 1;
                if (p.rc_owner[m] < lo_g) l = m + 1; else h = m;
            }
            r_lo = l;
        }
        const uint32_t r_hi = p.ncr + p.rng_off[p.bound_l ? p.bound_l[i] : i];
        uint32_t H = 0;
        // up to 8 query keys / ranges: held wave-uniform, every candidate tested by compares
        const uint32_t nq = q1 - q0;
        const bool few = nq <= 8;
        uint32_t qa[8], qb[8];                           // key: (key, key); range: (start, end)
        {
            uint32_t va = 0, vb = 0;
            if (few && lane < nq) {
                va = key_query ? p.key_ord[q0 + lane] : p.rng_start[q0 + lane];
                vb = key_query ? va : p.rng_end[q0 + lane];
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) { qa[q] = readlane(va, q); qb[q] = readlane(vb, q); }
        }
        if (q1 > q0) {
            for (uint32_t r0 = r_lo; r0 < r_hi; r0 += 64) {
                const uint32_t r = r0 + lane;
                bool hit = false;
                uint32_t j = 0, s = 0, e = 0;
                uint32_t jkind = 0;
                if (r < r_hi) {
                    if (r < p.ncr) {
                        j = p.rc_owner[r]; s = p.rc_start[r]; e = p.rc_end[r]; jkind = p.rc_kind[r];
                    } else {
                        const uint32_t rb = r - p.ncr, jl = p.rng_owner[rb];
                        j = p.g0 + jl; s = p.rng_start[rb]; e = p.rng_end[rb];
                        jkind = (uint32_t)(p.lsb[jl] >> 1) & 7;
                    }
                    bool inter = false;
                    if (few) {
#pragma unroll
                        for (int q = 0; q < 8; ++q)
                            inter = inter || ((uint32_t)q < nq && (key_query ? (qa[q] > s && qa[q] <= e)
                                                                             : (s < qb[q] && qa[q] < e)));
                    } else {
                        inter = rd_hits(p, s, e, key_query, q0, q1);
                    }
                    hit = inter && j != g && ((wmask >> jkind) & 1u);   // p1
                }
                const uint64_t bal = __ballot(hit);
                const uint32_t h = H + (uint32_t)__popcll(bal & lt);
                if (hit && h < HCAP) {
                    L.code[h] = ((unsigned long long)s << 32) | e;
                    L.j[h] = j;
                }
                H += (uint32_t)__popcll(bal);
            }
        }
        if (H > HCAP) {
            if (!FILL && lane == 0) {
                if (LIST) {
                    rd_overflow(p.status, i);
                    p.cnt_rngs[i] = 0; p.cnt_vals[i] = 0; p.cnt_r2v[i] = 0;
                } else {
                    p.rd_big_list[atomicAdd(p.rd_big_count, 1u)] = i;
                }
            }
            continue;
        }
        wave_lds_sync();
        // hits arrive in range-CSR order, i.e. TxnId order: distinct txnIds are the transitions
        uint32_t run = 0;
        for (uint32_t h0 = 0; h0 < H; h0 += 64) {
            const uint32_t h = h0 + lane;
            const bool tr = h < H && (h == 0 || L.j[h] != L.j[h - 1]);
            const uint64_t bal = __ballot(tr);
            if (h < H) L.jrank[h] = run + (uint32_t)__popcll(bal & ((lt << 1) | 1ull)) - 1u;
            run += (uint32_t)__popcll(bal);
        }
        const uint32_t uj = run;
        wave_lds_sync();
        // distinct ranges (Range.compare order) and sorted positions: O(H^2) over a tiny H
        uint32_t ur = 0;
        for (uint32_t h = lane; h < H; h += 64) {
            const unsigned long long c = L.code[h];
            bool first = true;
            for (uint32_t g = 0; g < H; ++g)
                if (L.code[g] == c && L.j[g] < L.j[h]) { first = false; break; }
            ur += first ? 1u : 0u;
            L.first[h] = first ? 1u : 0u;
        }
        ur = wave_sum(ur);
        wave_lds_sync();
        if (!FILL) {
            if (lane == 0) { p.cnt_rngs[i] = ur; p.cnt_vals[i] = uj; p.cnt_r2v[i] = ur + H; }
            continue;
        }
        const uint32_t rb = p.rd_rng_off[i], vb = p.rd_val_off[i], xb = p.rd_r2v_off[i];
        for (uint32_t h = lane; h < H; h += 64) {
            const unsigned long long c = L.code[h];
            const uint32_t jh = L.j[h];
            uint32_t le_code = 0, before = 0, first_before = 0;
            const bool first = L.first[h] != 0;
            for (uint32_t g = 0; g < H; ++g) {
                const unsigned long long cg = L.code[g];
                const uint32_t jg = L.j[g];
                le_code += cg <= c ? 1u : 0u;
                before += (cg < c || (cg == c && jg < jh)) ? 1u : 0u;
                first_before += (cg < c && L.first[g]) ? 1u : 0u;   // distinct ranges below c
            }
            p.rd_vals[vb + L.jrank[h]] = jh;
            p.rd_r2v[xb + ur + before] = (int32_t)L.jrank[h];
            if (first) {
                p.rd_rng_start[rb + first_before] = (uint32_t)(c >> 32);
                p.rd_rng_end[rb + first_before] = (uint32_t)c;
                p.rd_r2v[xb + first_before] = (int32_t)(ur + le_code);
            }
        }
    }
}

// Tile pass: one wave per 64 consecutive txns, a lane per txn.  Consecutive txns see nearly the
// same live range commands, so the wave stages the union of its lanes' candidate windows in LDS
// once and every lane scans its own window there (the per-txn pass reloads ~W live commands per
// txn).  A lane keeps up to RT_HL hits (candidate indices); a txn with more hits, more than 8 query
// keys/ranges, or a tile whose window exceeds RT_CAND goes to the per-txn pass (count: appended to
// rd_fb_list; fill: skipped, the per-txn pass fills it).  Same outputs as rangedeps_kernel.
constexpr uint32_t RT_CAND = 512, RT_HL = 16, RT_WAVES = 2;
struct RtLds {
    uint32_t s[RT_CAND], e[RT_CAND], jk[RT_CAND];     // jk = owner position | witness kind << 29
    uint32_t hit[64 * RT_HL];
};

__device__ __forceinline__ void rd_fb_push(const RangeDepsParams &p, uint32_t i)
{
    p.rd_fb_list[atomicAdd(p.rd_fb_count, 1u)] = i;
}

template <bool FILL>
__global__ __launch_bounds__(RT_WAVES * 64) void rangedeps_tile_kernel(RangeDepsParams p)
{
    __shared__ RtLds lds_all[RT_WAVES];
    const uint32_t w = wave_id(), lane = lane_id();
    RtLds &L = lds_all[w];
    const uint32_t ntiles = (p.n + 63) / 64;
    for (uint32_t tile = blockIdx.x * RT_WAVES + w; tile < ntiles; tile += gridDim.x * RT_WAVES) {
        const uint32_t i = tile * 64 + lane;
        const bool valid = i < p.n;
        const uint32_t g = p.g0 + i;
        uint32_t r_lo = 0, r_hi = 0;
        if (valid) {
            const uint32_t lo_g = g > p.window ? g - p.window : 0u;
            if (lo_g >= p.g0) {
                r_lo = p.ncr + p.rng_off[lo_g - p.g0];
            } else {
                uint32_t l = 0, h = p.ncr;
                while (l < h) {
                    const uint32_t m = (l + h) >> 1;
                    if (p.rc_owner[m] < lo_g) l = m + 1; else h = m;
                }
                r_lo = l;
            }
            r_hi = p.ncr + p.rng_off[p.bound_l ? p.bound_l[i] : i];
        }
        const uint32_t R_lo = ~readlane(wave_incl_max(valid ? ~r_lo : 0u), 63);
        const uint32_t R_hi = readlane(wave_incl_max(valid ? r_hi : 0u), 63);
        if (R_hi > R_lo && R_hi - R_lo > RT_CAND) {           // window too large: per-txn pass
            if (!FILL && valid) rd_fb_push(p, i);
            continue;
        }
        static_assert(RT_HL == 2 * RT_HIT_WORDS, "hit words");
        for (uint32_t c = lane; R_lo + c < R_hi; c += 64) {
            const uint32_t r = R_lo + c;
            uint32_t j, s, e, kind;
            if (r < p.ncr) {
                j = p.rc_owner[r]; s = p.rc_start[r]; e = p.rc_end[r]; kind = p.rc_kind[r];
            } else {
                const uint32_t rb = r - p.ncr, jl = p.rng_owner[rb];
                j = p.g0 + jl; s = p.rng_start[rb]; e = p.rng_end[rb];
                kind = (uint32_t)(p.lsb[jl] >> 1) & 7;
            }
            L.s[c] = s; L.e[c] = e; L.jk[c] = j | (kind << 29);
        }
        wave_lds_sync();
        bool fb = false;
        uint32_t H = 0;
        if (FILL && valid && p.rt_h) {
            // the count pass kept every txn's hits (candidate slots of this same window): no rescan
            const uint32_t hh = p.rt_h[i];
            fb = hh == 0xFFFFFFFFu;
            if (!fb) {
                H = hh;
                const uint32_t *src = p.rt_hits + (size_t)i * RT_HIT_WORDS;
                for (uint32_t h = 0; h < H; h += 2) {
                    const uint32_t v = src[h >> 1];
                    L.hit[lane * RT_HL + h] = v & 0xFFFFu;
                    if (h + 1 < H) L.hit[lane * RT_HL + h + 1] = v >> 16;
                }
            }
        } else if (valid) {
            const uint64_t lsb_i = p.lsb[i];
            const uint32_t wmask = witness_mask((uint32_t)(lsb_i >> 1) & 7);
            const bool key_query = (lsb_i & 1) == 0;
            const uint32_t q0 = key_query ? p.key_off[i] : p.rng_off[i];
            const uint32_t q1 = key_query ? p.key_off[i + 1] : p.rng_off[i + 1];
            const uint32_t nq = q1 - q0;
            if (nq > 8) {
                fb = true;
            } else if (nq > 0) {
                uint32_t qa[8], qb[8];
#pragma unroll
                for (uint32_t q = 0; q < 8; ++q) {
                    qa[q] = q < nq ? (key_query ? p.key_ord[q0 + q] : p.rng_start[q0 + q]) : 0u;
                    qb[q] = q < nq ? (key_query ? qa[q] : p.rng_end[q0 + q]) : 0u;
                }
                for (uint32_t c = r_lo - R_lo; c < r_hi - R_lo; ++c) {
                    const uint32_t s = L.s[c], e = L.e[c], jk = L.jk[c];
                    bool inter = false;
#pragma unroll
                    for (uint32_t q = 0; q < 8; ++q)
                        inter = inter || (q < nq && (key_query ? (qa[q] > s && qa[q] <= e) : (s < qb[q] && qa[q] < e)));
                    if (inter && (jk & ENT_TXN_MASK) != g && ((wmask >> (jk >> 29)) & 1u)) {
                        if (H < RT_HL) L.hit[lane * RT_HL + H] = c;
                        ++H;
                    }
                }
            }
            if (H > RT_HL) fb = true;
            if (!FILL && p.rt_h) {                        // the hits, for the fill pass
                p.rt_h[i] = fb ? 0xFFFFFFFFu : H;
                if (!fb) {
                    const uint32_t *hs = L.hit + lane * RT_HL;
                    uint32_t *dst = p.rt_hits + (size_t)i * RT_HIT_WORDS;
                    for (uint32_t h = 0; h < H; h += 2) dst[h >> 1] = hs[h] | (h + 1 < H ? hs[h + 1] << 16 : 0u);
                }
            }
        }
        if (fb) {
            if (!FILL) rd_fb_push(p, i);
        } else if (valid) {
            // hits in candidate order = ascending owner: distinct owners are the transitions; distinct
            // ranges (Range.compare order) by an O(H^2) pass over the few hits
            const uint32_t *hs = L.hit + lane * RT_HL;
            uint32_t ur = 0, uj = 0, prevj = 0xFFFFFFFFu;
            for (uint32_t h = 0; h < H; ++h) {
                const uint32_t c = hs[h], j = L.jk[c] & ENT_TXN_MASK;
                uj += j != prevj ? 1u : 0u;
                prevj = j;
                bool first = true;
                for (uint32_t x = 0; x < h; ++x) {
                    const uint32_t cx = hs[x];
                    if (L.s[cx] == L.s[c] && L.e[cx] == L.e[c]) { first = false; break; }
                }
                ur += first ? 1u : 0u;
            }
            if (!FILL) {
                p.cnt_rngs[i] = ur; p.cnt_vals[i] = uj; p.cnt_r2v[i] = ur + H;
            } else {
                const uint32_t rb = p.rd_rng_off[i], vb = p.rd_val_off[i], xb = p.rd_r2v_off[i];
                uint32_t jrank = 0xFFFFFFFFu;
                prevj = 0xFFFFFFFFu;
                for (uint32_t h = 0; h < H; ++h) {
                    const uint32_t c = hs[h], jh = L.jk[c] & ENT_TXN_MASK;
                    const unsigned long long code = ((unsigned long long)L.s[c] << 32) | L.e[c];
                    if (jh != prevj) { ++jrank; prevj = jh; p.rd_vals[vb + jrank] = jh; }
                    uint32_t le_code = 0, before = 0, first_before = 0;
                    bool first = true;
                    for (uint32_t x = 0; x < H; ++x) {
                        const uint32_t cx = hs[x];
                        const unsigned long long cg = ((unsigned long long)L.s[cx] << 32) | L.e[cx];
                        le_code += cg <= code ? 1u : 0u;
                        before += (cg < code || (cg == code && x < h)) ? 1u : 0u;
                        if (cg == code && x < h) first = false;
                        // distinct ranges below code: count each code at its first hit
                        if (cg < code) {
                            bool fx = true;
                            for (uint32_t y = 0; y < x; ++y) {
                                const uint32_t cy = hs[y];
                                if (L.s[cy] == L.s[cx] && L.e[cy] == L.e[cx]) { fx = false; break; }
                            }
                            first_before += fx ? 1u : 0u;
                        }
                    }
                    p.rd_r2v[xb + ur + before] = (int32_t)jrank;
                    if (first) {
                        p.rd_rng_start[rb + first_before] = (uint32_t)(code >> 32);
                        p.rd_rng_end[rb + first_before] = (uint32_t)code;
                        p.rd_r2v[xb + first_before] = (int32_t)(ur + le_code);
                    }
                }
            }
        }
        wave_lds_sync();
    }
}

// ---------------------------------------------------------------------------------------------
// KeyDeps of range txns.  Every key of the txn's ranges with history before it contributes the
// same [lcw, pos) slice as a key txn would (CommandsForKey.mapReduceActive :614-650): pos = first
// entry with txn >= i, lcw = last Write before i-W.  Both are found from per-key checkpoints
// (first history position at or after each 4096-txn block boundary) by a short gallop, so a query
// costs a handful of loads instead of two binary searches over the key's whole history.
//   count : per range txn (one wave), keys with witnessed deps and the body size
//   fill  : keys, keysToTxnIds header, and the body holding the dep txn indices (key order)
//   union : per range txn, the body sorted in LDS -> unique txnIds (kd_vals at the upper-bound
//           offsets, compacted with the key txns' later) and the body rewritten to ranks
// ---------------------------------------------------------------------------------------------
constexpr int RK_WAVES = 4;
constexpr int RK_FB = 4;                       // fill: groups of 64 history loads in flight
constexpr int RK_EMAX = 128;                   // largest union class: 8192 deps per range txn
// fill: a chunk whose raw candidates fit RK_CM (and no slice is longer than RK_CMRAW) maps every
// candidate to its history position through an LDS table, one read instead of a binary search
constexpr uint32_t RK_CM = 640, RK_CMRAW = 32;

// cp[b * K + k] = {x, yo | d << 12} (8 bytes): x = first position of key k's segment [a, c) with
// txn(x) >= b << RK_CP_SHIFT (c if none); yo = txn(x) - (b << RK_CP_SHIFT) saturated at 4095 (4095
// if none) -- enough to compare txn(x) with any query txn of block b; d = x - pw(x), pw(x) =
// (last Write at or before x - 1) + 1 (global history positions, 0 if none), RK_CP_DFAR when it
// does not fit 20 bits (the reader recomputes pw).  Thread per history position: it owns the
// blocks between its predecessor and itself.
constexpr uint32_t RK_CP_YMAX = (1u << RK_CP_SHIFT) - 1u, RK_CP_DFAR = (1u << (32 - RK_CP_SHIFT)) - 1u;
static_assert(RK_CP_SHIFT == 12, "checkpoint word: 12 bits of txn offset, 20 of Write distance");
__device__ __forceinline__ uint2 rk_cp_make(uint32_t x, uint32_t yo, uint32_t pw)
{
    const uint32_t d = x - pw;
    return make_uint2(x, yo | (d < RK_CP_DFAR ? d : RK_CP_DFAR) << RK_CP_SHIFT);
}
__device__ __forceinline__ uint32_t rk_pw_before(const RangeDepsParams &p, uint32_t x)
{
    return x ? max(p.pw_local[x - 1], p.pw_carry[(x - 1) / p.pw_tile]) : 0u;
}

// Hot keys (segments of more than RK_CP_COLD entries): a thread per history position writes the
// cells of the blocks it is the first entry at or after.  Cold keys: a lane per key walks the
// blocks and its few entries together (rk_checkpoint_cold_kernel), so each row's cells are written
// coalesced, where a thread per position had written a cold key's column of ~ncp cells as
// scattered 8-byte stores (config 3 rk_checkpoints stage 0.325 -> 0.258 ms with 96; 32 / 256
// measured 0.284 / 0.272, a walk prefetching the next entry 0.270; profiles/r05_cp/checkpoint_ab.txt).
constexpr uint32_t RK_CP_COLD = 96;
__global__ __launch_bounds__(256) void rk_checkpoint_kernel(uint32_t P, const uint32_t *__restrict__ sorted_key,
                                                            RangeDepsParams p)
{
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < P; x += gridDim.x * blockDim.x) {
        const uint32_t k = sorted_key[x];
        const uint32_t a = p.seg_start[k], c = p.seg_end[k];
        if (c - a <= RK_CP_COLD) continue;              // rk_checkpoint_cold_kernel's
        const uint32_t t = p.hist[x] & ENT_TXN_MASK;
        // absolute txn blocks [cp_base, cp_base + ncp) live in the table
        const uint32_t b_end = p.cp_base + p.ncp;
        const uint32_t b_lo = max(p.cp_base, x == a ? 0u : ((p.hist[x - 1] & ENT_TXN_MASK) >> RK_CP_SHIFT) + 1u);
        const uint32_t b_hi = min(t >> RK_CP_SHIFT, b_end - 1u);
        if (b_lo <= b_hi) {
            const uint2 v = rk_cp_make(x, RK_CP_YMAX, rk_pw_before(p, x));     // blocks before t's
            for (uint32_t b = b_lo; b < b_hi; ++b) p.cp[(size_t)(b - p.cp_base) * p.nkeys + k] = v;
            p.cp[(size_t)(b_hi - p.cp_base) * p.nkeys + k] =
                b_hi == t >> RK_CP_SHIFT ? rk_cp_make(x, t & RK_CP_YMAX, rk_pw_before(p, x)) : v;
        }
        if (x + 1 == c && (t >> RK_CP_SHIFT) + 1u < b_end) {
            const uint2 v = rk_cp_make(c, RK_CP_YMAX, rk_pw_before(p, c));
            for (uint32_t b = max(p.cp_base, (t >> RK_CP_SHIFT) + 1u); b < b_end; ++b)
                p.cp[(size_t)(b - p.cp_base) * p.nkeys + k] = v;
        }
    }
}

// a lane per key with 0 < entries <= RK_CP_COLD: every block of the table, the key's first entry with
// txn at or after the block's start (or the segment end), as rk_checkpoint_kernel would write it
__global__ __launch_bounds__(256) void rk_checkpoint_cold_kernel(RangeDepsParams p)
{
    const uint32_t b_end = p.cp_base + p.ncp;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < p.nkeys; k += gridDim.x * blockDim.x) {
        const uint32_t a = p.seg_start[k], c = p.seg_end[k];
        if (a >= c || c - a > RK_CP_COLD) continue;
        uint32_t q = a, tq = p.hist[a] & ENT_TXN_MASK;
        uint32_t pwq = rk_pw_before(p, a);
        for (uint32_t b = p.cp_base; b < b_end; ++b) {
            bool moved = false;
            while (q < c && tq < (b << RK_CP_SHIFT)) {
                ++q;
                tq = q < c ? p.hist[q] & ENT_TXN_MASK : 0xFFFFFFFFu;
                moved = true;
            }
            if (moved) pwq = rk_pw_before(p, q);
            const uint32_t yo = q < c && (tq >> RK_CP_SHIFT) == b ? (tq & RK_CP_YMAX) : RK_CP_YMAX;
            p.cp[(size_t)(b - p.cp_base) * p.nkeys + k] = rk_cp_make(q, yo, pwq);
        }
    }
}

// first position q in [from, to) with txn(q) >= t, given txn(from - 1) < t: gallop then bisect
__device__ __forceinline__ uint32_t rk_first_ge(const uint32_t *__restrict__ hist, uint32_t from, uint32_t to,
                                                uint32_t t)
{
    uint32_t lo = from, step = 1;
    while (lo < to && (hist[lo] & ENT_TXN_MASK) < t) {
        const uint32_t probe = lo + step;
        if (probe >= to || (hist[probe] & ENT_TXN_MASK) >= t) {
            uint32_t l = lo + 1, h = min(probe, to);
            while (l < h) {
                const uint32_t m = (l + h) >> 1;
                if ((hist[m] & ENT_TXN_MASK) < t) l = m + 1; else h = m;
            }
            return l;
        }
        lo = probe + 1;
        step <<= 1;
    }
    return lo;
}

struct RkSlice {
    uint32_t lo, raw, wcnt;
    uint32_t l, pre;        // first entry inside the window; 1 if lo is the last Write before it
};

// The deps slices of range txn i on U keys per lane (store-relative kk[u], valid[u]): raw entries
// [lo, lo + raw), of which wcnt are witnessed by wmask.  The checkpoints at blocks i and i - W
// usually give both bounds and the Write bound outright (coalesced loads, consecutive keys);
// only keys with entries between a checkpoint and the bound gallop.  Short slices count their
// witnessed entries directly (one cache line), long ones through the class counts.
constexpr uint32_t RK_SHORT = 8;
template <int U>
__device__ __forceinline__ void rk_slices(const RangeDepsParams &p, uint32_t i, const uint32_t (&kk)[U],
                                          const bool (&valid)[U], uint32_t wmask, RkSlice (&out)[U])
{
    const uint32_t g = p.g0 + i;                    // stream position (history entries hold them)
    const bool windowed = g > p.window;
    const uint32_t thr = windowed ? g - p.window : 0u;
    // slices end at the first entry with txn >= eb (g; Accept: the txns started before executeAt)
    const uint32_t eb = p.bound_l ? p.g0 + p.bound_l[i] : g;
    const bool past = (eb >> RK_CP_SHIFT) >= p.cp_base + p.ncp;   // eb on the last block boundary: whole segment
    const size_t row1 = (size_t)(past ? 0u : (eb >> RK_CP_SHIFT) - p.cp_base) * p.nkeys,
                 row2 = (size_t)((thr >> RK_CP_SHIFT) - p.cp_base) * p.nkeys;
    uint32_t a[U], c[U];
    uint2 e1[U], e2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        a[u] = c[u] = 0;
        e1[u] = e2[u] = make_uint2(0u, 0u);
        if (valid[u]) {
            a[u] = p.seg_start[kk[u]]; c[u] = p.seg_end[kk[u]];
            e1[u] = p.cp[row1 + kk[u]]; e2[u] = p.cp[row2 + kk[u]];
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        out[u] = RkSlice{0u, 0u, 0u};
        if (!(valid[u] && a[u] < c[u])) continue;
        const uint32_t pos = past ? c[u]
                           : (e1[u].y & RK_CP_YMAX) >= (eb & RK_CP_YMAX) ? e1[u].x
                                                                         : rk_first_ge(p.hist, e1[u].x + 1, c[u], eb);
        if (pos == a[u]) continue;
        uint32_t pw = 0, l = a[u];
        if (windowed) {
            if ((e2[u].y & RK_CP_YMAX) >= (thr & RK_CP_YMAX) || e2[u].x >= pos) {
                l = min(e2[u].x, pos);
                const uint32_t d = e2[u].y >> RK_CP_SHIFT;
                pw = l == e2[u].x && d != RK_CP_DFAR ? e2[u].x - d : rk_pw_before(p, l);
            } else {
                l = rk_first_ge(p.hist, e2[u].x + 1, pos, thr);
                pw = rk_pw_before(p, l);
            }
        }
        const bool pre = windowed && pw > a[u];
        const uint32_t lo = pre ? pw - 1 : a[u];
        out[u].lo = lo;
        out[u].raw = pos - lo;
        out[u].l = l;
        out[u].pre = pre ? 1u : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t raw = out[u].raw;
        if (raw == 0) continue;
        uint32_t wc = 0;
        if ((p.kinds_present & ~wmask) == 0) {
            wc = raw;                                   // every kind in the history is witnessed
        } else if ((p.kinds_present & ~3u) == 0 && wmask == 2u) {
            // Reads and Writes only, the txn witnesses Writes: before the window just the last Write
            // (lo; the entries after it there are Reads), inside it the Writes of [l, pos)
            const uint32_t l = out[u].l, pos = out[u].lo + raw;
            wc = out[u].pre;
            if (pos - l <= RK_SHORT) {
                for (uint32_t x = l; x < pos; ++x) wc += (p.hist[x] >> ENT_KIND_SHIFT) == 1u ? 1u : 0u;
            } else {
                wc += witnessed_upto(p.c_local, p.ccarry, pos - 1, wmask, p.pw_tile) -
                      (l ? witnessed_upto(p.c_local, p.ccarry, l - 1, wmask, p.pw_tile) : 0u);
            }
        } else if (raw <= RK_SHORT) {
            for (uint32_t r = 0; r < raw; ++r) wc += (wmask >> (p.hist[out[u].lo + r] >> ENT_KIND_SHIFT)) & 1u;
        } else {
            const uint32_t lo = out[u].lo, pos = lo + raw;
            wc = witnessed_upto(p.c_local, p.ccarry, pos - 1, wmask, p.pw_tile) -
                 (lo ? witnessed_upto(p.c_local, p.ccarry, lo - 1, wmask, p.pw_tile) : 0u);
        }
        out[u].wcnt = wc;
    }
}

// Stored slice (count pass -> fill pass): lo, and raw | wcnt << 16; RK_SLICE_WIDE marks a slice
// too long for 16-bit fields (the fill pass recomputes it).
constexpr uint32_t RK_SLICE_WIDE = 0xFFFFFFFFu;
constexpr uint32_t RK_BITMAP_SPAN = 4096;      // 128 LDS words of one wave's union buffer

// Per range txn (one wave): count pass computes and stores every key's slice (keys of its ranges
// in ascending order, clipped to the store) and the KeyDeps sizes; the fill pass writes keys, the
// keysToTxnIds header and the body holding the dep txn indices (key order).
template <bool FILL, int U>                          // U keys per lane per step
// (8 waves per SIMD: 67 -> 64 VGPRs with 12 B of scratch; rangekeys count 1.62 -> 1.39 ms, config 3
// 6.80 -> 6.58 ms/step on one box, profiles/r06_c3/union_occupancy.txt)
__global__ __launch_bounds__(RK_WAVES * 64) __attribute__((amdgpu_waves_per_eu(8))) void rangekeys_kernel(RangeDepsParams p)
{
    __shared__ uint32_t rex_all[RK_WAVES][64 * U], rlo_all[RK_WAVES][64 * U];
    __shared__ uint32_t cmap_all[FILL ? RK_WAVES : 1][FILL ? RK_CM : 1];
    const uint32_t w = wave_id(), lane = lane_id();
    uint32_t *rex = rex_all[w], *rlo = rlo_all[w];
    uint32_t *cmap = cmap_all[FILL ? w : 0];
    const uint64_t lt = lanemask_lt();
    for (uint32_t li = blockIdx.x * RK_WAVES + w; li < p.n_range_txns; li += gridDim.x * RK_WAVES) {
        const uint32_t i = p.range_txns[li];
        const uint32_t wmask = witness_mask((uint32_t)(p.lsb[i] >> 1) & 7);
        const uint32_t q0 = p.rng_off[i], q1 = p.rng_off[i + 1];
        uint2 *slices = p.rk_slices + p.rk_off[li];
        uint32_t key_base = 0, k2v_base = 0, kc_total = 0;
        if (FILL) {
            key_base = p.kd_key_off[i];
            kc_total = p.kd_key_off[i + 1] - key_base;
            k2v_base = p.kd_k2v_off[i];
        }
        uint32_t kc = 0, body = 0, kidx = 0;
        for (uint32_t r = q0; r < q1; ++r) {
            const uint32_t ks = max(p.rng_start[r] + 1, p.key_lo), ke = min(p.rng_end[r], p.key_hi - 1);   // keys (s, e]
            if (ks > ke) continue;
            for (uint32_t c0 = ks; c0 <= ke && c0 >= ks; c0 += 64 * U) {
                RkSlice sl[U];
                uint32_t kk[U];
                bool valid[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t key = c0 + 64 * u + lane;
                    valid[u] = key <= ke && key >= ks;
                    kk[u] = valid[u] ? key - p.key_lo : 0u;
                }
                if (!FILL) {
                    rk_slices<U>(p, i, kk, valid, wmask, sl);
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        if (valid[u]) {
                            const bool narrow = sl[u].raw < 65536u;
                            slices[kidx + (c0 - ks) + 64 * u + lane] =
                                make_uint2(sl[u].lo, narrow ? sl[u].raw | (sl[u].wcnt << 16) : RK_SLICE_WIDE);
                        }
                        kc += (uint32_t)__popcll(__ballot(sl[u].wcnt > 0));
                        body += wave_sum(sl[u].wcnt);
                    }
                    continue;
                }
                bool wide = false;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    sl[u] = RkSlice{0u, 0u, 0u};
                    if (valid[u]) {
                        const uint2 v = slices[kidx + (c0 - ks) + 64 * u + lane];
                        if (v.y == RK_SLICE_WIDE) wide = true;
                        else sl[u] = RkSlice{v.x, v.y & 0xFFFFu, v.y >> 16};
                    }
                }
                if (__ballot(wide)) {                 // rare: recompute the long slices
                    RkSlice re[U];
                    rk_slices<U>(p, i, kk, valid, wmask, re);
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        if (re[u].raw >= 65536u) sl[u] = re[u];
                }
                // headers of the chunk's U*64 keys, their raw entries' prefix in LDS, then the body of
                // the whole chunk with RK_FB groups of 64 history loads in flight
                const uint32_t body0 = body;
                uint32_t rbase = 0, rexu[U], rawu[U], mraw = 0;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t key = c0 + 64 * u + lane;
                    const bool has = sl[u].wcnt > 0;
                    const uint64_t hb = __ballot(has);
                    const uint32_t raw = has ? sl[u].raw : 0u;   // witnessed-free slices: no candidates
                    const uint32_t wincl = wave_incl_scan(sl[u].wcnt);
                    if (has) {
                        const uint32_t ns = kc + (uint32_t)__popcll(hb & lt);
                        p.kd_keys[key_base + ns] = key;
                        p.kd_k2v[k2v_base + ns] = (int32_t)(kc_total + body + wincl);
                    }
                    const uint32_t rincl = wave_incl_scan(raw);
                    rex[u * 64 + lane] = rexu[u] = rbase + rincl - raw;
                    rlo[u * 64 + lane] = sl[u].lo;
                    rawu[u] = raw;
                    mraw = max(mraw, raw);
                    rbase += readlane(rincl, 63);
                    kc += (uint32_t)__popcll(hb);
                    body += readlane(wincl, 63);
                }
                // candidates in key order; body position = running witnessed count
                uint32_t run = body0;
                if (rbase <= RK_CM && readlane(wave_incl_max(mraw), 63) <= RK_CMRAW) {   // wave-uniform
#pragma unroll
                    for (int u = 0; u < U; ++u)
                        for (uint32_t j = 0; j < rawu[u]; ++j) cmap[rexu[u] + j] = sl[u].lo + j;
                    wave_lds_sync();
                    for (uint32_t w0 = 0; w0 < rbase; w0 += 64 * RK_FB) {
                        uint32_t e[RK_FB];
#pragma unroll
                        for (int b = 0; b < RK_FB; ++b) {
                            const uint32_t rr = w0 + 64 * b + lane;
                            e[b] = rr < rbase ? p.hist[cmap[rr]] : 0u;
                        }
#pragma unroll
                        for (int b = 0; b < RK_FB; ++b) {
                            const uint32_t rr = w0 + 64 * b + lane;
                            const bool wit = rr < rbase && ((wmask >> (e[b] >> ENT_KIND_SHIFT)) & 1u);
                            const uint64_t wb = __ballot(wit);
                            if (wit) p.kd_k2v[k2v_base + kc_total + run + (uint32_t)__popcll(wb & lt)] = (int32_t)(e[b] & ENT_TXN_MASK);
                            run += (uint32_t)__popcll(wb);
                        }
                    }
                    wave_lds_sync();
                    continue;
                }
                wave_lds_sync();
                for (uint32_t w0 = 0; w0 < rbase; w0 += 64 * RK_FB) {
                    uint32_t e[RK_FB];
#pragma unroll
                    for (int b = 0; b < RK_FB; ++b) {
                        const uint32_t rr = w0 + 64 * b + lane;
                        e[b] = 0;
                        if (rr < rbase) {
                            uint32_t sidx = 0;       // last slot with rex <= rr (rex[0] = 0)
#pragma unroll
                            for (uint32_t step = 32 * U; step >= 1; step >>= 1)
                                if (sidx + step < 64u * U && rex[sidx + step] <= rr) sidx += step;
                            e[b] = p.hist[rlo[sidx] + (rr - rex[sidx])];
                        }
                    }
#pragma unroll
                    for (int b = 0; b < RK_FB; ++b) {
                        const uint32_t rr = w0 + 64 * b + lane;
                        const bool wit = rr < rbase && ((wmask >> (e[b] >> ENT_KIND_SHIFT)) & 1u);
                        const uint64_t wb = __ballot(wit);
                        if (wit) p.kd_k2v[k2v_base + kc_total + run + (uint32_t)__popcll(wb & lt)] = (int32_t)(e[b] & ENT_TXN_MASK);
                        run += (uint32_t)__popcll(wb);
                    }
                }
                wave_lds_sync();
            }
            kidx += ke - ks + 1;
        }
        if (!FILL && lane == 0) {
            p.cnt_keys[i] = kc;
            p.cnt_vals_k[i] = body;        // txnIds upper bound (exact count: the union pass)
            p.cnt_k2v[i] = kc + body;
        }
    }
}

// keys of every range txn's ranges (clipped to the store): the offsets of its stored slices
__global__ __launch_bounds__(256) void rk_nkeys_kernel(RangeDepsParams p, uint32_t *__restrict__ cnt)
{
    for (uint32_t li = blockIdx.x * blockDim.x + threadIdx.x; li < p.n_range_txns; li += gridDim.x * blockDim.x) {
        const uint32_t i = p.range_txns[li];
        uint32_t c = 0;
        for (uint32_t r = p.rng_off[i]; r < p.rng_off[i + 1]; ++r) {
            const uint32_t ks = max(p.rng_start[r] + 1, p.key_lo), ke = min(p.rng_end[r], p.key_hi - 1);
            if (ks <= ke) c += ke - ks + 1;
        }
        cnt[li] = c;
    }
}

// ---- union sort: a bitonic network over n = 64*E keys held in registers ----
// Two register layouts: striped (element g = r*64 + lane, register bits = g bits 6..) and blocked
// (g = lane*E + r, register bits = g bits 0..e-1).  A stage on bit jb runs in-lane, as plain
// min/max on register pairs, in the layout whose register bits hold jb; the layout switches by a
// transposition through the wave's LDS (E stores + E loads per lane, conflict-free padding), and
// only bits in neither layout (E < 64: bits e..5) exchange through lane shuffles.  Every stage is
// resolved at compile time (template recursion over the stage index).
constexpr int ilog2c(int x) { return x <= 1 ? 0 : 1 + ilog2c(x >> 1); }
constexpr int us_stages(int logn) { return logn * (logn + 1) / 2; }
constexpr int us_kb(int s) { int kb = 1; while (s >= kb) { s -= kb; ++kb; } return kb; }
constexpr int us_jb(int s) { int kb = 1; while (s >= kb) { s -= kb; ++kb; } return kb - 1 - s; }
// layout a stage on bit jb runs in (1 striped, 0 blocked), given the current one
constexpr int us_need(int e, int jb, int cur) { return jb >= 6 ? 1 : jb < e ? 0 : cur; }
constexpr int us_layout_before(int e, int s)
{
    int cur = 1;                                     // loaded striped (coalesced)
    for (int t = 0; t < s; ++t) cur = us_need(e, us_jb(t), cur);
    return cur;
}
// LDS words of one wave's sort buffer: element g at g + g/32 + g/1024
constexpr uint32_t us_lds_words(int E) { return 64u * E + 2u * E + (uint32_t)E / 16u + 1u; }

// lane base / per-register offset of element (lane, r) in the padded buffer (exact for powers of 2)
template <int E> __device__ __forceinline__ uint32_t us_base(int layout, uint32_t lane)
{
    return layout ? lane + (lane >> 5) : lane * E + ((lane * E) >> 5) + ((lane * E) >> 10);
}
template <int E> __host__ __device__ constexpr uint32_t us_off(int layout, int r)
{
    return layout ? (uint32_t)r * 66u + ((uint32_t)r >> 4) : (uint32_t)r + ((uint32_t)r >> 5);
}

template <int E, int FROM>
__device__ __forceinline__ void us_transpose(uint32_t (&v)[E], uint32_t *lds, uint32_t lane)
{
    const uint32_t bw = us_base<E>(FROM, lane), br = us_base<E>(1 - FROM, lane);
#pragma unroll
    for (int r = 0; r < E; ++r) lds[bw + us_off<E>(FROM, r)] = v[r];
    wave_lds_sync();
#pragma unroll
    for (int r = 0; r < E; ++r) v[r] = lds[br + us_off<E>(1 - FROM, r)];
    wave_lds_sync();
}

template <int E, int S>
__device__ __forceinline__ void us_stage(uint32_t (&v)[E], uint32_t *lds, uint32_t lane)
{
    constexpr int e = ilog2c(E), logn = e + 6;
    constexpr int kb = us_kb(S), jb = us_jb(S);
    constexpr int cur = us_layout_before(e, S), lay = us_need(e, jb, cur);
    if constexpr (lay != cur) us_transpose<E, cur>(v, lds, lane);
    // ascending iff bit kb of g is 0 (kb == logn: the last merge, all ascending)
    constexpr bool k_all = kb >= logn;
    constexpr bool k_reg = !k_all && (lay ? kb >= 6 : kb < e);
    constexpr int krb = k_reg ? (lay ? kb - 6 : kb) : 0;
    constexpr int klb = (!k_all && !k_reg) ? (lay ? kb : kb - e) : 0;
    const bool asc_lane = (k_all || k_reg) ? true : ((lane >> klb) & 1u) == 0;
    constexpr bool j_reg = lay ? jb >= 6 : jb < e;
    if constexpr (j_reg) {
        constexpr int rb = lay ? jb - 6 : jb;
#pragma unroll
        for (int r = 0; r < E; ++r) {
            if ((r >> rb) & 1) continue;
            const int r2 = r | (1 << rb);
            const bool asc = k_reg ? ((r >> krb) & 1) == 0 : asc_lane;
            const uint32_t a = v[r], b = v[r2];
            const uint32_t lo = min(a, b), hi = max(a, b);
            v[r] = asc ? lo : hi;
            v[r2] = asc ? hi : lo;
        }
    } else {
        constexpr int lb = lay ? jb : jb - e;
        const bool lower = ((lane >> lb) & 1u) == 0;
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const bool asc = k_reg ? ((r >> krb) & 1) == 0 : asc_lane;
            const uint32_t o = (uint32_t)__shfl_xor((int)v[r], 1 << lb, 64);
            v[r] = (lower == asc) ? min(v[r], o) : max(v[r], o);
        }
    }
}

// all stages from S on; ends in the blocked layout
template <int E, int S>
__device__ __forceinline__ void us_run(uint32_t (&v)[E], uint32_t *lds, uint32_t lane)
{
    constexpr int e = ilog2c(E);
    if constexpr (S < us_stages(e + 6)) {
        us_stage<E, S>(v, lds, lane);
        us_run<E, S + 1>(v, lds, lane);
    } else if constexpr (us_layout_before(e, S) != 0) {
        us_transpose<E, 1>(v, lds, lane);
    }
}

// One range txn's union with E keys per lane (D <= 64*E): sort the body, write the unique dep txn
// indices (txnIds, ascending = TxnId order) and replace every body entry by its rank.  When the
// body's values span less than 2^(32 - log2 n) the sort runs on packed (value - min, position)
// keys, so each entry's rank comes out of the sorted order directly; otherwise it sorts the values
// and finds the ranks by binary search over the unique values in LDS.
template <int E>
__device__ __forceinline__ void rk_union(const RangeDepsParams &p, uint32_t i, uint32_t D, uint32_t k2v_base,
                                         uint32_t vb, uint32_t *lds, uint32_t lane)
{
    constexpr int IB = ilog2c(E) + 6;
    constexpr uint32_t IMASK = (1u << IB) - 1u;
    uint32_t v[E];
    uint32_t vmin = 0xFFFFFFFFu, vmax = 0;
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const uint32_t g = (uint32_t)r * 64 + lane;
        v[r] = g < D ? (uint32_t)p.kd_k2v[k2v_base + g] : 0xFFFFFFFFu;
        if (g < D) { vmin = min(vmin, v[r]); vmax = max(vmax, v[r]); }
    }
    vmin = ~readlane(wave_incl_max(~vmin), 63);
    vmax = readlane(wave_incl_max(vmax), 63);
    if (vmax - vmin < RK_BITMAP_SPAN && p.rk_bitmap) {
        // the body's values span < 4096 txns (always, in a store whose window is <= 4096): the union
        // is a bitmap over the span in LDS (lane l owns words 2l, 2l+1), the unique txns its set bits
        // in order and each entry's rank the set bits below it -- no sort
        lds[lane] = 0u; lds[64 + lane] = 0u;
        wave_lds_sync();
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const uint32_t g = (uint32_t)r * 64 + lane;
            if (g < D) {
                const uint32_t off = v[r] - vmin;
                atomicOr(&lds[off >> 5], 1u << (off & 31));
            }
        }
        wave_lds_sync();
        const uint32_t w0 = lds[2 * lane], w1 = lds[2 * lane + 1];
        const uint32_t c0 = (uint32_t)__popc(w0), c = c0 + (uint32_t)__popc(w1);
        const uint32_t incl = wave_incl_scan(c);
        const uint32_t U = readlane(incl, 63), excl = incl - c;
        lds[128 + 2 * lane] = excl;
        lds[128 + 2 * lane + 1] = excl + c0;
        if (lane == 0) p.cnt_vals_exact[i] = U;
        wave_lds_sync();
        uint32_t pos = vb + excl;
        for (uint32_t m = w0; m; m &= m - 1) p.kd_vals[pos++] = vmin + 64 * lane + (uint32_t)__builtin_ctz(m);
        for (uint32_t m = w1; m; m &= m - 1) p.kd_vals[pos++] = vmin + 64 * lane + 32 + (uint32_t)__builtin_ctz(m);
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const uint32_t g = (uint32_t)r * 64 + lane;
            if (g < D) {
                const uint32_t off = v[r] - vmin, wd = off >> 5;
                p.kd_k2v[k2v_base + g] = (int32_t)(lds[128 + wd] + (uint32_t)__popc(lds[wd] & ((1u << (off & 31)) - 1u)));
            }
        }
        wave_lds_sync();
        return;
    }
    const bool packed = vmax - vmin < (1u << (32 - IB)) - 1u;
    if (packed) {
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const uint32_t g = (uint32_t)r * 64 + lane;
            if (g < D) v[r] = ((v[r] - vmin) << IB) | g;
        }
    }
    us_run<E, 0>(v, lds, lane);                       // blocked: element g = lane*E + r, ascending
    const uint32_t sh = packed ? (uint32_t)IB : 0u;
    const uint32_t prev_last = (uint32_t)__shfl_up((int)v[E - 1], 1, 64);
    uint32_t cnt = 0;
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const uint32_t g = lane * E + (uint32_t)r;
        const uint32_t prev = r ? v[r - 1] : prev_last;
        cnt += (g < D && (g == 0 || (v[r] >> sh) != (prev >> sh))) ? 1u : 0u;
    }
    const uint32_t incl = wave_incl_scan(cnt);
    const uint32_t U = readlane(incl, 63);
    uint32_t idx = incl - cnt;
    if (lane == 0) p.cnt_vals_exact[i] = U;
    // outputs leave through the LDS buffer (free after the sort), so the stores coalesce
    if (packed) {
        // ranks by body position
        uint32_t run = idx;
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const uint32_t g = lane * E + (uint32_t)r;
            const uint32_t prev = r ? v[r - 1] : prev_last;
            if (g < D) {
                run += (g == 0 || (v[r] >> IB) != (prev >> IB)) ? 1u : 0u;
                lds[v[r] & IMASK] = run - 1u;
            }
        }
        wave_lds_sync();
        for (uint32_t x = lane; x < D; x += 64) p.kd_k2v[k2v_base + x] = (int32_t)lds[x];
        wave_lds_sync();
#pragma unroll
        for (int r = 0; r < E; ++r) {
            const uint32_t g = lane * E + (uint32_t)r;
            const uint32_t prev = r ? v[r - 1] : prev_last;
            if (g < D && (g == 0 || (v[r] >> IB) != (prev >> IB))) lds[idx++] = (v[r] >> IB) + vmin;
        }
        wave_lds_sync();
        for (uint32_t x = lane; x < U; x += 64) p.kd_vals[vb + x] = lds[x];
        wave_lds_sync();
        return;
    }
    uint32_t *ubuf = lds;
#pragma unroll
    for (int r = 0; r < E; ++r) {
        const uint32_t g = lane * E + (uint32_t)r;
        const uint32_t prev = r ? v[r - 1] : prev_last;
        if (g < D && (g == 0 || v[r] != prev)) ubuf[idx++] = v[r];
    }
    wave_lds_sync();
    for (uint32_t x = lane; x < U; x += 64) p.kd_vals[vb + x] = ubuf[x];
    // ranks: four lower-bound searches per lane in lockstep (one LDS round trip per step)
    for (uint32_t x0 = 0; x0 < D; x0 += 256) {
        uint32_t j[4], l[4], h[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t x = x0 + (uint32_t)q * 64 + lane;
            j[q] = x < D ? (uint32_t)p.kd_k2v[k2v_base + x] : 0u;
            l[q] = 0;
            h[q] = U;
        }
        for (uint32_t span = U; span > 0; span >>= 1) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (l[q] < h[q]) {
                    const uint32_t m = (l[q] + h[q]) >> 1;
                    if (ubuf[m] < j[q]) l[q] = m + 1; else h[q] = m;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            // a search may need one step more than log2(U) iterations of the halving span
            while (l[q] < h[q]) {
                const uint32_t m = (l[q] + h[q]) >> 1;
                if (ubuf[m] < j[q]) l[q] = m + 1; else h[q] = m;
            }
            const uint32_t x = x0 + (uint32_t)q * 64 + lane;
            if (x < D) p.kd_k2v[k2v_base + x] = (int32_t)l[q];
        }
    }
    wave_lds_sync();
}

// Size classes of the range txns' bodies: D in (0, 256], (256, 1024], (1024, 2048], (2048, 4096],
// (4096, 8192] -> lists (wave-aggregated appends); D = 0 is finished here, larger overflows.
__global__ __launch_bounds__(256) void rk_classes_kernel(RangeDepsParams p)
{
    __shared__ uint32_t cnt_s[RK_CLASSES], base_s[RK_CLASSES];
    const uint32_t lane = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint32_t nrt = p.n_range_txns;
    for (uint32_t b = blockIdx.x * blockDim.x; b < nrt; b += gridDim.x * blockDim.x) {
        const uint32_t li = b + threadIdx.x;
        int c = -1;
        uint4 rec = make_uint4(0u, 0u, 0u, 0u);
        if (li < nrt) {
            const uint32_t i = p.range_txns[li];
            const uint32_t kc = p.kd_key_off[i + 1] - p.kd_key_off[i];
            const uint32_t D = p.kd_k2v_off[i + 1] - p.kd_k2v_off[i] - kc;
            if (D == 0) p.cnt_vals_exact[i] = 0;
            else if (D > 8192u) rd_overflow(p.status, i);
            else c = D <= 256u ? 0 : D <= 1024u ? 1 : D <= 2048u ? 2 : D <= 4096u ? 3 : 4;
            rec = make_uint4(i, D, p.kd_k2v_off[i] + kc, p.kd_val_off[i]);
        }
        // block-level appends: wave offsets in LDS, one global atomic per class per block
        uint32_t mine = 0;
        __syncthreads();
        if (threadIdx.x < RK_CLASSES) cnt_s[threadIdx.x] = 0;
        __syncthreads();
        for (int k = 0; k < (int)RK_CLASSES; ++k) {
            const uint64_t m = __ballot(c == k);
            if (!m) continue;
            const uint32_t leader = (uint32_t)__builtin_ctzll(m);
            uint32_t wb = 0;
            if (lane == leader) wb = atomicAdd(&cnt_s[k], (uint32_t)__popcll(m));
            wb = readlane(wb, (int)leader);
            if (c == k) mine = wb + (uint32_t)__popcll(m & lt);
        }
        __syncthreads();
        if (threadIdx.x < RK_CLASSES) base_s[threadIdx.x] = cnt_s[threadIdx.x] ? atomicAdd(&p.rk_cls[threadIdx.x], cnt_s[threadIdx.x]) : 0u;
        __syncthreads();
        if (c >= 0) reinterpret_cast<uint4 *>(p.rk_cls + 8)[(size_t)c * nrt + base_s[c] + mine] = rec;
    }
}

// Union pass of one size class: one wave per listed range txn, the registers and LDS of its class.
template <int E, int WPE>
__global__ __launch_bounds__(RK_WAVES * 64) __attribute__((amdgpu_waves_per_eu(WPE)))
void rangekeys_union_kernel(RangeDepsParams p, uint32_t cls)
{
    __shared__ uint32_t buf_all[RK_WAVES][us_lds_words(E)];
    const uint32_t w = wave_id(), lane = lane_id();
    uint32_t *buf = buf_all[w];
    const uint32_t count = p.rk_cls[cls];
    const uint4 *list = reinterpret_cast<const uint4 *>(p.rk_cls + 8) + (size_t)cls * p.n_range_txns;
    const uint32_t stride = gridDim.x * RK_WAVES;
    uint32_t it = blockIdx.x * RK_WAVES + w;
    uint4 rec = it < count ? list[it] : make_uint4(0u, 0u, 0u, 0u);
    for (; it < count; it += stride) {
        const uint4 cur = rec;                          // {txn, D, body base, txnIds base}
        if (it + stride < count) rec = list[it + stride];   // the next record, in flight meanwhile
        rk_union<E>(p, cur.x, cur.y, cur.z, cur.w, buf, lane);
    }
}

} // namespace

static uint32_t rt_blocks(uint32_t n)
{
    const uint32_t tiles = (n + 63) / 64;
    uint32_t b = (tiles + RT_WAVES - 1) / RT_WAVES;
    return b > 8192u ? 8192u : b;
}

void launch_rangedeps_count(const RangeDepsParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    hipLaunchKernelGGL(rangedeps_tile_kernel<false>, dim3(rt_blocks(p.n)), dim3(RT_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL((rangedeps_kernel<false, RD_HCAP, RD_WAVES, false>), dim3(1024), dim3(RD_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL((rangedeps_kernel<false, RD_HCAP_BIG, 1, true>), dim3(256), dim3(64), 0, s, p);
}

void launch_rangedeps_fill(const RangeDepsParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    hipLaunchKernelGGL(rangedeps_tile_kernel<true>, dim3(rt_blocks(p.n)), dim3(RT_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL((rangedeps_kernel<true, RD_HCAP, RD_WAVES, false>), dim3(1024), dim3(RD_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL((rangedeps_kernel<true, RD_HCAP_BIG, 1, true>), dim3(256), dim3(64), 0, s, p);
}

size_t rangekeys_cp_bytes(uint32_t ncp, uint32_t nkeys)
{
    return (size_t)ncp * nkeys * sizeof(uint2) + 64;
}

void launch_rangekeys_checkpoints(uint32_t PH, const uint32_t *sorted_key, const RangeDepsParams &p, hipStream_t s)
{
    if (p.n_range_txns == 0 || PH == 0) return;
    // (a thread per (block, key) cell with coalesced row stores and a bisection per cell measured
    // slower: config-3 count 2.88 vs 2.40 ms, profiles/r04_b/rangekeys_ab.txt)
    uint32_t blocks = (PH + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(rk_checkpoint_kernel, dim3(blocks), dim3(256), 0, s, PH, sorted_key, p);
    hipLaunchKernelGGL(rk_checkpoint_cold_kernel, dim3(std::min<uint32_t>((p.nkeys + 255) / 256, 8192u)), dim3(256), 0, s, p);
}

namespace {

// first candidate (carried, then the batch's) whose owner >= thr: owners ascend along the order
__global__ void rc_first_kernel(RangeDepsParams p, uint32_t R, uint32_t thr, uint32_t *first,
                                unsigned long long *kept)
{
    uint32_t l = 0, h = p.ncr + R;
    while (l < h) {
        const uint32_t m = (l + h) >> 1;
        const uint32_t o = m < p.ncr ? p.rc_owner[m] : p.g0 + p.rng_owner[m - p.ncr];
        if (o < thr) l = m + 1; else h = m;
    }
    first[0] = l;
    *kept = p.ncr + R - l;
}

__global__ __launch_bounds__(256) void rc_copy_kernel(RangeDepsParams p, uint32_t R, const uint32_t *__restrict__ first,
                                                      uint32_t *__restrict__ oo, uint32_t *__restrict__ os,
                                                      uint32_t *__restrict__ oe, uint32_t *__restrict__ ok)
{
    const uint32_t f = first[0], tot = p.ncr + R;
    for (uint32_t e = f + blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += gridDim.x * blockDim.x) {
        uint32_t o, s, en, k;
        if (e < p.ncr) { o = p.rc_owner[e]; s = p.rc_start[e]; en = p.rc_end[e]; k = p.rc_kind[e]; }
        else {
            const uint32_t r = e - p.ncr, jl = p.rng_owner[r];
            o = p.g0 + jl; s = p.rng_start[r]; en = p.rng_end[r]; k = (uint32_t)(p.lsb[jl] >> 1) & 7;
        }
        oo[e - f] = o; os[e - f] = s; oe[e - f] = en; ok[e - f] = k;
    }
}

// registered-status stores: keep the commands not erased (ACCORD_ST_ERASED: off the range scan for
// good, impl/InMemoryCommandStore.java:891), owners stay ascending
__device__ __forceinline__ void rc_entry(const RangeDepsParams &p, uint32_t e, uint32_t &o, uint32_t &s, uint32_t &en,
                                         uint32_t &k)
{
    if (e < p.ncr) { o = p.rc_owner[e]; s = p.rc_start[e]; en = p.rc_end[e]; k = p.rc_kind[e]; }
    else {
        const uint32_t r = e - p.ncr, jl = p.rng_owner[r];
        o = p.g0 + jl; s = p.rng_start[r]; en = p.rng_end[r]; k = (uint32_t)(p.lsb[jl] >> 1) & 7;
    }
}

__global__ __launch_bounds__(256) void rc_flag_kernel(RangeDepsParams p, uint32_t R, uint32_t thr, uint32_t *__restrict__ flag)
{
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < p.ncr + R; e += gridDim.x * blockDim.x) {
        uint32_t o, s, en, k;
        rc_entry(p, e, o, s, en, k);
        flag[e] = o >= thr && k != RC_KIND_ERASED ? 1u : 0u;
    }
}

__global__ __launch_bounds__(256) void rc_scatter_kernel(RangeDepsParams p, uint32_t R, const uint32_t *__restrict__ flag,
                                                         const uint32_t *__restrict__ off, uint32_t *__restrict__ oo,
                                                         uint32_t *__restrict__ os, uint32_t *__restrict__ oe,
                                                         uint32_t *__restrict__ ok)
{
    for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < p.ncr + R; e += gridDim.x * blockDim.x) {
        if (!flag[e]) continue;
        uint32_t o, s, en, k;
        rc_entry(p, e, o, s, en, k);
        const uint32_t d = off[e];
        oo[d] = o; os[d] = s; oe[d] = en; ok[d] = k;
    }
}

} // namespace

void launch_range_carry(const RangeDepsParams &p, uint32_t R, uint32_t thr, uint32_t *out_owner, uint32_t *out_start,
                        uint32_t *out_end, uint32_t *out_kind, uint32_t *first_tmp, unsigned long long *kept,
                        uint32_t *flags, uint32_t *offs, void *scan_state, hipStream_t s)
{
    uint32_t blocks = (p.ncr + R + 255) / 256;
    if (blocks < 1) blocks = 1;
    if (blocks > 4096) blocks = 4096;
    if (flags) {
        hipLaunchKernelGGL(rc_flag_kernel, dim3(blocks), dim3(256), 0, s, p, R, thr, flags);
        exclusive_scan_u32(flags, offs, p.ncr + R, kept, scan_state, s);
        hipLaunchKernelGGL(rc_scatter_kernel, dim3(blocks), dim3(256), 0, s, p, R, flags, offs, out_owner, out_start,
                           out_end, out_kind);
        return;
    }
    hipLaunchKernelGGL(rc_first_kernel, dim3(1), dim3(1), 0, s, p, R, thr, first_tmp, kept);
    hipLaunchKernelGGL(rc_copy_kernel, dim3(blocks), dim3(256), 0, s, p, R, first_tmp, out_owner, out_start, out_end, out_kind);
}

static uint32_t rk_blocks(uint32_t nrt)
{
    // grid cap: 32768 blocks (about a wave per range txn at config 3) put config 3 at 8.03 ms against
    // 8.40 with 4096, 8.06 with 16384 and 8.13 with 65536 (profiles/r04_b/rangekeys_ab.txt)
    const uint32_t cap = 32768u;
    uint32_t b = (nrt + RK_WAVES - 1) / RK_WAVES;
    return b > cap ? cap : b;
}

void launch_rangekeys_nkeys(const RangeDepsParams &p, uint32_t *cnt, hipStream_t s)
{
    if (p.n_range_txns == 0) return;
    uint32_t blocks = (p.n_range_txns + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(rk_nkeys_kernel, dim3(blocks), dim3(256), 0, s, p, cnt);
}

void launch_rangekeys_count(const RangeDepsParams &p, hipStream_t s)
{
    if (p.n_range_txns == 0) return;
    // 4 keys per lane: at 8 waves per SIMD, 1.38 -> 1.355 ms against 8 (12: 2.39, spilling;
    // profiles/r06_c3/union_occupancy.txt)
    hipLaunchKernelGGL((rangekeys_kernel<false, 4>), dim3(rk_blocks(p.n_range_txns)), dim3(RK_WAVES * 64), 0, s, p);
}

void launch_rangekeys_fill(const RangeDepsParams &p, hipStream_t s)
{
    if (p.n_range_txns == 0) return;
    hipLaunchKernelGGL((rangekeys_kernel<true, 4>), dim3(rk_blocks(p.n_range_txns)), dim3(RK_WAVES * 64), 0, s, p);
}

void launch_rangekeys_union(const RangeDepsParams &p, hipStream_t s)
{
    if (p.n_range_txns == 0) return;
    uint32_t cb = (p.n_range_txns + 255) / 256;
    hipLaunchKernelGGL(rk_classes_kernel, dim3(cb > 2048 ? 2048 : cb), dim3(256), 0, s, p);
    const dim3 g(rk_blocks(p.n_range_txns)), b(RK_WAVES * 64);
    // occupancy targets per class (waves per SIMD; no spills at any of them): 1024-element sorts at 5
    // (105 -> 96 VGPRs) and 2048-element ones at 4 (163 -> 128 VGPRs, LDS-balanced at 4 blocks per CU)
    // took config 3 from 7.13 to 6.93 ms/step (profiles/r06_c3/union_occupancy.txt)
    hipLaunchKernelGGL((rangekeys_union_kernel<4, 8>), g, b, 0, s, p, 0u);
    hipLaunchKernelGGL((rangekeys_union_kernel<16, 5>), g, b, 0, s, p, 1u);
    hipLaunchKernelGGL((rangekeys_union_kernel<32, 4>), g, b, 0, s, p, 2u);
    hipLaunchKernelGGL((rangekeys_union_kernel<64, 2>), g, b, 0, s, p, 3u);
    hipLaunchKernelGGL((rangekeys_union_kernel<RK_EMAX, 1>), g, b, 0, s, p, 4u);
}

} // namespace accord
