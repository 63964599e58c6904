// Deps-set operations over every txn of device-resident PartialDeps:
//
//   union  : RelationMultiMap.linearUnion / Deps.merge (utils/RelationMultiMap.java:561-816,
//            primitives/KeyDeps.java:115-140, primitives/RangeDeps.java:101-126) of G sets whose
//            keys may overlap -- the coordinator-side merge of replica replies and PartialDeps.with.
//   slice  : KeyDeps.slice (primitives/KeyDeps.java:189-236), RangeDeps.slice
//            (primitives/RangeDeps.java:545-565 with the RangeAndMapCollector :727-848 driven by
//            CheckpointIntervalArray.forEach, utils/CheckpointIntervalArray.java:100-221) and
//            trimUnusedValues (utils/RelationMultiMap.java:491-532).
//   invert : RelationMultiMap.invert (utils/RelationMultiMap.java:907-938), the lazy
//            txnIdsToKeys / txnIdsToRanges (KeyDeps.java:350-362, RangeDeps.java:537-543).
//
// Values of every set index one TxnId table sorted ascending (the batch), so TxnId order is index
// order.  A "side" is the KeyDeps or the RangeDeps half; RangeDeps keys are ranges compared by
// Range.compare (start, then end: primitives/Range.java:310-317) == the u64 code start<<32|end.
//
// Layout: one wave per txn (grid-stride), lanes over a txn's elements.  Every sorted-set union is
// computed without capacity limits and without sorting, as ranks: an element of list g is the
// owner of its value when no earlier list of the group holds it; its rank in the union is the
// number of owners smaller than it, summed over the lists (one binary search per list).  Kernels
// never read global memory another lane of the same launch wrote.
#include "device_common.h"
#include "kernels.h"
#include "../../include/accord_deps.h"

namespace accord {

namespace {

constexpr int DS_WAVES = 4;

struct PI {   // one part's txn: element bases (relative to the part's arrays) and counts
    uint32_t kb, nk, vb, nv, xb, nx;
};

__device__ __forceinline__ PI part_info(const DsSide &S, uint32_t g, uint32_t t)
{
    PI p;
    const uint32_t *ko = S.key_off[g], *vo = S.val_off[g], *xo = S.x_off[g];
    p.kb = ko[t] - ko[0]; p.nk = ko[t + 1] - ko[t];
    p.vb = vo[t] - vo[0]; p.nv = S.val_cnt[g] ? S.val_cnt[g][t] : vo[t + 1] - vo[t];
    p.xb = xo[t] - xo[0]; p.nx = xo[t + 1] - xo[t];
    return p;
}

__device__ __forceinline__ uint64_t key_code(const DsSide &S, uint32_t g, uint32_t idx)
{
    const uint64_t lo = S.lo[g][idx];
    return S.range ? (lo << 32 | S.hi[g][idx]) : lo;
}

// first position in [0, len) whose element is >= x (elements via f(i))
template <typename F>
__device__ __forceinline__ uint32_t lower_bound_f(uint32_t len, uint64_t x, F f)
{
    uint32_t l = 0, h = len;
    while (l < h) {
        const uint32_t m = (l + h) >> 1;
        if (f(m) < x) l = m + 1; else h = m;
    }
    return l;
}

// key index a of body position q (relative to the body start): first a with header > nk + q
__device__ __forceinline__ uint32_t key_of_body(const int32_t *x, uint32_t nk, uint32_t q)
{
    uint32_t l = 0, h = nk;
    while (l < h) {
        const uint32_t m = (l + h) >> 1;
        if ((uint32_t)x[m] <= nk + q) l = m + 1; else h = m;
    }
    return l;
}

__device__ __forceinline__ uint32_t body_lo(const int32_t *x, uint32_t nk, uint32_t a)   // relative to body
{
    return (a == 0 ? nk : (uint32_t)x[a - 1]) - nk;
}

#define DS_TXN_LOOP(t, n) for (uint32_t t = blockIdx.x * DS_WAVES + wave_id(); t < (n); t += gridDim.x * DS_WAVES)

// ------------------------------------------------------------------------------------------
// union
// ------------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void un_lens_kernel(DsUnionParams p)
{
    const uint32_t G = p.S.G;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.n * G; i += gridDim.x * blockDim.x) {
        const PI pi = part_info(p.S, i % G, i / G);
        p.vlen[i] = pi.nv; p.klen[i] = pi.nk; p.blen[i] = pi.nx - pi.nk;
    }
}

// KIND 0: txnIds, KIND 1: keys.  Owner prefix per element, owners per list, union size per txn.
template <int KIND>
__global__ __launch_bounds__(DS_WAVES * 64) void un_owner_kernel(DsUnionParams p)
{
    const uint32_t lane = lane_id(), G = p.S.G;
    const uint32_t *eoff = KIND ? p.keoff : p.veoff;
    uint32_t *own = KIND ? p.kown : p.vown, *lst = KIND ? p.klst : p.vlst, *cnt = KIND ? p.cnt_keys : p.cnt_vals;
    DS_TXN_LOOP(t, p.n) {
        uint32_t total = 0;
        for (uint32_t g = 0; g < G; ++g) {
            const PI pg = part_info(p.S, g, t);
            const uint32_t len = KIND ? pg.nk : pg.nv, eo = eoff[t * G + g];
            uint32_t carry = 0;
            for (uint32_t j0 = 0; j0 < len; j0 += 64) {
                const uint32_t j = j0 + lane;
                const bool active = j < len;
                const uint64_t x = !active ? 0 : KIND ? key_code(p.S, g, pg.kb + j) : (uint64_t)p.S.vals[g][pg.vb + j];
                bool owner = active;
                for (uint32_t h = 0; h < g && owner; ++h) {
                    const PI ph = part_info(p.S, h, t);
                    const uint32_t lh = KIND ? ph.nk : ph.nv;
                    const uint32_t q = KIND ? lower_bound_f(lh, x, [&](uint32_t i) { return key_code(p.S, h, ph.kb + i); })
                                            : lower_bound_f(lh, x, [&](uint32_t i) { return (uint64_t)p.S.vals[h][ph.vb + i]; });
                    if (q < lh && (KIND ? key_code(p.S, h, ph.kb + q) : (uint64_t)p.S.vals[h][ph.vb + q]) == x) owner = false;
                }
                const uint64_t b = __ballot(owner);
                if (active) own[eo + j] = carry + (uint32_t)__popcll(b & lanemask_lt());
                carry += (uint32_t)__popcll(b);
            }
            if (lane == 0) lst[t * G + g] = carry;
            total += carry;
        }
        if (lane == 0) cnt[t] = total;
    }
}

// rank of every element in its txn's union; owners write the union
template <int KIND>
__global__ __launch_bounds__(DS_WAVES * 64) void un_rank_kernel(DsUnionParams p)
{
    const uint32_t lane = lane_id(), G = p.S.G;
    const uint32_t *eoff = KIND ? p.keoff : p.veoff;
    const uint32_t *own = KIND ? p.kown : p.vown, *lst = KIND ? p.klst : p.vlst, *ooff = KIND ? p.out_key_off : p.out_val_off;
    uint32_t *rank_out = KIND ? p.krank : p.vrank;
    DS_TXN_LOOP(t, p.n) {
        const uint32_t ob = ooff[t];
        for (uint32_t g = 0; g < G; ++g) {
            const PI pg = part_info(p.S, g, t);
            const uint32_t len = KIND ? pg.nk : pg.nv, eo = eoff[t * G + g];
            for (uint32_t j = lane; j < len; j += 64) {
                const uint64_t x = KIND ? key_code(p.S, g, pg.kb + j) : (uint64_t)p.S.vals[g][pg.vb + j];
                uint32_t rank = 0;
                for (uint32_t h = 0; h < G; ++h) {
                    if (h == g) { rank += own[eo + j]; continue; }
                    const PI ph = part_info(p.S, h, t);
                    const uint32_t lh = KIND ? ph.nk : ph.nv, eh = eoff[t * G + h];
                    const uint32_t q = KIND ? lower_bound_f(lh, x, [&](uint32_t i) { return key_code(p.S, h, ph.kb + i); })
                                            : lower_bound_f(lh, x, [&](uint32_t i) { return (uint64_t)p.S.vals[h][ph.vb + i]; });
                    rank += q < lh ? own[eh + q] : lst[t * G + h];
                }
                rank_out[eo + j] = rank;
                const uint32_t nxt = j + 1 < len ? own[eo + j + 1] : lst[t * G + g];
                if (nxt != own[eo + j]) {
                    if (KIND == 0) p.out_vals[ob + rank] = (uint32_t)x;
                    else {
                        p.out_lo[ob + rank] = p.S.range ? (uint32_t)(x >> 32) : (uint32_t)x;
                        if (p.S.range) p.out_hi[ob + rank] = (uint32_t)x;
                    }
                }
            }
        }
    }
}

// body entries remapped into union-rank space
__global__ __launch_bounds__(DS_WAVES * 64) void un_body_remap_kernel(DsUnionParams p)
{
    const uint32_t lane = lane_id(), G = p.S.G;
    DS_TXN_LOOP(t, p.n) {
        for (uint32_t g = 0; g < G; ++g) {
            const PI pg = part_info(p.S, g, t);
            const uint32_t bo = p.beoff[t * G + g], vo = p.veoff[t * G + g];
            const int32_t *x = p.S.x[g] + pg.xb + pg.nk;
            for (uint32_t q = lane; q < pg.nx - pg.nk; q += 64) p.rb[bo + q] = p.vrank[vo + (uint32_t)x[q]];
        }
    }
}

struct BodyAcc {   // owner prefix B(g, i) over part g's flattened body, B(g, nb) = part total
    const uint32_t *bown, *btot;
    __device__ __forceinline__ uint32_t operator()(uint32_t bo, uint32_t nb, uint32_t tg, uint32_t i) const
    {
        return i < nb ? bown[bo + i] : btot[tg];
    }
};

// position of key `code` in part h's txn keys, or ~0
__device__ __forceinline__ uint32_t find_key(const DsSide &S, uint32_t h, const PI &ph, uint64_t code)
{
    const uint32_t q = lower_bound_f(ph.nk, code, [&](uint32_t i) { return key_code(S, h, ph.kb + i); });
    return q < ph.nk && key_code(S, h, ph.kb + q) == code ? q : ~0u;
}

__global__ __launch_bounds__(DS_WAVES * 64) void un_body_owner_kernel(DsUnionParams p)
{
    const uint32_t lane = lane_id(), G = p.S.G;
    DS_TXN_LOOP(t, p.n) {
        for (uint32_t g = 0; g < G; ++g) {
            const PI pg = part_info(p.S, g, t);
            const uint32_t nb = pg.nx - pg.nk, bo = p.beoff[t * G + g];
            const int32_t *x = p.S.x[g] + pg.xb;
            uint32_t carry = 0;
            for (uint32_t q0 = 0; q0 < nb; q0 += 64) {
                const uint32_t q = q0 + lane;
                const bool active = q < nb;
                bool owner = active;
                if (active && g > 0) {
                    const uint32_t a = key_of_body(x, pg.nk, q);
                    const uint64_t code = key_code(p.S, g, pg.kb + a);
                    const uint32_t r = p.rb[bo + q];
                    for (uint32_t h = 0; h < g && owner; ++h) {
                        const PI ph = part_info(p.S, h, t);
                        const uint32_t ah = find_key(p.S, h, ph, code);
                        if (ah == ~0u) continue;
                        const int32_t *xh = p.S.x[h] + ph.xb;
                        const uint32_t s = body_lo(xh, ph.nk, ah), e = (uint32_t)xh[ah] - ph.nk;
                        const uint32_t *seg = p.rb + p.beoff[t * G + h] + s;
                        const uint32_t w = lower_bound_f(e - s, r, [&](uint32_t i) { return (uint64_t)seg[i]; });
                        if (w < e - s && seg[w] == r) owner = false;
                    }
                }
                const uint64_t b = __ballot(owner);
                if (active) p.bown[bo + q] = carry + (uint32_t)__popcll(b & lanemask_lt());
                carry += (uint32_t)__popcll(b);
            }
            if (lane == 0) p.btot[t * G + g] = carry;
        }
    }
}

__global__ __launch_bounds__(DS_WAVES * 64) void un_body_sizes_kernel(DsUnionParams p)
{
    const uint32_t lane = lane_id(), G = p.S.G;
    const BodyAcc B{p.bown, p.btot};
    DS_TXN_LOOP(t, p.n) {
        const uint32_t ub = p.out_key_off[t];
        for (uint32_t g = 0; g < G; ++g) {
            const PI pg = part_info(p.S, g, t);
            const uint32_t nb = pg.nx - pg.nk, bo = p.beoff[t * G + g], ko = p.keoff[t * G + g];
            const int32_t *x = p.S.x[g] + pg.xb;
            for (uint32_t a = lane; a < pg.nk; a += 64) {
                const uint32_t s = body_lo(x, pg.nk, a), e = (uint32_t)x[a] - pg.nk;
                const uint32_t c = B(bo, nb, t * G + g, e) - B(bo, nb, t * G + g, s);
                if (c) atomicAdd(&p.bsz[ub + p.krank[ko + a]], c);
            }
        }
    }
}

__global__ __launch_bounds__(DS_WAVES * 64) void un_write_body_kernel(DsUnionParams p)
{
    const uint32_t lane = lane_id(), G = p.S.G;
    const BodyAcc B{p.bown, p.btot};
    DS_TXN_LOOP(t, p.n) {
        const uint32_t ub = p.out_key_off[t], nku = p.out_key_off[t + 1] - ub;
        const uint32_t bbase = p.bscan[ub], xo = ub + bbase;
        if (lane == 0) {
            p.out_x_off[t] = xo;
            if (t + 1 == p.n) p.out_x_off[p.n] = p.out_key_off[p.n] + p.bscan[p.out_key_off[p.n]];
        }
        for (uint32_t u = lane; u < nku; u += 64) p.out_x[xo + u] = (int32_t)(nku + (p.bscan[ub + u + 1] - bbase));
        for (uint32_t g = 0; g < G; ++g) {
            const PI pg = part_info(p.S, g, t);
            const uint32_t nb = pg.nx - pg.nk, bo = p.beoff[t * G + g], ko = p.keoff[t * G + g], tg = t * G + g;
            const int32_t *x = p.S.x[g] + pg.xb;
            for (uint32_t q = lane; q < nb; q += 64) {
                if (B(bo, nb, tg, q + 1) == B(bo, nb, tg, q)) continue;   // not the owner
                const uint32_t a = key_of_body(x, pg.nk, q);
                const uint64_t code = key_code(p.S, g, pg.kb + a);
                const uint32_t r = p.rb[bo + q], u = p.krank[ko + a];
                uint32_t rank = B(bo, nb, tg, q) - B(bo, nb, tg, body_lo(x, pg.nk, a));
                for (uint32_t h = 0; h < G; ++h) {
                    if (h == g) continue;
                    const PI ph = part_info(p.S, h, t);
                    const uint32_t ah = find_key(p.S, h, ph, code);
                    if (ah == ~0u) continue;
                    const int32_t *xh = p.S.x[h] + ph.xb;
                    const uint32_t s = body_lo(xh, ph.nk, ah), e = (uint32_t)xh[ah] - ph.nk;
                    const uint32_t bh = p.beoff[t * G + h], nbh = ph.nx - ph.nk;
                    const uint32_t *seg = p.rb + bh + s;
                    const uint32_t w = lower_bound_f(e - s, r, [&](uint32_t i) { return (uint64_t)seg[i]; });
                    rank += B(bh, nbh, t * G + h, s + w) - B(bh, nbh, t * G + h, s);
                }
                p.out_x[xo + nku + (p.bscan[ub + u] - bbase) + rank] = (int32_t)r;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// slice
// ------------------------------------------------------------------------------------------

// select ranges of txn t
struct Sel {
    const uint32_t *s, *e;
    uint32_t n;
};
__device__ __forceinline__ Sel sel_of(const DsSliceParams &p, uint32_t t)
{
    if (!p.sel_off) return Sel{p.sel_start, p.sel_end, p.nsel};
    const uint32_t a = p.sel_off[t];
    return Sel{p.sel_start + a, p.sel_end + a, p.sel_off[t + 1] - a};
}

// Per txn: selected flags per key, mode (0 empty result, 1 input unchanged, 2 trimmed), counts of
// keys and keysToTxnIds, and the txnIds referenced by the selected keys marked in `used`.
template <bool RANGE>
__global__ __launch_bounds__(DS_WAVES * 64) void sl_select_kernel(DsSliceParams p)
{
    const uint32_t lane = lane_id();
    const DsSide &S = p.S;
    DS_TXN_LOOP(t, p.n) {
        const PI pi = part_info(S, 0, t);
        const Sel q = sel_of(p, t);
        const int32_t *x = S.x[0] + pi.xb;
        uint32_t m = 0, nb = 0;
        if (pi.nx != pi.nk) {   // isEmpty() returns the input unchanged (KeyDeps.java:191, RangeDeps.java:547)
            if (!RANGE) {
                // Keys.slice: keys inside some (s, e] select range (sorted, de-overlapped)
                for (uint32_t a = lane; a < pi.nk; a += 64) {
                    const uint32_t key = S.lo[0][pi.kb + a];
                    const uint32_t r = lower_bound_f(q.n, key, [&](uint32_t i) { return (uint64_t)q.e[i]; });
                    const bool sel = r < q.n && q.s[r] < key;
                    p.ksel[pi.kb + a] = sel ? 1u : 0u;
                    m += sel ? 1u : 0u;
                    nb += sel ? (uint32_t)x[a] - (a == 0 ? pi.nk : (uint32_t)x[a - 1]) : 0u;
                }
            } else {
                // RangeDeps.forEach(Ranges) through the collector (see the oracle's
                // rangedeps_slice_one): per select range a run [start, end) and buffered matches in
                // [minIndex, floor) ending after qs, flushed only by a later non-empty run.
                const uint32_t *rs = S.lo[0] + pi.kb, *re = S.hi[0] + pi.kb;
                const uint32_t nr = pi.nk;
                int last_run = -1;
                {
                    uint32_t minIndex = 0;
                    for (uint32_t k = 0; k < q.n; ++k) {
                        if (minIndex == nr) break;
                        const uint32_t qs = q.s[k], qe = q.e[k];
                        const uint32_t end = minIndex + lower_bound_f(nr - minIndex, qe, [&](uint32_t i) { return (uint64_t)rs[minIndex + i]; });
                        if (end <= minIndex) continue;
                        const uint32_t ins = minIndex + lower_bound_f(nr - minIndex, qs, [&](uint32_t i) { return (uint64_t)rs[minIndex + i]; });
                        int64_t start;
                        if (ins < nr && rs[ins] == qs) start = ins;
                        else {
                            start = (int64_t)ins - 1;
                            if (start < 0) start = 0;
                            else if (re[start] <= qs) ++start;
                        }
                        if (start < (int64_t)minIndex) start = minIndex;
                        if ((uint32_t)start != end) last_run = (int)k;
                        minIndex = end;
                    }
                }
                for (uint32_t c0 = 0; c0 < nr; c0 += 64 * 32) {
                    uint32_t mask = 0, minIndex = 0;
                    for (uint32_t k = 0; k < q.n && (int)k <= last_run; ++k) {
                        if (minIndex == nr) break;
                        const uint32_t qs = q.s[k], qe = q.e[k];
                        const uint32_t end = minIndex + lower_bound_f(nr - minIndex, qe, [&](uint32_t i) { return (uint64_t)rs[minIndex + i]; });
                        if (end <= minIndex) continue;
                        const uint32_t ins = minIndex + lower_bound_f(nr - minIndex, qs, [&](uint32_t i) { return (uint64_t)rs[minIndex + i]; });
                        int64_t floor, start;
                        if (ins < nr && rs[ins] == qs) floor = start = ins;
                        else {
                            floor = start = (int64_t)ins - 1;
                            if (start < 0) floor = start = 0;
                            else if (re[start] <= qs) ++start;
                        }
                        if (start < (int64_t)minIndex) start = minIndex;
#pragma unroll 4
                        for (uint32_t j = 0; j < 32; ++j) {
                            const uint32_t r = c0 + j * 64 + lane;
                            if (r >= nr) break;
                            const bool in_run = (int64_t)r >= start && r < end;
                            const bool in_buf = r >= minIndex && (int64_t)r < floor && re[r] > qs;   // flushed: k <= last_run
                            if (in_run || in_buf) mask |= 1u << j;
                        }
                        minIndex = end;
                    }
                    for (uint32_t j = 0; j < 32; ++j) {
                        const uint32_t r = c0 + j * 64 + lane;
                        if (r >= nr) break;
                        const bool sel = (mask >> j) & 1u;
                        p.ksel[pi.kb + r] = sel ? 1u : 0u;
                        m += sel ? 1u : 0u;
                        nb += sel ? (uint32_t)x[r] - (r == 0 ? nr : (uint32_t)x[r - 1]) : 0u;
                    }
                }
            }
        }
        m = wave_sum(m);
        nb = wave_sum(nb);
        const uint32_t mode = (pi.nx == pi.nk || m == pi.nk) ? 1u : m == 0 ? 0u : 2u;
        if (lane == 0) {
            p.mode[t] = mode;
            p.cnt_keys[t] = mode == 1 ? pi.nk : mode == 0 ? 0u : m;
            p.cnt_x[t] = mode == 1 ? pi.nx : mode == 0 ? 0u : m + nb;
        }
    }
}

// mark the txnIds the selected lists reference (trimUnusedValues, RelationMultiMap.java:497-503)
__global__ __launch_bounds__(DS_WAVES * 64) void sl_mark_kernel(DsSliceParams p)
{
    const uint32_t lane = lane_id();
    DS_TXN_LOOP(t, p.n) {
        if (p.mode[t] != 2) continue;
        const PI pi = part_info(p.S, 0, t);
        const int32_t *x = p.S.x[0] + pi.xb;
        for (uint32_t a = 0; a < pi.nk; ++a) {
            if (!p.ksel[pi.kb + a]) continue;
            const uint32_t s = a == 0 ? pi.nk : (uint32_t)x[a - 1], e = (uint32_t)x[a];
            for (uint32_t y = s + lane; y < e; y += 64) p.used[pi.vb + (uint32_t)x[y]] = 1u;
        }
    }
}

__global__ __launch_bounds__(DS_WAVES * 64) void sl_count_vals_kernel(DsSliceParams p)
{
    const uint32_t lane = lane_id();
    DS_TXN_LOOP(t, p.n) {
        const PI pi = part_info(p.S, 0, t);
        const uint32_t mode = p.mode[t];
        uint32_t c = 0;
        if (mode == 2)
            for (uint32_t v = lane; v < pi.nv; v += 64) c += p.used[pi.vb + v];
        c = wave_sum(c);
        if (lane == 0) p.cnt_vals[t] = mode == 1 ? pi.nv : mode == 0 ? 0u : c;
    }
}

// txnIds (kept ones, in order) + the remap of every kept txnId; keys of the result
__global__ __launch_bounds__(DS_WAVES * 64) void sl_write_vals_kernel(DsSliceParams p)
{
    const uint32_t lane = lane_id();
    DS_TXN_LOOP(t, p.n) {
        const PI pi = part_info(p.S, 0, t);
        const uint32_t mode = p.mode[t];
        if (mode == 0) continue;
        const uint32_t ov = p.out_val_off[t], ok = p.out_key_off[t];
        const uint32_t *vals = p.S.vals[0] + pi.vb;
        uint32_t carry = 0;
        for (uint32_t v0 = 0; v0 < pi.nv; v0 += 64) {
            const uint32_t v = v0 + lane;
            const bool keep = v < pi.nv && (mode == 1 || p.used[pi.vb + v]);
            const uint64_t b = __ballot(keep);
            const uint32_t r = carry + (uint32_t)__popcll(b & lanemask_lt());
            if (keep) { p.out_vals[ov + r] = vals[v]; p.remap[pi.vb + v] = r; }
            carry += (uint32_t)__popcll(b);
        }
        carry = 0;
        for (uint32_t a0 = 0; a0 < pi.nk; a0 += 64) {
            const uint32_t a = a0 + lane;
            const bool keep = a < pi.nk && (mode == 1 || p.ksel[pi.kb + a]);
            const uint64_t b = __ballot(keep);
            const uint32_t r = carry + (uint32_t)__popcll(b & lanemask_lt());
            if (keep) {
                p.out_lo[ok + r] = p.S.lo[0][pi.kb + a];
                if (p.S.range) p.out_hi[ok + r] = p.S.hi[0][pi.kb + a];
            }
            carry += (uint32_t)__popcll(b);
        }
    }
}

// keysToTxnIds of the result: headers + the selected lists with remapped txnIds
__global__ __launch_bounds__(DS_WAVES * 64) void sl_write_body_kernel(DsSliceParams p)
{
    const uint32_t lane = lane_id();
    DS_TXN_LOOP(t, p.n) {
        const PI pi = part_info(p.S, 0, t);
        const uint32_t mode = p.mode[t];
        if (mode == 0) continue;
        const uint32_t ox = p.out_x_off[t], m = p.out_key_off[t + 1] - p.out_key_off[t];
        const int32_t *x = p.S.x[0] + pi.xb;
        if (mode == 1) {
            for (uint32_t y = lane; y < pi.nx; y += 64) p.out_x[ox + y] = x[y];
            continue;
        }
        uint32_t j = 0, o = m;   // selected key index, body write cursor (wave-uniform)
        for (uint32_t a0 = 0; a0 < pi.nk; a0 += 64) {
            const uint32_t a = a0 + lane;
            const bool keep = a < pi.nk && p.ksel[pi.kb + a];
            const uint32_t len = keep ? (uint32_t)x[a] - (a == 0 ? pi.nk : (uint32_t)x[a - 1]) : 0u;
            const uint32_t incl = wave_incl_scan(len);
            const uint64_t b = __ballot(keep);
            if (keep) p.out_x[ox + j + (uint32_t)__popcll(b & lanemask_lt())] = (int32_t)(o + incl);
            o += readlane(incl, 63);
            j += (uint32_t)__popcll(b);
        }
        // bodies: walk the selected keys in order, lanes over each list
        uint32_t w = m;
        for (uint32_t a = 0; a < pi.nk; ++a) {
            if (!p.ksel[pi.kb + a]) continue;
            const uint32_t s = a == 0 ? pi.nk : (uint32_t)x[a - 1], e = (uint32_t)x[a];
            for (uint32_t y = s + lane; y < e; y += 64) p.out_x[ox + w + (y - s)] = (int32_t)p.remap[pi.vb + (uint32_t)x[y]];
            w += e - s;
        }
    }
}

// ------------------------------------------------------------------------------------------
// invert
// ------------------------------------------------------------------------------------------

// per txn the inverse's size: |txnIds| header + one entry per body element (scanned into out_off)
__global__ __launch_bounds__(256) void inv_sizes_kernel(DsInvertParams p)
{
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < p.n; t += gridDim.x * blockDim.x) {
        const PI pi = part_info(p.S, 0, t);
        p.sizes[t] = pi.nv + pi.nx - pi.nk;
    }
}

// first pass of invert (:912-914): per txnId the number of keys listing it, in the header slots
__global__ __launch_bounds__(DS_WAVES * 64) void inv_count_kernel(DsInvertParams p)
{
    const uint32_t lane = lane_id();
    DS_TXN_LOOP(t, p.n) {
        const PI pi = part_info(p.S, 0, t);
        const int32_t *x = p.S.x[0] + pi.xb;
        const uint32_t o = p.out_off[t];
        for (uint32_t y = pi.nk + lane; y < pi.nx; y += 64) atomicAdd((uint32_t *)&p.out[o + (uint32_t)x[y]], 1u);
    }
}

// offsets (:916-923): header v = |txnIds| + inclusive count, cursor v = |txnIds| + exclusive
__global__ __launch_bounds__(DS_WAVES * 64) void inv_scan_kernel(DsInvertParams p)
{
    const uint32_t lane = lane_id();
    DS_TXN_LOOP(t, p.n) {
        const PI pi = part_info(p.S, 0, t);
        const uint32_t o = p.out_off[t];
        uint32_t carry = pi.nv;
        for (uint32_t v0 = 0; v0 < pi.nv; v0 += 64) {
            const uint32_t v = v0 + lane;
            const uint32_t c = v < pi.nv ? (uint32_t)p.out[o + v] : 0u;
            const uint32_t incl = wave_incl_scan(c);
            if (v < pi.nv) { p.cursor[pi.vb + v] = carry + incl - c; p.out[o + v] = (int32_t)(carry + incl); }
            carry += readlane(incl, 63);
        }
    }
}

// placement (:926-935): keys in ascending order; a key lists each txnId once, so the lanes of one
// key never share a cursor and the returned cursor orders the keys of every txnId
__global__ __launch_bounds__(DS_WAVES * 64) void inv_place_kernel(DsInvertParams p)
{
    const uint32_t lane = lane_id();
    DS_TXN_LOOP(t, p.n) {
        const PI pi = part_info(p.S, 0, t);
        const int32_t *x = p.S.x[0] + pi.xb;
        const uint32_t o = p.out_off[t];
        for (uint32_t a = 0; a < pi.nk; ++a) {
            const uint32_t s = a == 0 ? pi.nk : (uint32_t)x[a - 1], e = (uint32_t)x[a];
            for (uint32_t y = s + lane; y < e; y += 64) {
                const uint32_t pos = atomicAdd(&p.cursor[pi.vb + (uint32_t)x[y]], 1u);
                p.out[o + pos] = (int32_t)a;
            }
        }
    }
}

uint32_t wave_blocks(uint32_t n)
{
    uint32_t b = (n + DS_WAVES - 1) / DS_WAVES;
    if (b > 16384) b = 16384;
    return b ? b : 1;
}
uint32_t flat_blocks(uint64_t n)
{
    uint64_t b = (n + 255) / 256;
    if (b > 16384) b = 16384;
    return b ? (uint32_t)b : 1;
}

} // namespace

void launch_union_lens(const DsUnionParams &p, hipStream_t s)
{
    if (p.n) hipLaunchKernelGGL(un_lens_kernel, dim3(flat_blocks((uint64_t)p.n * p.S.G)), dim3(256), 0, s, p);
}
void launch_union_owners(const DsUnionParams &p, hipStream_t s)
{
    if (!p.n) return;
    hipLaunchKernelGGL(un_owner_kernel<0>, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL(un_owner_kernel<1>, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
}
void launch_union_ranks(const DsUnionParams &p, hipStream_t s)
{
    if (!p.n) return;
    hipLaunchKernelGGL(un_rank_kernel<0>, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL(un_rank_kernel<1>, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL(un_body_remap_kernel, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL(un_body_owner_kernel, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL(un_body_sizes_kernel, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
}
void launch_union_write(const DsUnionParams &p, hipStream_t s)
{
    if (p.n) hipLaunchKernelGGL(un_write_body_kernel, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
}

void launch_slice_select(const DsSliceParams &p, hipStream_t s)
{
    if (!p.n) return;
    if (p.S.range) hipLaunchKernelGGL(sl_select_kernel<true>, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
    else hipLaunchKernelGGL(sl_select_kernel<false>, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL(sl_mark_kernel, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL(sl_count_vals_kernel, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
}
void launch_slice_write(const DsSliceParams &p, hipStream_t s)
{
    if (!p.n) return;
    hipLaunchKernelGGL(sl_write_vals_kernel, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL(sl_write_body_kernel, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
}

void launch_invert_sizes(const DsInvertParams &p, hipStream_t s)
{
    if (p.n) hipLaunchKernelGGL(inv_sizes_kernel, dim3(flat_blocks(p.n)), dim3(256), 0, s, p);
}

void launch_invert(const DsInvertParams &p, hipStream_t s)
{
    if (!p.n) return;
    hipLaunchKernelGGL(inv_count_kernel, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL(inv_scan_kernel, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
    hipLaunchKernelGGL(inv_place_kernel, dim3(wave_blocks(p.n)), dim3(DS_WAVES * 64), 0, s, p);
}

} // namespace accord
