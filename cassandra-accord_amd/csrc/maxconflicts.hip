// MaxConflicts fold on the device: the executeAt-proposal input of
// CommandStore.preaccept (local/CommandStore.java:320-349) for a batch of key txns in TxnId order.
//
//   minNonConflicting[t] = MaxConflicts.get(keys_t)            (local/MaxConflicts.java:46-49)
//                        = foldl(keys_t, Timestamp::max, NONE) over the keys that hold an entry
//   fast[t]              = txnId_t.compareTo(minNonConflicting[t]) >= 0    (:345, epoch excluded)
//   then, for globally visible kinds, MaxConflicts.update(keys_t, executeAt_t)
//                        (local/SafeCommandStore.java:192-210, local/CommandStore.java:280-289)
//
// The sequential map updates become one segmented scan: the (key, pair) list is radix-sorted by key
// (stable, so each key's pairs stay in stream order) and every pair gets the exclusive prefix of
// its key segment under the operator "later wins only if strictly greater" (Timestamp.max(old, new)
// inside ReducingIntervalMap.merge keeps the old value on ties), seeded with the store's current
// per-key value.  A per-txn pass then folds its pairs in key order with ">=" (foldl applies
// Timestamp.max(value, acc), so a tie takes the later key's value).  The per-key map is a dense
// array over the store's key ordinals, resident in HBM between batches (CommandStore.maxConflicts).
//
// Bytes per pair: key ordinal 4 + sort (≈3 passes × 16) + scan read 4+4+24 + prefix write 24 +
// fold read 24 ≈ 130 B; HBM-bound integer work, no MFMA.
#include "store_impl.h"

#include <algorithm>
#include <vector>

namespace {

struct TsV {                 // one MaxConflicts value: Timestamp bits + "entry present"
    uint64_t msb, lsb;
    int32_t node;
    uint32_t has;
};

constexpr uint32_t MC_TILE = 1024;   // one element per thread, 16 waves
constexpr uint32_t MC_INVISIBLE = 0x80000000u;   // sorted txn value: the txn is not globally visible
constexpr uint32_t MC_TXN = 0x7FFFFFFFu;
constexpr uint32_t MC_CARRY_THREADS = 1024;

__device__ __forceinline__ int tcmp(const TsV &a, const TsV &b)
{
    return ts_cmp(a.msb, a.lsb, a.node, b.msb, b.lsb, b.node);
}
// a earlier, b later: the merge's Timestamp.max(old, new) keeps old unless new is strictly greater
__device__ __forceinline__ TsV max_keep_old(const TsV &a, const TsV &b)
{
    if (!b.has) return a;
    if (!a.has) return b;
    return tcmp(b, a) > 0 ? b : a;
}

struct Comp {                // segmented-scan composite: head seen in the span, value of the open segment
    TsV v;
    uint32_t head;
};
__device__ __forceinline__ Comp comp(const Comp &a, const Comp &b)
{
    if (b.head) return b;
    Comp r;
    r.v = max_keep_old(a.v, b.v);
    r.head = a.head;
    return r;
}

__device__ __forceinline__ void record_error(accord::DevStatus *st, uint32_t i, int32_t code)
{
    unsigned long long v = ((unsigned long long)i << 32) | (uint32_t)(-code);
    atomicMin(&st->first, v);
}

// Store keys a txn reads and writes: its keys (key domain) or the keys its ranges (s, e] cover,
// clipped to the store [key_lo, key_hi) -- MaxConflicts is a ReducingRangeMap over routing keys and
// an IntKey range has no points between keys, so a range is exactly the keys it covers
// (local/MaxConflicts.java:46-80; keys sliced to the store, local/CommandStore.java:318).
__device__ __forceinline__ uint32_t mc_range_keys(uint32_t rs, uint32_t re, uint32_t key_lo, uint32_t key_hi,
                                                  uint32_t &a)
{
    const uint64_t lo = max((uint64_t)rs + 1, (uint64_t)key_lo), hi = min((uint64_t)re + 1, (uint64_t)key_hi);
    a = (uint32_t)lo;
    return hi > lo ? (uint32_t)(hi - lo) : 0u;
}

// Per-txn pair counts over [first, last) (cnt[last - first] = 0 so the exclusive scan ends with the total).
__global__ void __launch_bounds__(256) mc_count_kernel(uint32_t first, uint32_t last, const uint64_t *__restrict__ lsb,
                                                       const uint32_t *__restrict__ key_off,
                                                       const uint32_t *__restrict__ rng_off,
                                                       const uint32_t *__restrict__ rng_start,
                                                       const uint32_t *__restrict__ rng_end, uint32_t key_lo,
                                                       uint32_t key_hi, uint32_t *__restrict__ cnt)
{
    const uint32_t t = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (t > last) return;
    uint32_t c = 0;
    if (t < last) {
        if (lsb[t] & 1) {
            for (uint32_t r = rng_off[t]; r < rng_off[t + 1]; ++r) {
                uint32_t a;
                c += mc_range_keys(rng_start[r], rng_end[r], key_lo, key_hi, a);
            }
        } else {
            c = key_off[t + 1] - key_off[t];
        }
    }
    cnt[t - first] = c;
}

// txn-major over txns [first, last): validate and pack (key, txn, pair) for the sort at the txn's
// pair offset po[t - first].  Key txns: keys sorted-unique inside the store.  Range txns: ranges
// non-empty, sorted, non-overlapping.  ExclusiveSyncPoint in the key domain is rejected:
// CommandStore.preaccept hands its keys to markExclusiveSyncPoint as Ranges (:335-339).
__global__ void __launch_bounds__(256) mc_pack_kernel(uint32_t first, uint32_t last, const uint64_t *__restrict__ lsb,
                                                      const uint32_t *__restrict__ key_off,
                                                      const uint32_t *__restrict__ key_ord,
                                                      const uint32_t *__restrict__ rng_off,
                                                      const uint32_t *__restrict__ rng_start,
                                                      const uint32_t *__restrict__ rng_end, uint32_t key_lo,
                                                      uint32_t key_hi, const uint32_t *__restrict__ po,
                                                      uint32_t *__restrict__ pk, uint32_t *__restrict__ pv,
                                                      uint32_t *__restrict__ pe, accord::DevStatus *st)
{
    const uint32_t t = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= last) return;
    const uint64_t l = lsb[t];
    const uint32_t kind = (uint32_t)(l >> 1) & 7, domain = (uint32_t)l & 1;
    if (kind >= 5 || (domain == 0 && kind == 4)) record_error(st, t, ACCORD_ERR_KIND);
    uint32_t o = po[t - first];
    const uint32_t inv = kind == 2u ? MC_INVISIBLE : 0u;   // EphemeralRead: merges nothing (elem_value)
    if (domain) {
        for (uint32_t r = rng_off[t]; r < rng_off[t + 1]; ++r) {
            const uint32_t rs = rng_start[r], re = rng_end[r];
            if (rs >= re || (r > rng_off[t] && rs < rng_end[r - 1])) record_error(st, t, ACCORD_ERR_KEYS);
            uint32_t a;
            const uint32_t c = mc_range_keys(rs, re, key_lo, key_hi, a);
            for (uint32_t j = 0; j < c; ++j, ++o) {
                pk[o] = a + j - key_lo;
                pv[o] = t | inv;
                pe[o] = o;
            }
        }
        return;
    }
    const uint32_t b = key_off[t], e = key_off[t + 1];
    uint32_t prev = 0;
    for (uint32_t p = b; p < e; ++p, ++o) {
        const uint32_t k = key_ord[p];
        if (k < key_lo || k >= key_hi || (p > b && k <= prev)) record_error(st, t, ACCORD_ERR_KEYS);
        pk[o] = (k >= key_lo && k < key_hi) ? k - key_lo : 0;
        pv[o] = t | inv;
        pe[o] = o;
        prev = k;
    }
}

// The executeAt a txn merges: the caller's value for txn ov_t (the continuation point of
// accord_max_conflicts_fold_from), else the batch's exec_* (Accept batch) or the TxnId.
struct McValues {
    const uint64_t *vm, *vl;
    const int32_t *vn;
    uint32_t ov_t;
    uint64_t ov_msb, ov_lsb;
    int32_t ov_node;
};

__device__ __forceinline__ TsV elem_value(uint32_t t, const uint64_t *lsb, const McValues &mv)
{
    TsV v;
    const uint32_t kind = (uint32_t)(lsb[t] >> 1) & 7;
    v.has = kind != 2u;          // EphemeralRead is not globally visible (LocalOnly rejected)
    if (t == mv.ov_t) { v.msb = mv.ov_msb; v.lsb = mv.ov_lsb; v.node = mv.ov_node; }
    else { v.msb = mv.vm[t]; v.lsb = mv.vl[t]; v.node = mv.vn[t]; }
    return v;
}

// Tile-local segmented inclusive scan in LDS.  mode 0: write the tile composite.  mode 1: apply the
// tile's carry, write each pair's exclusive prefix (pair order) and each segment's final value.
template <int MODE>
__global__ void __launch_bounds__(MC_TILE) mc_scan_kernel(
    uint32_t P, const uint32_t *__restrict__ sk, const uint32_t *__restrict__ sv, const uint32_t *__restrict__ se,
    TsV *__restrict__ svals,
    const uint64_t *__restrict__ lsb, McValues mv, const TsV *__restrict__ state, Comp *__restrict__ tile_comp,
    const TsV *__restrict__ carry, TsV *__restrict__ prefix, TsV *__restrict__ state_out)
{
    __shared__ Comp buf[MC_TILE];
    const uint32_t q = blockIdx.x * MC_TILE + threadIdx.x;
    const bool live = q < P;
    Comp c;
    c.head = 0;
    c.v.has = 0; c.v.msb = 0; c.v.lsb = 0; c.v.node = 0;
    uint32_t key = 0;
    TsV seed;
    seed.has = 0; seed.msb = 0; seed.lsb = 0; seed.node = 0;
    if (live) {
        key = sk[q];
        // mode 0 gathers the txn's value once and leaves it in sorted order for mode 1
        TsV v;
        if (MODE == 0) { v = elem_value(sv[q] & MC_TXN, lsb, mv); svals[q] = v; }
        else v = svals[q];
        c.head = (q == 0 || sk[q - 1] != key) ? 1u : 0u;
        if (c.head) {
            seed = state[key];
            v = max_keep_old(seed, v);
        }
        c.v = v;
    }
    buf[threadIdx.x] = c;
    __syncthreads();
    for (uint32_t off = 1; off < MC_TILE; off <<= 1) {
        Comp x = c;
        if (threadIdx.x >= off) x = comp(buf[threadIdx.x - off], c);
        __syncthreads();
        buf[threadIdx.x] = x;
        c = x;
        __syncthreads();
    }
    if (MODE == 0) {
        if (threadIdx.x == MC_TILE - 1) tile_comp[blockIdx.x] = c;
        return;
    }
    if (!live) return;
    const TsV cin = carry[blockIdx.x];
    const TsV incl = c.head ? c.v : max_keep_old(cin, c.v);
    TsV excl;
    bool own_head = q == 0 || sk[q - 1] != key;
    if (own_head) excl = seed;
    else if (threadIdx.x == 0) excl = cin;
    else {
        const Comp pc = buf[threadIdx.x - 1];
        excl = pc.head ? pc.v : max_keep_old(cin, pc.v);
    }
    prefix[se[q]] = excl;
    if (q + 1 == P || sk[q + 1] != key) state_out[key] = incl;
}

// Exclusive scan of the tile composites (one block): carry[t] = value open at the start of tile t
__global__ void __launch_bounds__(MC_CARRY_THREADS) mc_carry_kernel(uint32_t ntiles, const Comp *__restrict__ tc,
                                                                    TsV *__restrict__ carry)
{
    __shared__ Comp buf[MC_CARRY_THREADS];
    const uint32_t per = (ntiles + MC_CARRY_THREADS - 1) / MC_CARRY_THREADS;
    const uint32_t b = min(ntiles, threadIdx.x * per), e = min(ntiles, b + per);
    Comp c;
    c.head = 0; c.v.has = 0; c.v.msb = 0; c.v.lsb = 0; c.v.node = 0;
    for (uint32_t i = b; i < e; ++i) c = comp(c, tc[i]);
    buf[threadIdx.x] = c;
    __syncthreads();
    for (uint32_t off = 1; off < MC_CARRY_THREADS; off <<= 1) {
        Comp x = c;
        if (threadIdx.x >= off) x = comp(buf[threadIdx.x - off], c);
        __syncthreads();
        buf[threadIdx.x] = x;
        c = x;
        __syncthreads();
    }
    Comp run;
    if (threadIdx.x == 0) { run.head = 0; run.v.has = 0; run.v.msb = 0; run.v.lsb = 0; run.v.node = 0; }
    else run = buf[threadIdx.x - 1];
    for (uint32_t i = b; i < e; ++i) {
        carry[i] = run.v;
        run = comp(run, tc[i]);
    }
}

// txn-major fold of the pairs' prefixes in key order: foldl(keys, Timestamp::max(value, acc), NONE).
// *stop = the first globally visible txn that takes the slow path with no executeAt known here: its
// executeAt is time.uniqueNow(minNonConflicting) (local/CommandStore.java:348), chosen by the caller,
// so neither it nor any later txn of the batch may be merged before the caller supplies it.  A
// range-domain ExclusiveSyncPoint returns txnId without reading the map (:335-339): NONE, fast.
__global__ void __launch_bounds__(256) mc_fold_kernel(uint32_t first, uint32_t last, const uint64_t *__restrict__ msb,
                                                      const uint64_t *__restrict__ lsb, const int32_t *__restrict__ node,
                                                      const uint32_t *__restrict__ po, const TsV *__restrict__ prefix,
                                                      uint64_t *__restrict__ om, uint64_t *__restrict__ ol,
                                                      int32_t *__restrict__ on, uint8_t *__restrict__ ohas,
                                                      uint8_t *__restrict__ ofast, uint32_t known_exec, uint32_t ov_t,
                                                      uint32_t *__restrict__ stop)
{
    const uint32_t t = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= last) return;
    const uint32_t kind = (uint32_t)(lsb[t] >> 1) & 7;
    const bool xsp = (lsb[t] & 1) && kind == 4;
    TsV acc;
    acc.has = 0; acc.msb = 0; acc.lsb = 0; acc.node = 0;
    if (!xsp)
        for (uint32_t p = po[t - first]; p < po[t - first + 1]; ++p) {
            const TsV x = prefix[p];
            if (x.has && (!acc.has || tcmp(x, acc) >= 0)) acc = x;
        }
    om[t] = acc.msb; ol[t] = acc.lsb; on[t] = acc.node; ohas[t] = (uint8_t)acc.has;
    const bool fast = xsp || ts_cmp(msb[t], lsb[t], node[t], acc.msb, acc.lsb, acc.node) >= 0;
    ofast[t] = (uint8_t)fast;
    if (!fast && !known_exec && t != ov_t && kind != 2u) atomicMin(stop, t);
}

// ---- PreAccept batches: monotone values ----
// Without exec_* every merged value is the txn's TxnId (the batch is strictly ascending) except the
// pass's first txn when the caller supplied its executeAt (accord_max_conflicts_fold_from): that txn
// is the head of every key segment it touches (stable sort, first in stream order).  The fold over a
// segment prefix [seed, v_f?, v_1 < v_2 < ...] is then max_keep_old(max_keep_old(seed, v_f), v_last):
// only the LAST visible txn before the pair matters, which a plain u32 max-scan of sorted positions
// finds.  Each pair gets a 4-byte code -- that txn (or none) and whether the override txn precedes it
// -- and the fold gathers the timestamps, instead of the general path's 24-byte prefix per pair.
constexpr uint32_t MM_THREADS = 256, MM_ITEMS = 4, MM_TILE = MM_THREADS * MM_ITEMS;
constexpr uint32_t MM_NONE = 0x7FFFFFFFu, MM_F = 0x80000000u;

// every txn's merged value once, 32-byte aligned: one sector per gather in the apply / fold passes
struct alignas(32) TsV32 {
    TsV v;
    uint64_t pad;
};
__global__ void __launch_bounds__(256) mm_values_kernel(uint32_t first, uint32_t last, const uint64_t *__restrict__ lsb,
                                                        McValues mv, TsV32 *__restrict__ vt)
{
    const uint32_t t = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (t < last) vt[t].v = elem_value(t, lsb, mv);
}

// segment starts + per tile the largest (sorted position + 1) of a visible non-override pair
__global__ void __launch_bounds__(MM_THREADS) mm_tile_kernel(uint32_t P, const uint32_t *__restrict__ sk,
                                                             const uint32_t *__restrict__ sv, uint32_t ov_t,
                                                             uint32_t *__restrict__ segstart,
                                                             uint32_t *__restrict__ tile_max)
{
    __shared__ uint32_t wm[MM_THREADS / 64];
    const uint32_t q0 = blockIdx.x * MM_TILE + threadIdx.x * MM_ITEMS;
    uint32_t m = 0;
#pragma unroll
    for (uint32_t j = 0; j < MM_ITEMS; ++j) {
        const uint32_t q = q0 + j;
        if (q >= P) break;
        const uint32_t k = sk[q], t = sv[q];
        if (q == 0 || sk[q - 1] != k) segstart[k] = q;
        if (t != ov_t && !(t & MC_INVISIBLE)) m = q + 1;
    }
    m = wave_incl_max(m);
    if (lane_id() == 63) wm[wave_id()] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t x = 0;
        for (uint32_t w = 0; w < MM_THREADS / 64; ++w) x = max(x, wm[w]);
        tile_max[blockIdx.x] = x;
    }
}

// exclusive max-scan of the tile maxima (one block)
__global__ void __launch_bounds__(256) mm_carry_kernel(uint32_t ntiles, uint32_t *__restrict__ tile_max)
{
    __shared__ uint32_t wm[4];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < ntiles; base += 256) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < ntiles ? tile_max[i] : 0u;
        const uint32_t incl = wave_incl_max(v);
        if (lane_id() == 63) wm[wave_id()] = incl;
        __syncthreads();
        uint32_t ex = __shfl_up(incl, 1, 64);
        if (lane_id() == 0) ex = 0;
        uint32_t blk = 0;
        for (uint32_t w = 0; w < 4; ++w) {
            if (w < wave_id()) ex = max(ex, wm[w]);
            blk = max(blk, wm[w]);
        }
        if (i < ntiles) tile_max[i] = max(carry, ex);
        carry = max(carry, blk);
        __syncthreads();
    }
}


// per pair (sorted order): its code at its pair index; per segment end: the key's new map value
__global__ void __launch_bounds__(MM_THREADS) mm_apply_kernel(uint32_t P, const uint32_t *__restrict__ sk,
                                                              const uint32_t *__restrict__ sv,
                                                              const uint32_t *__restrict__ se,
                                                              const TsV32 *__restrict__ vt, uint32_t ov_t,
                                                              const uint32_t *__restrict__ segstart,
                                                              const uint32_t *__restrict__ carry,
                                                              const TsV *__restrict__ state,
                                                              uint32_t *__restrict__ code, TsV *__restrict__ state_out)
{
    __shared__ uint32_t wm[MM_THREADS / 64];
    const uint32_t q0 = blockIdx.x * MM_TILE + threadIdx.x * MM_ITEMS;
    uint32_t v[MM_ITEMS], k[MM_ITEMS], t[MM_ITEMS];
    uint32_t m = 0;
#pragma unroll
    for (uint32_t j = 0; j < MM_ITEMS; ++j) {
        const uint32_t q = q0 + j;
        v[j] = 0; k[j] = 0; t[j] = 0;
        if (q < P) {
            k[j] = sk[q]; t[j] = sv[q];
            if (t[j] != ov_t && !(t[j] & MC_INVISIBLE)) v[j] = q + 1;
        }
        m = max(m, v[j]);
    }
    const uint32_t incl = wave_incl_max(m);
    if (lane_id() == 63) wm[wave_id()] = incl;
    __syncthreads();
    uint32_t run = __shfl_up(incl, 1, 64);
    if (lane_id() == 0) run = 0;
    for (uint32_t w = 0; w < wave_id(); ++w) run = max(run, wm[w]);
    run = max(run, carry[blockIdx.x]);
#pragma unroll
    for (uint32_t j = 0; j < MM_ITEMS; ++j) {
        const uint32_t q = q0 + j;
        if (q >= P) break;
        const uint32_t ss = segstart[k[j]];
        const bool f_head = ov_t != MC_TXN && (sv[ss] & MC_TXN) == ov_t;   // the override txn opens the segment
        const uint32_t last = run > ss ? sv[run - 1] & MC_TXN : MM_NONE;   // last visible pair before q in the segment
        code[se[q]] = last | ((f_head && q != ss) ? MM_F : 0u);
        run = max(run, v[j]);
        if (q + 1 == P || sk[q + 1] != k[j]) {                 // segment end: the key's map value
            TsV x = state[k[j]];
            if (f_head) x = max_keep_old(x, vt[ov_t].v);
            if (run > ss) x = max_keep_old(x, vt[sv[run - 1] & MC_TXN].v);
            state_out[k[j]] = x;
        }
    }
}

// txn-major fold: each pair's prefix value rebuilt from its code, then foldl(keys, max(value, acc))
__global__ void __launch_bounds__(256) mm_fold_kernel(uint32_t first, uint32_t last, const uint64_t *__restrict__ msb,
                                                      const uint64_t *__restrict__ lsb, const int32_t *__restrict__ node,
                                                      const TsV32 *__restrict__ vt, uint32_t ov_t,
                                                      const uint32_t *__restrict__ po,
                                                      const uint32_t *__restrict__ pk, const uint32_t *__restrict__ code,
                                                      const TsV *__restrict__ state, uint64_t *__restrict__ om,
                                                      uint64_t *__restrict__ ol, int32_t *__restrict__ on,
                                                      uint8_t *__restrict__ ohas, uint8_t *__restrict__ ofast,
                                                      uint32_t *__restrict__ stop)
{
    const uint32_t t = first + blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= last) return;
    const uint32_t kind = (uint32_t)(lsb[t] >> 1) & 7;
    const bool xsp = (lsb[t] & 1) && kind == 4;
    TsV acc;
    acc.has = 0; acc.msb = 0; acc.lsb = 0; acc.node = 0;
    if (!xsp) {
        // A pair's value is max_keep_old(y, v_c): y = the key's map value merged with the override
        // txn's, v_c = the TxnId of its last visible predecessor c.  TxnIds ascend with c, so the
        // largest v_c is that of the largest c: fold the y's (small, L2-resident map), take the max c,
        // and gather one TxnId per txn.  Only a y comparing equal to that TxnId needs the exact
        // per-pair order of the fold (ties keep the later key's value).
        const uint32_t p0 = po[t - first], p1 = po[t - first + 1];
        TsV Y;
        Y.has = 0; Y.msb = 0; Y.lsb = 0; Y.node = 0;
        uint32_t cmax = 0;                                  // 1 + largest c
        for (uint32_t p = p0; p < p1; ++p) {
            const uint32_t c = code[p];
            TsV y = state[pk[p]];
            if (c & MM_F) y = max_keep_old(y, vt[ov_t].v);
            if (y.has && (!Y.has || tcmp(y, Y) >= 0)) Y = y;
            if ((c & MM_NONE) != MM_NONE) cmax = max(cmax, (c & MM_NONE) + 1u);
        }
        acc = Y;
        if (cmax) {
            const TsV V = vt[cmax - 1].v;
            const int r = Y.has ? tcmp(V, Y) : 1;
            if (r > 0) acc = V;
            else if (r == 0) {                              // rare: replay the exact fold
                acc.has = 0;
                for (uint32_t p = p0; p < p1; ++p) {
                    const uint32_t c = code[p];
                    TsV x = state[pk[p]];
                    if (c & MM_F) x = max_keep_old(x, vt[ov_t].v);
                    if ((c & MM_NONE) != MM_NONE) x = max_keep_old(x, vt[c & MM_NONE].v);
                    if (x.has && (!acc.has || tcmp(x, acc) >= 0)) acc = x;
                }
            }
        }
    }
    om[t] = acc.msb; ol[t] = acc.lsb; on[t] = acc.node; ohas[t] = (uint8_t)acc.has;
    const bool fast = xsp || ts_cmp(msb[t], lsb[t], node[t], acc.msb, acc.lsb, acc.node) >= 0;
    ofast[t] = (uint8_t)fast;
    if (!fast && t != ov_t && kind != 2u) atomicMin(stop, t);
}

inline uint32_t bits_for_mc(uint32_t v)
{
    uint32_t b = 1;
    while (b < 32 && (v >> b)) ++b;
    return b;
}

} // namespace

// --------------------------------------------------------------------------------- C ABI

static int32_t mc_ensure_state(accord_store *s)
{
    const uint32_t nkeys = s->cfg.key_hi - s->cfg.key_lo;
    if (s->mc_state.p) return ACCORD_OK;
    HIPCHECK(s, s->mc_state.ensure((size_t)nkeys * sizeof(TsV)));
    HIPCHECK(s, s->mc_state2.ensure((size_t)nkeys * sizeof(TsV)));
    HIPCHECK(s, hipMemsetAsync(s->mc_state.p, 0, (size_t)nkeys * sizeof(TsV), s->stream));
    return ACCORD_OK;
}

extern "C" int32_t accord_max_conflicts_reset(accord_store *s)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    int32_t rc = mc_ensure_state(s);
    if (rc) return rc;
    HIPCHECK(s, hipMemsetAsync(s->mc_state.p, 0, (size_t)(s->cfg.key_hi - s->cfg.key_lo) * sizeof(TsV), s->stream));
    HIPCHECK(s, hipStreamSynchronize(s->stream));
    return ACCORD_OK;
}

namespace {

// Device buffers for a pass over P (txn, key) pairs.
int32_t mc_buffers(accord_store *s, uint32_t P)
{
    DevBuf *T = s->op_tmp;   // pk, pv(txn), sk, sv, tk, tv, pe(pair), prefix, tile comps, carry, radix temp, se, te, sorted values
    for (int b = 0; b < 7; ++b) HIPCHECK(s, T[b].ensure((size_t)P * 4 + 4));
    HIPCHECK(s, T[7].ensure((size_t)P * sizeof(TsV) + 32));
    const uint32_t ntiles = (P + MC_TILE - 1) / MC_TILE;
    HIPCHECK(s, T[8].ensure((size_t)ntiles * sizeof(Comp) + 64));
    HIPCHECK(s, T[9].ensure((size_t)ntiles * sizeof(TsV) + 32));
    HIPCHECK(s, T[10].ensure(accord::radix_sort_temp_bytes(P)));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(std::max(P, accord::radix_sort_scan_len(P))), s->stream));
    HIPCHECK(s, T[11].ensure((size_t)P * 4 + 4));                 // sorted pair index
    HIPCHECK(s, T[12].ensure((size_t)P * 4 + 4));                 // its ping-pong buffer
    HIPCHECK(s, T[13].ensure((size_t)P * sizeof(TsV) + 32));      // values in sorted order
    return ACCORD_OK;
}

// One fold pass over txns [first, last): pack, stable sort by key, segmented scan seeded by the
// store's map (written into mc_state2), and -- with outputs -- the per-txn fold and the stop index.
int32_t mc_pass(accord_store *s, uint32_t first, uint32_t last, const McValues &mv, bool outputs, uint32_t *stop_dev)
{
    const uint32_t nkeys = s->cfg.key_hi - s->cfg.key_lo;
    hipStream_t st = s->stream;
    DevBuf *T = s->op_tmp;
    HostTotals *dev = s->status_totals.as<HostTotals>();
    uint64_t *om = s->mc_out.as<uint64_t>(), *ol = om + s->n;
    int32_t *on = (int32_t *)(ol + s->n);
    uint8_t *ohas = (uint8_t *)(on + s->n), *ofast = ohas + s->n;
    const uint32_t nt = last - first;
    // pair offsets of [first, last): counts, exclusive scan (po[nt] = total), read the total
    uint32_t *po = s->mc_po.as<uint32_t>();
    mc_count_kernel<<<(nt + 1 + 255) / 256, 256, 0, st>>>(first, last, s->lsb.as<uint64_t>(), s->key_off.as<uint32_t>(),
                                                         s->rng_off.as<uint32_t>(), s->rng_start.as<uint32_t>(),
                                                         s->rng_end.as<uint32_t>(), s->cfg.key_lo, s->cfg.key_hi,
                                                         s->mc_cnt.as<uint32_t>());
    unsigned long long *tot = (unsigned long long *)&dev->totals[6];
    accord::exclusive_scan_u32(s->mc_cnt.as<uint32_t>(), po, nt + 1, tot, s->scan_tmp.p, st);
    unsigned long long Pt = 0;
    HIPCHECK(s, hipMemcpyAsync(&Pt, tot, 8, hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    if (Pt >= (1ull << 31)) return fail(s, ACCORD_ERR_CAPACITY, "MaxConflicts fold: %llu (txn, key) pairs", Pt);
    const uint32_t P = (uint32_t)Pt;
    int32_t rc = mc_buffers(s, P);
    if (rc) return rc;
    const uint32_t ntiles = (P + MC_TILE - 1) / MC_TILE;
    HIPCHECK(s, hipMemcpyAsync(s->mc_state2.p, s->mc_state.p, (size_t)nkeys * sizeof(TsV), hipMemcpyDeviceToDevice, st));
    if (nt)
        mc_pack_kernel<<<(nt + 255) / 256, 256, 0, st>>>(first, last, s->lsb.as<uint64_t>(), s->key_off.as<uint32_t>(),
                                                         s->key_ord.as<uint32_t>(), s->rng_off.as<uint32_t>(),
                                                         s->rng_start.as<uint32_t>(), s->rng_end.as<uint32_t>(),
                                                         s->cfg.key_lo, s->cfg.key_hi, po, T[0].as<uint32_t>(),
                                                         T[1].as<uint32_t>(), T[6].as<uint32_t>(), &dev->status);
    if (P) {
        accord::radix_sort_pairs(T[0].as<uint32_t>(), T[1].as<uint32_t>(), T[2].as<uint32_t>(), T[3].as<uint32_t>(),
                                 T[4].as<uint32_t>(), T[5].as<uint32_t>(), T[6].as<uint32_t>(), T[11].as<uint32_t>(),
                                 T[12].as<uint32_t>(), P, (int)bits_for_mc(nkeys ? nkeys - 1 : 0), T[10].p, s->scan_tmp.p, st);
        if (!s->has_exec) {          // PreAccept: monotone values, 4-byte codes (see mm_tile_kernel)
            const uint32_t mt = (P + MM_TILE - 1) / MM_TILE;
            HIPCHECK(s, T[14].ensure((size_t)nkeys * 4 + 4));
            HIPCHECK(s, T[15].ensure((size_t)mt * 4 + 4));
            HIPCHECK(s, T[16].ensure((size_t)s->n * sizeof(TsV32) + 64));
            TsV32 *vt = T[16].as<TsV32>();
            const uint32_t ovt = mv.ov_t == 0xFFFFFFFFu ? MC_TXN : mv.ov_t;
            mm_values_kernel<<<(nt + 255) / 256, 256, 0, st>>>(first, last, s->lsb.as<uint64_t>(), mv, vt);
            uint32_t *segstart = T[14].as<uint32_t>(), *tmax = T[15].as<uint32_t>();
            uint32_t *code = T[12].as<uint32_t>();            // the sort's ping-pong pair index: free now
            mm_tile_kernel<<<mt, MM_THREADS, 0, st>>>(P, T[2].as<uint32_t>(), T[3].as<uint32_t>(), ovt, segstart, tmax);
            mm_carry_kernel<<<1, 256, 0, st>>>(mt, tmax);
            mm_apply_kernel<<<mt, MM_THREADS, 0, st>>>(P, T[2].as<uint32_t>(), T[3].as<uint32_t>(), T[11].as<uint32_t>(),
                                                       vt, ovt, segstart, tmax, s->mc_state.as<TsV>(),
                                                       code, s->mc_state2.as<TsV>());
            if (outputs && nt)
                mm_fold_kernel<<<(nt + 255) / 256, 256, 0, st>>>(first, last, s->msb.as<uint64_t>(), s->lsb.as<uint64_t>(),
                                                                 s->node.as<int32_t>(), vt, ovt, po, T[0].as<uint32_t>(), code,
                                                                 s->mc_state.as<TsV>(), om, ol, on, ohas, ofast, stop_dev);
            HIPCHECK(s, hipGetLastError());
            return ACCORD_OK;
        }
        mc_scan_kernel<0><<<ntiles, MC_TILE, 0, st>>>(P, T[2].as<uint32_t>(), T[3].as<uint32_t>(), T[11].as<uint32_t>(),
                                                      T[13].as<TsV>(), s->lsb.as<uint64_t>(), mv, s->mc_state.as<TsV>(),
                                                      T[8].as<Comp>(), nullptr, nullptr, nullptr);
        mc_carry_kernel<<<1, MC_CARRY_THREADS, 0, st>>>(ntiles, T[8].as<Comp>(), T[9].as<TsV>());
        mc_scan_kernel<1><<<ntiles, MC_TILE, 0, st>>>(P, T[2].as<uint32_t>(), T[3].as<uint32_t>(), T[11].as<uint32_t>(),
                                                      T[13].as<TsV>(), s->lsb.as<uint64_t>(), mv, s->mc_state.as<TsV>(),
                                                      nullptr, T[9].as<TsV>(), T[7].as<TsV>(), s->mc_state2.as<TsV>());
    }
    if (outputs && nt)
        mc_fold_kernel<<<(nt + 255) / 256, 256, 0, st>>>(first, last, s->msb.as<uint64_t>(), s->lsb.as<uint64_t>(),
                                                         s->node.as<int32_t>(), po, T[7].as<TsV>(),
                                                         om, ol, on, ohas, ofast, s->has_exec ? 1u : 0u, mv.ov_t, stop_dev);
    HIPCHECK(s, hipGetLastError());
    return ACCORD_OK;
}

int32_t mc_fold(accord_store *s, uint32_t first, bool override, uint64_t ov_msb, uint64_t ov_lsb, int32_t ov_node,
                accord_max_conflicts_out *out)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (!s->has_batch) return fail(s, ACCORD_ERR_STATE, "accord_max_conflicts_fold before accord_batch_upload");
    if (first != s->mc_next || first >= s->n + (s->n == 0 ? 1u : 0u))
        return fail(s, ACCORD_ERR_STATE, "MaxConflicts fold of this batch must continue at txn %u (asked: %u)", s->mc_next, first);
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    int32_t rc = mc_ensure_state(s);
    if (rc) return rc;
    const uint32_t n = s->n;
    hipStream_t st = s->stream;
    HIPCHECK(s, s->mc_cnt.ensure(((size_t)n + 2) * 4));
    HIPCHECK(s, s->mc_po.ensure(((size_t)n + 2) * 4));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(n + 1), s->stream));
    HIPCHECK(s, s->mc_out.ensure((size_t)n * 22 + 64));
    HIPCHECK(s, s->status_totals.ensure(sizeof(HostTotals)));
    HostTotals *dev = s->status_totals.as<HostTotals>();
    uint32_t *stop_dev = (uint32_t *)&dev->totals[7];
    McValues mv;
    mv.vm = s->has_exec ? s->exec_msb.as<uint64_t>() : s->msb.as<uint64_t>();
    mv.vl = s->has_exec ? s->exec_lsb.as<uint64_t>() : s->lsb.as<uint64_t>();
    mv.vn = s->has_exec ? s->exec_node.as<int32_t>() : s->node.as<int32_t>();
    mv.ov_t = override ? first : 0xFFFFFFFFu;
    mv.ov_msb = ov_msb; mv.ov_lsb = ov_lsb; mv.ov_node = ov_node;

    if (s->events) HIPCHECK(s, hipEventRecord(s->ev[EV_OP_START], st));
    HIPCHECK(s, hipMemsetAsync(dev, 0xFF, sizeof(HostTotals), st));
    rc = mc_pass(s, first, n, mv, true, stop_dev);
    if (rc) return rc;
    if (s->events) HIPCHECK(s, hipEventRecord(s->ev[EV_OP_END], st));
    struct { accord::DevStatus status; uint32_t stop; } hs;
    HIPCHECK(s, hipMemcpyAsync(&hs.status, &dev->status, sizeof(hs.status), hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipMemcpyAsync(&hs.stop, stop_dev, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    if (hs.status.first != ~0ull) {
        const uint32_t txn = (uint32_t)(hs.status.first >> 32);
        const int32_t code = -(int32_t)(uint32_t)hs.status.first;
        return fail(s, code, "accord_max_conflicts_fold: txn %u rejected (code %d)", txn, code);
    }
    const uint32_t folded = hs.stop < n ? hs.stop : n;
    // a slow-path txn without a known executeAt: only [first, folded) may enter the map
    if (folded < n && folded > first) {
        rc = mc_pass(s, first, folded, mv, false, nullptr);
        if (rc) return rc;
    }
    if (folded > first) std::swap(s->mc_state, s->mc_state2);   // the merged txns' updates become the store's map
    s->mc_next = folded;
    if (s->events) HIPCHECK(s, hipEventElapsedTime(&s->ops_ms, s->ev[EV_OP_START], s->ev[EV_OP_END]));
    if (out) {
        uint64_t *om = s->mc_out.as<uint64_t>(), *ol = om + n;
        int32_t *on = (int32_t *)(ol + n);
        uint8_t *ohas = (uint8_t *)(on + n), *ofast = ohas + n;
        const size_t m = (size_t)n - first;
        if (out->msb && m) HIPCHECK(s, hipMemcpyAsync(out->msb + first, om + first, m * 8, hipMemcpyDeviceToHost, st));
        if (out->lsb && m) HIPCHECK(s, hipMemcpyAsync(out->lsb + first, ol + first, m * 8, hipMemcpyDeviceToHost, st));
        if (out->node && m) HIPCHECK(s, hipMemcpyAsync(out->node + first, on + first, m * 4, hipMemcpyDeviceToHost, st));
        if (out->present && m) HIPCHECK(s, hipMemcpyAsync(out->present + first, ohas + first, m, hipMemcpyDeviceToHost, st));
        if (out->fast && m) HIPCHECK(s, hipMemcpyAsync(out->fast + first, ofast + first, m, hipMemcpyDeviceToHost, st));
        HIPCHECK(s, hipStreamSynchronize(st));
        out->folded = folded;
    }
    return ACCORD_OK;
}

} // namespace

extern "C" int32_t accord_max_conflicts_fold(accord_store *s, accord_max_conflicts_out *out)
{
    return mc_fold(s, 0, false, 0, 0, 0, out);
}

extern "C" int32_t accord_max_conflicts_fold_from(accord_store *s, uint32_t first, uint64_t exec_msb, uint64_t exec_lsb,
                                                  int32_t exec_node, accord_max_conflicts_out *out)
{
    return mc_fold(s, first, true, exec_msb, exec_lsb, exec_node, out);
}

extern "C" int32_t accord_max_conflicts_state(accord_store *s, uint64_t *msb, uint64_t *lsb, int32_t *node,
                                              uint8_t *present)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (!msb || !lsb || !node || !present) return fail(s, ACCORD_ERR_ARG, "null output array");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    int32_t rc = mc_ensure_state(s);
    if (rc) return rc;
    const uint32_t nkeys = s->cfg.key_hi - s->cfg.key_lo;
    std::vector<TsV> h(nkeys);
    HIPCHECK(s, hipMemcpyAsync(h.data(), s->mc_state.p, (size_t)nkeys * sizeof(TsV), hipMemcpyDeviceToHost, s->stream));
    HIPCHECK(s, hipStreamSynchronize(s->stream));
    for (uint32_t k = 0; k < nkeys; ++k) {
        msb[k] = h[k].msb; lsb[k] = h[k].lsb; node[k] = h[k].node; present[k] = (uint8_t)(h[k].has != 0);
    }
    return ACCORD_OK;
}
