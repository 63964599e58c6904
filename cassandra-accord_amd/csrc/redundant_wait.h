// Commands.updateWaitingOn's removal step on the device (status.hip: initialiseWaitingOn, ready.hip:
// every evaluation), and WaitingOn.executeAtLeast.
//
// Reference (paths relative to accord-core/src/main/java/accord/):
//   Commands.updateWaitingOn            local/Commands.java:755-761 (removal before the dep visit)
//   WaitingOn.Update.minWaitingOnTxnId  local/Command.java:1500-1504 (first set bit, if a range dep)
//   hasLocallyRedundantDependencies     local/CommandStore.java:672-678: RedundantBefore.status >=
//                                       PARTIALLY_PRE_BOOTSTRAP_OR_STALE (Entry.getAndMerge / get,
//                                       local/RedundantBefore.java:157-161, 225-240; RedundantStatus.merge)
//   removeRedundantDependencies         local/CommandStore.java:601-670
//
// The status fold is >= PARTIALLY_PRE_BOOTSTRAP_OR_STALE iff some in-bounds entry the participants touch
// gives minWaitingOnTxnId a status other than LIVE (the merge table never returns to LIVE / NOT_OWNED
// once another status joined).  The removal, folded over those entries in ascending order, comes to
// (tests/test_ready.py checks it against the oracle's literal fold, or_lstore_ready):
//   rule 1  a range dep j whose RangeDeps ranges meet entry e, with bootstrapIdx_e <= j < appliedIdx_e;
//   rule 2  a range dep j covered by bootstrapping entries: every range r of j lies inside the union of
//           the fold's entries with j < bootstrapIdx_e -- they are disjoint, so the entries meeting r must
//           tile it without a gap (a map gap or an entry the participants do not touch leaves part of r
//           uncovered) and each have j < bootstrapIdx_e: j < cb_r = min bootstrapIdx over them (0 when r
//           is not tiled), for every r of j.  isFullyBootstrapping's remaining-ranges bookkeeping is
//           that union, order-free.
// A wave evaluates one txn: lane 0 lists the entries its participants touch, lanes take the RangeDeps
// ranges; the bits to clear gather in the wave's scratch -- LDS (RrLds: <= RR_MAXE entries, <= RR_MAXR
// range deps) or, for a txn over those caps, HBM sized by the spill pass (RrSpill below): the caps only
// decide where the scratch lives, never whether a txn is evaluated.
#pragma once
#include "status_view.h"

namespace accord_status {

constexpr uint32_t RR_NONE = 0xFFFFFFFFu;
constexpr uint32_t RR_MAXE = 64;             // entries a txn's participants may touch
constexpr uint32_t RR_MAXR = 4096;           // range deps of a txn (LDS masks of 64 words)

struct RrMap {
    uint32_t m;                              // entries (s, e] ascending and disjoint
    const uint32_t *s, *e, *local, *boot;    // locallyAppliedOrInvalidatedBefore / bootstrappedAt: positions
    const uint64_t *sep, *eep;               // [startEpoch, endEpoch)
    const uint8_t *stale;                    // staleUntilAtLeast != null
};

struct RrLds {
    unsigned long long rm[RR_MAXR / 64];     // rule 1: removed
    unsigned long long keep[RR_MAXR / 64];   // rule 2: some range of the dep not covered
    uint32_t E[RR_MAXE], bidx[RR_MAXE], aidx[RR_MAXE];
    uint32_t nE;
};

// One wave's removal scratch: the RrLds fields, in LDS or in HBM
struct RrBuf {
    unsigned long long *rm, *keep;           // [cap_r / 64]
    uint32_t *E, *bidx, *aidx;               // [cap_e]
    uint32_t *nE;
    uint32_t cap_r, cap_e;
};

__device__ __forceinline__ RrBuf rr_buf_lds(RrLds &L)
{
    return RrBuf{L.rm, L.keep, L.E, L.bidx, L.aidx, &L.nE, RR_MAXR, RR_MAXE};
}

// HBM scratch per spill wave for txns of up to cap_r range deps touching up to cap_e entries
__host__ __device__ __forceinline__ size_t rr_spill_wave_bytes(uint32_t cap_r, uint32_t cap_e)
{
    const size_t words = ((size_t)cap_r + 63u) / 64u;
    return (16u * words + 4u * (3u * (size_t)cap_e + 1u) + 255u) & ~(size_t)255u;
}

__device__ __forceinline__ RrBuf rr_buf_hbm(void *base, uint32_t wave, uint32_t cap_r, uint32_t cap_e)
{
    char *p = (char *)base + (size_t)wave * rr_spill_wave_bytes(cap_r, cap_e);
    const size_t words = ((size_t)cap_r + 63u) / 64u;
    RrBuf b;
    b.rm = (unsigned long long *)p;
    b.keep = b.rm + words;
    b.E = (uint32_t *)(b.keep + words);
    b.bidx = b.E + cap_e;
    b.aidx = b.bidx + cap_e;
    b.nE = b.aidx + cap_e;
    b.cap_r = (uint32_t)(words * 64u);
    b.cap_e = cap_e;
    return b;
}

// Txns over the LDS caps, evaluated again by a spill pass with HBM scratch: the ids, how many, and
// the largest range-dep / entry counts among them (the spill pass sizes its scratch from these)
struct RrSpill {
    uint32_t *count, *max_r, *max_e;
    uint32_t *list;
};

__device__ __forceinline__ void rr_spill_add(const RrSpill &sp, uint32_t id, uint32_t R, uint32_t nE)
{
    sp.list[atomicAdd(sp.count, 1u)] = id;
    atomicMax(sp.max_r, R);
    atomicMax(sp.max_e, nE);
}

// the waiting txn: its participants and its RangeDeps
struct RrTxn {
    bool rdom;                               // Range domain: participants are ranges (ps, pe]
    uint32_t np;
    const uint32_t *pk, *ps, *pe;            // keys [np] | ranges [np]
    uint32_t R;                              // RangeDeps txnIds (positions, ascending)
    const uint32_t *rvals;
    uint32_t nrr;                            // RangeDeps ranges (rs, re] and rangesToTxnIds (header nrr, body)
    const uint32_t *rs, *re;
    const uint32_t *r2v;
};

// the store's map (store_impl.h fields; host side)
template <typename S> inline RrMap rr_map_of(const S *s)
{
    RrMap M{};
    M.m = s->rb_m;
    M.s = s->rb_start.template as<uint32_t>(); M.e = s->rb_end.template as<uint32_t>();
    M.local = s->rb_local.template as<uint32_t>(); M.boot = s->rb_boot.template as<uint32_t>();
    M.sep = s->rb_sep.template as<uint64_t>(); M.eep = s->rb_eep.template as<uint64_t>();
    M.stale = s->rb_stale.template as<uint8_t>();
    return M;
}

__device__ __forceinline__ uint32_t rr_first_end_above(const RrMap &M, uint32_t x)   // first entry with e > x
{
    uint32_t lo = 0, hi = M.m;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (M.e[mid] > x) hi = mid; else lo = mid + 1;
    }
    return lo;
}

// insertion point of bound among the txn's range deps (positions ascend with TxnIds; NONE first)
__device__ __forceinline__ uint32_t rr_find(const RrTxn &T, uint32_t bound)
{
    if (bound == RR_NONE) return 0;
    uint32_t lo = 0, hi = T.R;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (T.rvals[mid] < bound) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// first index of list[lo, hi) whose value >= v
__device__ __forceinline__ uint32_t rr_lower(const uint32_t *list, uint32_t lo, uint32_t hi, uint32_t v)
{
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (list[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// set bits list[a, b) of a mask in LDS (runs in one word OR'ed at once)
__device__ __forceinline__ void rr_mark(unsigned long long *mask, const uint32_t *list, uint32_t a, uint32_t b)
{
    uint32_t w = RR_NONE;
    unsigned long long acc = 0;
    for (uint32_t y = a; y < b; ++y) {
        const uint32_t j = list[y];
        if ((j >> 6) != w) {
            if (acc) atomicOr(&mask[w], acc);
            w = j >> 6;
            acc = 0;
        }
        acc |= 1ull << (j & 63u);
    }
    if (acc) atomicOr(&mask[w], acc);
}

// The range-dep bits of a waiting txn to clear (words[] holds its current WaitingOn; minimum set bit j0
// a range dep at position min_pos): returns false when the status fold keeps everything; when the
// txn exceeds the scratch's caps, returns false with *ovf set and *need_e = its entry count (nothing
// was decided: the caller leaves the txn to the spill pass).  On true, rr_clear(q) below gives word q's
// bits to clear.  Every lane of the wave calls it (wave-uniform arguments).
__device__ inline bool rr_removal(const RrMap &M, const RrTxn &T, const RrBuf &L, uint32_t lane, uint32_t min_pos,
                                  uint64_t min_epoch, uint64_t exec_epoch, bool *ovf, uint32_t *need_e)
{
    if (lane == 0) {            // the entries the participants touch, ascending, once (ReducingRangeMap.foldl)
        uint32_t n = 0;
        int64_t last = -1;
        for (uint32_t i = 0; i < T.np; ++i) {
            const uint32_t a = T.rdom ? T.ps[i] : T.pk[i] - 1u, b = T.rdom ? T.pe[i] : T.pk[i];   // key k = (k-1, k]
            for (uint32_t x = rr_first_end_above(M, a); x < M.m && M.s[x] < b; ++x) {
                if ((int64_t)x <= last) continue;
                last = x;
                if (n < L.cap_e) L.E[n] = x;
                ++n;
            }
        }
        *L.nE = n;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    const uint32_t nE = *L.nE;
    __builtin_amdgcn_wave_barrier();
    if (nE > L.cap_e || T.R > L.cap_r) { *ovf = true; *need_e = nE; return false; }
    // the status fold: an in-bounds entry giving minWaitingOnTxnId a status other than LIVE
    bool hot = false;
    for (uint32_t i = lane; i < nE; i += 64) {
        const uint32_t x = L.E[i];
        const bool out = exec_epoch < M.sep[x] || min_epoch >= M.eep[x];                 // Entry.outOfBounds
        hot |= !out && (M.stale[x] || (M.boot[x] != RR_NONE && M.boot[x] > min_pos) ||
                        (M.local[x] != RR_NONE && M.local[x] > min_pos));
        L.bidx[i] = rr_find(T, M.boot[x]);
        L.aidx[i] = rr_find(T, M.local[x]);
    }
    const uint32_t nw = (T.R + 63u) / 64u;
    for (uint32_t q = lane; q < nw; q += 64) { L.rm[q] = 0; L.keep[q] = 0; }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    if (__ballot(hot) == 0ull) return false;
    for (uint32_t r = lane; r < T.nrr; r += 64) {
        const uint32_t rs = T.rs[r], re = T.re[r];
        const uint32_t la = r == 0 ? T.nrr : T.r2v[r - 1], lb = T.r2v[r];     // its txn indices, ascending
        uint32_t cursor = rs, cb = RR_NONE;
        bool tiled = true;
        for (uint32_t i = 0; i < nE; ++i) {
            const uint32_t x = L.E[i], es = M.s[x], ee = M.e[x];
            if (!(es < re && rs < ee)) continue;                              // meets r
            const uint32_t bi = L.bidx[i], ai = L.aidx[i];
            if (ai > bi)                                                      // rule 1
                rr_mark(L.rm, T.r2v, rr_lower(T.r2v, la, lb, bi), rr_lower(T.r2v, la, lb, ai));
            if (es > cursor) tiled = false;                                   // a gap before this entry
            cursor = max(cursor, ee);
            cb = min(cb, bi);
        }
        if (!tiled || cursor < re || cb == RR_NONE) cb = 0;
        rr_mark(L.keep, T.r2v, rr_lower(T.r2v, la, lb, cb), lb);              // rule 2 fails for these
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    return true;
}

// word q of the range bits to clear after rr_removal returned true
__device__ __forceinline__ unsigned long long rr_clear(const RrBuf &L, const RrTxn &T, uint32_t q)
{
    const uint32_t nw = (T.R + 63u) / 64u;
    if (q >= nw) return 0ull;
    const unsigned long long valid = (q + 1u) * 64u <= T.R ? ~0ull : ((1ull << (T.R & 63u)) - 1ull);
    return (L.rm[q] | ~L.keep[q]) & valid;
}

// WaitingOn.executeAtLeast per waiting txn (has = 0: null)
struct EalRec {
    uint64_t msb, lsb;
    int32_t node;
    uint32_t has;
};

// a = take ? b : a, field by field.  Written as value selects with a non-short-circuit condition:
// the branchy form (if (b.has && (!a.has || ts_cmp(a, b) < 0)) a = b) is miscompiled for gfx950 by
// ROCm 7.2's clang inside wo_init_kernel's loop -- on the a.has path the node / has pair is carried
// over unselected while msb / lsb take b's (profiles/r05_eal/wo_init_merge_isa_before.s).
__device__ __forceinline__ void eal_take(EalRec &a, const EalRec &b, bool take)
{
    a.msb = take ? b.msb : a.msb;
    a.lsb = take ? b.lsb : a.lsb;
    a.node = take ? b.node : a.node;
    a.has = take ? b.has : a.has;
}

// wave maximum of the lanes' candidates (has = false: none); the result is uniform
__device__ inline EalRec eal_wave_max(bool has, const Ts &t)
{
    EalRec r{t.msb, t.lsb, t.node, has ? 1u : 0u};
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        EalRec u;
        u.msb = __shfl_xor(r.msb, o, 64); u.lsb = __shfl_xor(r.lsb, o, 64);
        u.node = __shfl_xor(r.node, o, 64); u.has = __shfl_xor(r.has, o, 64);
        eal_take(r, u, (u.has != 0u) & ((r.has == 0u) | (ts_cmp(r.msb, r.lsb, r.node, u.msb, u.lsb, u.node) < 0)));
    }
    return r;
}

__device__ __forceinline__ void eal_merge(EalRec &a, const EalRec &b)      // Timestamp.nonNullOrMax
{
    eal_take(a, b, (b.has != 0u) & ((a.has == 0u) | (ts_cmp(a.msb, a.lsb, a.node, b.msb, b.lsb, b.node) < 0)));
}

} // namespace accord_status
