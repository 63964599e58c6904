// WaitingOn bitsets and execution levelling (config 5).
//
// Reference:
//   Commands.initialiseWaitingOn   local/Commands.java:735-753   (bits [0,R) range-dep txnIds,
//   WaitingOn.Update               local/Command.java:1403-1437   [R, R+K) keyDeps keys)
//   Commands.updateWaitingOn       local/Commands.java:755-830   (clears deps executing later /
//                                                                 applied / invalidated)
//   CommandsForKey.notify          local/CommandsForKey.java:1501-1635 (execution in executeAt order)
// Model of config 5: every txn STABLE with executeAt = txnId, none applied, so
// every dep executes earlier and no bit is cleared: the bitset is R+K ones.  Levelling
// abstraction (§8a a13): level(T) = 0 if no dep executes before T, else 1 + max level(dep).
//
// Levelling on a reduced DAG.  For a key txn i and key k, its deps on k are the witnessed entries
// of k's history in [lo, i).  Every Write w in that slice depends on every earlier witnessed entry
// of the slice (their slices nest), so max level over the slice = max over {the last Write lw of
// the slice} and, when i is a Write, the Reads after lw.  Only those are kept as predecessors.
// The levels themselves come from a chunked max-plus closure of that DAG (see lv_closure_kernel /
// lv_staged_kernel below).
#include "device_common.h"
#include "kernels.h"
#include "../../include/accord_deps.h"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace accord {

namespace {

__global__ __launch_bounds__(256) void wo_bits_kernel(uint32_t n, const uint32_t *__restrict__ kd_key_off,
                                                      const uint32_t *__restrict__ rd_val_off,
                                                      const uint32_t *__restrict__ wo_off,
                                                      unsigned long long *__restrict__ words)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t bits = (rd_val_off[i + 1] - rd_val_off[i]) + (kd_key_off[i + 1] - kd_key_off[i]);
        const uint32_t w0 = wo_off[i], nw = wo_off[i + 1] - w0;
        for (uint32_t q = 0; q < nw; ++q) {
            const uint32_t hi = bits - q * 64;
            words[w0 + q] = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
        }
    }
}

__global__ __launch_bounds__(256) void wo_words_count_kernel(uint32_t n, const uint32_t *__restrict__ kd_key_off,
                                                             const uint32_t *__restrict__ rd_val_off,
                                                             uint32_t *__restrict__ cnt)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t bits = (rd_val_off[i + 1] - rd_val_off[i]) + (kd_key_off[i + 1] - kd_key_off[i]);
        cnt[i] = (bits + 63) / 64;
    }
}

// Reduced predecessors of every txn (count pass: FILL=false; fill pass: FILL=true).
// The reduction needs witnesses(i) ⊆ witnesses(Write) = {R, W}; SyncPoints (which also witness
// SyncPoints, that a Write does not) and range txns (whose KeyDeps come from rangekeys, not from
// key histories) keep their full dependency lists.
constexpr uint32_t WO_KB = 4;      // keys per txn walked with batched loads (larger txns: one key at a time)
template <bool FILL>
__global__ __launch_bounds__(256) void wo_preds_kernel(WaitingOnParams p)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.n; i += gridDim.x * blockDim.x) {
        const uint64_t l = p.lsb[i];
        const uint32_t kind = (uint32_t)(l >> 1) & 7;
        const uint32_t wmask = witness_mask(kind);
        const bool reduce = (l & 1) == 0 && (wmask & ~0x3u) == 0;
        uint32_t cnt = 0;
        uint32_t o = FILL ? p.pred_off[i] : 0;
        const uint32_t q0 = p.key_off[i], k = p.key_off[i + 1] - q0;
        if (reduce && k <= WO_KB) {
            // the same walk with each dependent round (slices, Write bounds, last Writes) issued for
            // all keys at once
            PairSlice ps[WO_KB];
            uint32_t pw[WO_KB], lw[WO_KB];
#pragma unroll
            for (uint32_t j = 0; j < WO_KB; ++j) ps[j] = j < k ? p.slice[q0 + j] : PairSlice{0u, 0u, 0u, 0u};
#pragma unroll
            for (uint32_t j = 0; j < WO_KB; ++j) {
                const uint32_t x = ps[j].pos - 1;
                pw[j] = ps[j].pos != ps[j].lo ? max(p.pw_local[x], p.pw_carry[x / p.pw_tile]) : 0u;   // (last Write <= x) + 1
            }
#pragma unroll
            for (uint32_t j = 0; j < WO_KB; ++j) lw[j] = FILL && pw[j] > ps[j].lo ? p.hist[pw[j] - 1] : 0u;
#pragma unroll
            for (uint32_t j = 0; j < WO_KB; ++j) {
                const uint32_t pos = ps[j].pos, lo = ps[j].lo;
                if (pos == lo) continue;
                uint32_t from = lo;
                if (pw[j] > lo) {                                                   // lw inside the slice
                    ++cnt;
                    if (FILL) p.preds[o++] = lw[j] & ENT_TXN_MASK;
                    from = pw[j];
                }
                if (wmask & 1u) {                                                   // Reads after lw
                    if (!FILL && p.rw_only) {        // after the slice's last Write every entry is a Read
                        cnt += pos - from;
                        continue;
                    }
                    for (uint32_t e = from; e < pos; ++e) {
                        const uint32_t ev = p.hist[e];
                        if ((wmask >> (ev >> ENT_KIND_SHIFT)) & 1u) {
                            ++cnt;
                            if (FILL) p.preds[o++] = ev & ENT_TXN_MASK;
                        }
                    }
                }
            }
        } else if (reduce) {
            for (uint32_t q = p.key_off[i]; q < p.key_off[i + 1]; ++q) {
                const PairSlice ps = p.slice[q];
                const uint32_t pos = ps.pos, lo = ps.lo;
                if (pos == lo) continue;
                const uint32_t x = pos - 1;
                const uint32_t pw = max(p.pw_local[x], p.pw_carry[x / p.pw_tile]);   // (last Write <= x) + 1
                uint32_t from = lo;
                if (pw > lo) {                                                      // lw inside the slice
                    ++cnt;
                    if (FILL) p.preds[o++] = p.hist[pw - 1] & ENT_TXN_MASK;
                    from = pw;
                }
                if (wmask & 1u) {                                                   // Reads after lw
                    for (uint32_t e = from; e < pos; ++e) {
                        const uint32_t ev = p.hist[e];
                        if ((wmask >> (ev >> ENT_KIND_SHIFT)) & 1u) {
                            ++cnt;
                            if (FILL) p.preds[o++] = ev & ENT_TXN_MASK;
                        }
                    }
                }
            }
        } else {
            const uint32_t v1 = p.kd_val_cnt ? p.kd_val_off[i] + p.kd_val_cnt[i] : p.kd_val_off[i + 1];
            for (uint32_t v = p.kd_val_off[i]; v < v1; ++v) {
                ++cnt;
                if (FILL) p.preds[o++] = p.kd_vals[v];
            }
        }
        for (uint32_t v = p.rd_val_off[i]; v < p.rd_val_off[i + 1]; ++v) {     // range deps: all
            ++cnt;
            if (FILL) p.preds[o++] = p.rd_vals[v];
        }
        if (!FILL) p.pred_cnt[i] = cnt;
        if (FILL && p.pred_own)
            for (uint32_t e = p.pred_off[i]; e < o; ++e) p.pred_own[e] = (uint8_t)(i & 63u);
    }
}

// ---- execution levelling: chunked max-plus closure ----
// The chain depth of the reduced DAG is a large fraction of n (config 5: ~0.36 n, the Write
// chain of the hottest key), so resolving one level per step is hopeless.  Instead:
//   pass 1 (parallel, one wave per chunk of 64 consecutive txns): the longest-path closure of the
//     chunk's own sub-DAG, dist(i, j) for j -> ... -> i inside the chunk, and the chunk's far
//     predecessors.  With v = level + 1 and basev(j) = 1 + max v over j's far predecessors (1
//     without), v(i) = max over in-chunk ancestors j of i (and j = i) of basev(j) + dist(i, j).
//     Columns of txns without far predecessors (basev = 1) fold into one constant per row.
//   pass 2 (one workgroup, lv_staged_kernel): helper waves stage each chunk -- its far
//     predecessors' v (LDS ring of the last LV_RING txns, older ones from HBM) folded into the
//     columns whose predecessors lie in chunks <= x-3 -- and one resolver wave, alone on its SIMD,
//     walks the chain doing only the "late" columns (a predecessor in chunk x-1 or x-2) with a
//     max-plus matrix-vector product (lane = row).  (The earlier all-waves resolver, every wave
//     owning every 8th chunk, measured 48.3 against 44.7 ms and is gone, round 5.)
constexpr uint32_t LC = 64;                 // txns per chunk
constexpr int LV_REFS = 8;                  // far predecessors kept per entry column
constexpr uint32_t LV_RING = 16384;         // pass-2 LDS ring of v (64 KiB)
constexpr uint32_t LV_ROW = 68;             // closure row stride in LDS (bytes; 17 dwords)
constexpr uint32_t REF_NONE = 0xFFFFFFFFu;
// per-chunk record (u32 words): cst[64] | bq[16][64] | ref[LV_REFS][64] | node[64] | hdr[64]
constexpr uint32_t RC_CST = 0, RC_BQ = 64, RC_REF = RC_BQ + 16 * 64, RC_NODE = RC_REF + LV_REFS * 64,
                   RC_HDR = RC_NODE + 64, RC_WORDS = RC_HDR + 64;
static_assert(LV_RING % LC == 0, "ring holds whole chunks");

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l)
{
    const uint32_t lo = readlane((uint32_t)v, l), hi = readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// Pass 1.  Record layout per row i (node order): cst = max over non-entry columns j reaching i of
// 1 + b(i,j); bq = b(i, slot) bytes in slot order, b = dist + 1 (0 = j does not reach i).  Slots:
// late entries, then early entries, then non-entries.  ref[s][slot] = the slot's far predecessors.
// hdr = nl | ne << 8 | slow << 16 (slow: some entry has more than LV_REFS far predecessors).
// late_chunks: an entry is late when a predecessor lies in the previous late_chunks chunks (2: the
// staged resolver lv_staged_kernel).
__global__ __launch_bounds__(256) void lv_closure_kernel(uint32_t n, uint32_t nchunks,
                                                         const uint32_t *__restrict__ pred_off,
                                                         const uint32_t *__restrict__ preds,
                                                         uint32_t *__restrict__ rec, uint32_t *__restrict__ info,
                                                         uint32_t late_chunks)
{
    __shared__ __attribute__((aligned(16))) uint8_t rows_all[4][64 * LV_ROW];
    __shared__ uint32_t snode_all[4][64];
    const uint32_t w = wave_id(), lane = lane_id();
    const uint32_t x = blockIdx.x * 4 + w;
    if (x >= nchunks) return;                       // wave-uniform
    uint8_t *rows = rows_all[w];
    uint32_t *snode = snode_all[w];
    const uint32_t base = x * LC, t = base + lane;
    const bool valid = t < n;
    uint64_t inmask = 0;
    uint32_t ref[LV_REFS];
#pragma unroll
    for (int s = 0; s < LV_REFS; ++s) ref[s] = REF_NONE;
    uint32_t nfar = 0;
    bool late = false, bad = false;
    if (valid) {
        const uint32_t q0 = pred_off[t], q1 = pred_off[t + 1];
        for (uint32_t q = q0; q < q1; ++q) {
            const uint32_t f = preds[q];
            if (f >= t) { bad = true; continue; }
            if (f >= base) { inmask |= 1ull << (f - base); continue; }
            bool dup = false;
#pragma unroll
            for (int s = 0; s < LV_REFS; ++s) dup = dup || ref[s] == f;
            if (dup) continue;
            late = late || f + late_chunks * LC >= base;
#pragma unroll
            for (int s = 0; s < LV_REFS; ++s)
                if (s == (int)nfar) ref[s] = f;
            ++nfar;
        }
    }
    if (bad) atomicOr(&info[2], 1u);
    const bool entry = nfar > 0;
    const uint64_t lm = __ballot(entry && late), em = __ballot(entry && !late);
    const uint32_t nl = (uint32_t)__popcll(lm), ne = nl + (uint32_t)__popcll(em);
    const uint64_t lt = lanemask_lt();
    const uint32_t slot = entry ? (late ? (uint32_t)__popcll(lm & lt) : nl + (uint32_t)__popcll(em & lt))
                                : ne + (uint32_t)__popcll(~(lm | em) & lt);
    const bool slow = __ballot(nfar > (uint32_t)LV_REFS) != 0;
    snode[slot] = lane;
    wave_lds_sync();
    const uint32_t mynode = snode[lane];           // the node of column slot `lane`

    // closure, rows in node order; every lane owns one column (its own LDS bytes only)
    for (uint32_t i = 0; i < LC; ++i) {
        uint64_t mm = readlane64(inmask, (int)i);
        uint32_t v = mynode == i ? 1u : 0u;
        while (mm) {
            const uint32_t p = (uint32_t)__builtin_ctzll(mm);
            mm &= mm - 1;
            const uint32_t bp = rows[p * LV_ROW + lane];
            v = max(v, bp ? bp + 1u : 0u);
        }
        rows[i * LV_ROW + lane] = (uint8_t)v;
    }
    wave_lds_sync();

    uint32_t *r = rec + (size_t)x * RC_WORDS;
    uint32_t cst = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const uint32_t d = *(const uint32_t *)(rows + lane * LV_ROW + 4 * q);
        r[RC_BQ + q * 64 + lane] = d;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t b = (d >> (8 * c)) & 0xFFu;
            if ((uint32_t)(4 * q + c) >= ne && b) cst = max(cst, b + 1u);
        }
    }
    r[RC_CST + lane] = cst;
#pragma unroll
    for (int s = 0; s < LV_REFS; ++s) r[RC_REF + s * 64 + slot] = ref[s];
    r[RC_NODE + slot] = lane;
    r[RC_HDR + lane] = nl | (ne << 8) | (slow ? 1u << 16 : 0u);
}

struct LvRec {
    uint32_t cst, bq[16], ref[LV_REFS], node, hdr;
};

__device__ __forceinline__ void lv_load(const uint32_t *__restrict__ rec, uint32_t x, uint32_t nchunks, uint32_t lane,
                                        LvRec &o)
{
    if (x >= nchunks) { o.hdr = 0; return; }
    const uint32_t *r = rec + (size_t)x * RC_WORDS;
    o.cst = r[RC_CST + lane];
#pragma unroll
    for (int q = 0; q < 16; ++q) o.bq[q] = r[RC_BQ + q * 64 + lane];
#pragma unroll
    for (int s = 0; s < LV_REFS; ++s) o.ref[s] = r[RC_REF + s * 64 + lane];
    o.node = r[RC_NODE + lane];
    o.hdr = r[RC_HDR + lane];
}

// Column slot m of row `lane` as a signed addend: b(row, m) (= dist + 1) when m reaches the row,
// INT_MIN otherwise, so basev(m) + d never wins a signed max (basev < 2^31).
__device__ __forceinline__ void lv_expand(const uint32_t (&bq)[16], int32_t (&d)[64])
{
#pragma unroll
    for (int m = 0; m < 64; ++m) {
        const uint32_t b = (bq[m >> 2] >> (8 * (m & 3))) & 0xFFu;
        d[m] = b ? (int32_t)b : INT32_MIN;
    }
}

// acc = max(acc, basev(m) + d(row, m)) over column slots [lo, hi) widened to groups of 8.  Extra
// columns are harmless: a non-entry column has basev 1 (its share is already in cst) and a column
// seen with a partial basev only yields a lower bound of the row's value.
__device__ __forceinline__ int32_t lv_matvec(int32_t acc, const int32_t (&d)[64], uint32_t bv, uint32_t lo,
                                             uint32_t hi)
{
    int32_t acc2 = acc;                     // two max chains: half the dependent-latency depth
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        if ((uint32_t)(8 * g) < hi && (uint32_t)(8 * g + 8) > lo) {      // wave-uniform
#pragma unroll
            for (int m = 8 * g; m < 8 * g + 8; m += 4) {
                const int32_t s0 = (int32_t)readlane(bv, m), s1 = (int32_t)readlane(bv, m + 1);
                const int32_t s2 = (int32_t)readlane(bv, m + 2), s3 = (int32_t)readlane(bv, m + 3);
                acc = max(acc, max(s0 + d[m], s1 + d[m + 1]));
                acc2 = max(acc2, max(s2 + d[m + 2], s3 + d[m + 3]));
            }
        }
    }
    return max(acc, acc2);
}

constexpr uint32_t LS_K = 4;                  // staged chunks in flight
constexpr int LS_LREF = 8;                    // late predecessors per column in the slot
constexpr int LS_HELPERS = 7;
constexpr uint32_t LS_ZERO = LV_RING;         // ring word that stays 0: an absent reference
struct LsSlot {
    int4 d[16][64];                           // d[g][row] = b(row, 4g..4g+3), INT_MIN if unreachable
    int32_t acc_e[64];                        // per row: max(cst, early columns' products)
    uint32_t bv_e[64];                        // per column slot: base from predecessors in chunks <= x-3
    uint32_t lref[LS_LREF / 2][64];           // per column slot: two 16-bit ring indices per word
    uint32_t node[64];                        // column slot -> row
    uint32_t ready;                           // (chunk + 1) << 9 | slowlate << 8 | nl, once staged
    uint32_t dready;                          // chunk + 1 once d is staged (the resolver prefetches it)
};
struct LsShared {
    uint32_t ring[LV_RING + 1];
    LsSlot slot[LS_K];
    uint32_t done, abort_flag, maxlv;
};

// Spin until *flag == target (EQ) or >= target; false once any wave gave up.  The asm barrier keeps
// the compiler from moving the caller's LDS reads above the wait (LDS ops of a wave execute in
// order, and the writer's data lands before its flag).  Helpers sleep between polls so their spins
// leave the LDS and the issue slots to the resolver.
template <bool EQ, bool SLEEP>
__device__ __forceinline__ bool ls_spin(const uint32_t *flag, uint32_t *abort_flag, uint32_t target)
{
    uint32_t spins = 0;
    for (;;) {
        const uint32_t v = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (EQ ? v == target : v >= target) break;
        if (SLEEP) __builtin_amdgcn_s_sleep(1);
        if ((++spins & 255u) == 0) {
            if (__builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
                return false;
            if (spins > (1u << 26)) {
                __hip_atomic_store(abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                return false;
            }
        }
    }
    asm volatile("" ::: "memory");
    return true;
}
__device__ __forceinline__ bool ls_wait_done(const uint32_t *done, uint32_t *abort_flag, uint32_t target)
{
    return ls_spin<false, true>(done, abort_flag, target);
}

// Helper: stage chunk x (record `cur`) into its slot.  False on abort.
__device__ __forceinline__ bool ls_stage(LsShared &S, uint32_t n, uint32_t x, const LvRec &cur,
                                         const uint32_t *__restrict__ pred_off, const uint32_t *__restrict__ preds,
                                         uint32_t *level, uint32_t lane, unsigned long long *stats)
{
    const uint32_t base = x * LC;
    const uint32_t hdr = __builtin_amdgcn_readfirstlane(cur.hdr);
    const uint32_t nl = hdr & 0xFFu, ne = (hdr >> 8) & 0xFFu;
    const bool slow = (hdr >> 16) & 1u;
    // predecessors older than the ring: final long ago, loaded now
    uint32_t oldv[LV_REFS];
#pragma unroll
    for (int s = 0; s < LV_REFS; ++s) {
        const uint32_t f = cur.ref[s];
        const bool old = !slow && f != REF_NONE && f + LV_RING < base;
        oldv[s] = level[old ? f : 0u];
    }
    int32_t d[64];
    lv_expand(cur.bq, d);
    LsSlot &sl = S.slot[x % LS_K];
    // the slot is free once the resolver has finished chunk x - LS_K
    if (!ls_wait_done(&S.done, &S.abort_flag, x + 1 >= LS_K ? x + 1 - LS_K : 0u)) return false;
    // the late columns' closure, in the resolver's groups of 8 columns
#pragma unroll
    for (int g = 0; g < 16; ++g)
        if ((uint32_t)(8 * (g >> 1)) < nl) sl.d[g][lane] = make_int4(d[4 * g], d[4 * g + 1], d[4 * g + 2], d[4 * g + 3]);
    wave_lds_sync();
    if (lane == 0) __hip_atomic_store(&sl.dready, x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // chunks <= x-3 final
    if (!ls_wait_done(&S.done, &S.abort_flag, x >= 2 ? x - 2 : 0u)) return false;
    const unsigned long long tp = stats ? __builtin_amdgcn_s_memtime() : 0ull;
    if (x >= 3) {                                     // chunk x-3 is final: its levels to HBM (the
        const uint32_t c = (x - 3) * LC + lane;       // resolver itself issues no vector-memory op)
        if (c < n) level[c] = S.ring[c % LV_RING] - 1u;
    }
    uint32_t e = 0, lr[LS_LREF];
#pragma unroll
    for (int s = 0; s < LS_LREF; ++s) lr[s] = LS_ZERO;
    bool slowlate = false;
    if (!slow) {
        uint32_t rv[LV_REFS];
#pragma unroll
        for (int s = 0; s < LV_REFS; ++s) {          // LDS reads issued together
            const uint32_t f = cur.ref[s];
            const bool mid = f != REF_NONE && f + 2 * LC < base && f + LV_RING >= base;
            rv[s] = S.ring[mid ? f % LV_RING : LS_ZERO];
        }
#pragma unroll
        for (int s = 0; s < LV_REFS; ++s) {
            const uint32_t f = cur.ref[s];
            if (f == REF_NONE) continue;
            if (f + 2 * LC >= base) lr[s] = f % LV_RING;
            else e = max(e, f + LV_RING < base ? oldv[s] + 1u : rv[s]);
        }
    } else if (lane < ne) {
        // some entry has more predecessors than the record holds: its full list
        const uint32_t t = base + cur.node;
        uint32_t nlr = 0;
        if (t < n) {
            for (uint32_t q = pred_off[t], q1 = pred_off[t + 1]; q < q1; ++q) {
                const uint32_t f = preds[q];
                if (f >= base) continue;
                if (f + 2 * LC >= base) {
                    bool dup = false;
#pragma unroll
                    for (int s = 0; s < LS_LREF; ++s) dup = dup || lr[s] == f % LV_RING;
                    if (dup) continue;
#pragma unroll
                    for (int s = 0; s < LS_LREF; ++s)
                        if (s == (int)nlr) lr[s] = f % LV_RING;
                    if (nlr == (uint32_t)LS_LREF) slowlate = true;
                    else ++nlr;
                } else {
                    e = max(e, f + LV_RING >= base ? S.ring[f % LV_RING] : level[f] + 1u);
                }
            }
        }
    }
    const uint32_t bv = e + 1u;
    int32_t acc = lv_matvec((int32_t)cur.cst, d, bv, nl, ne);
    sl.acc_e[lane] = acc;
    sl.bv_e[lane] = bv;
#pragma unroll
    for (int s = 0; s < LS_LREF / 2; ++s) sl.lref[s][lane] = lr[2 * s] | lr[2 * s + 1] << 16;
    sl.node[lane] = cur.node;
    const bool any_slowlate = __ballot(slowlate) != 0;
    wave_lds_sync();                                  // the slot's contents before its flag
    if (lane == 0)
        __hip_atomic_store(&sl.ready, (x + 1) << 9 | (any_slowlate ? 1u << 8 : 0u) | nl, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_WORKGROUP);
    if (stats) *stats += __builtin_amdgcn_s_memtime() - tp;
    return true;
}

// Resolver: chunk x from its staged slot.  (Prefetching the next chunk's closure into a second
// register set measured slower: the compiler's register shuffles between the two sets drain the
// prefetch loads.)  The poll reads the flag and the slot's small fields together (LDS ops of a wave
// run in order: fields read after a flag that shows the chunk are the staged ones).  False on abort.
// lv_matvec over the resolver's int4 register image of the late columns
__device__ __forceinline__ int32_t ls_matvec(int32_t acc, const int4 (&d)[16], uint32_t bv, uint32_t hi)
{
    int32_t acc2 = acc;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        if ((uint32_t)(8 * g) < hi) {                 // wave-uniform
            const int4 p = d[2 * g], q = d[2 * g + 1];
            const int m = 8 * g;
            const int32_t s0 = (int32_t)readlane(bv, m), s1 = (int32_t)readlane(bv, m + 1);
            const int32_t s2 = (int32_t)readlane(bv, m + 2), s3 = (int32_t)readlane(bv, m + 3);
            acc = max(acc, max(s0 + p.x, s1 + p.y));
            acc2 = max(acc2, max(s2 + p.z, s3 + p.w));
            const int32_t s4 = (int32_t)readlane(bv, m + 4), s5 = (int32_t)readlane(bv, m + 5);
            const int32_t s6 = (int32_t)readlane(bv, m + 6), s7 = (int32_t)readlane(bv, m + 7);
            acc = max(acc, max(s4 + q.x, s5 + q.y));
            acc2 = max(acc2, max(s6 + q.z, s7 + q.w));
        }
    }
    return max(acc, acc2);
}

__device__ __forceinline__ bool ls_resolve(LsShared &S, uint32_t n, uint32_t nchunks, uint32_t x,
                                           const uint32_t *__restrict__ pred_off, const uint32_t *__restrict__ preds,
                                           uint32_t *level, uint32_t lane, uint32_t &mymax, unsigned long long *tmid)
{
    const uint32_t base = x * LC;
    LsSlot &sl = S.slot[x % LS_K];
    uint32_t hdr, spins = 0;
    int32_t acc_e;
    uint32_t bv_e, lw[LS_LREF / 2];
    for (;;) {
        hdr = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&sl.ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        asm volatile("" ::: "memory");
        acc_e = sl.acc_e[lane];
        bv_e = sl.bv_e[lane];
#pragma unroll
        for (int s = 0; s < LS_LREF / 2; ++s) lw[s] = sl.lref[s][lane];
        if ((hdr >> 9) == x + 1) break;
        if ((++spins & 255u) == 0) {
            if (__builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(&S.abort_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
                return false;
            if (spins > (1u << 26)) {
                __hip_atomic_store(&S.abort_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                return false;
            }
        }
    }
    const uint32_t nl = hdr & 0xFFu;
    uint32_t rv[LS_LREF];
#pragma unroll
    for (int s = 0; s < LS_LREF; ++s) rv[s] = S.ring[(lw[s >> 1] >> (16 * (s & 1))) & 0xFFFFu];
    // the first 40 columns' closure unconditionally (columns past nl are not used; a uniform branch
    // per read would make the compiler wait after each), the rest only for the rare wider chunk
    int4 d[16];
#pragma unroll
    for (int g = 0; g < 10; ++g) d[g] = sl.d[g][lane];
    if (nl > 40) {                                    // (else d[10..15] stay unset: not read)
#pragma unroll
        for (int g = 10; g < 16; ++g) d[g] = sl.d[g][lane];
    }
    uint32_t lat = max(max(max(rv[0], rv[1]), max(rv[2], rv[3])), max(max(rv[4], rv[5]), max(rv[6], rv[7])));
    if ((hdr >> 8) & 1u) {                            // a late column with more than LS_LREF: its full list
        const uint32_t t = base + sl.node[lane];
        if (lane < nl && t < n) {
            for (uint32_t q = pred_off[t], q1 = pred_off[t + 1]; q < q1; ++q) {
                const uint32_t f = preds[q];
                if (f < base && f + 2 * LC >= base) lat = max(lat, S.ring[f % LV_RING]);
            }
        }
    }
    const uint32_t bv = max(bv_e, lat + 1u);
    if (tmid) *tmid = __builtin_amdgcn_s_memtime();
    const int32_t acc = ls_matvec(acc_e, d, bv, nl);
    const uint32_t t = base + lane;
    if (t < n) {                                      // level[] is written from the ring by a helper
        const uint32_t v = (uint32_t)acc - 1u;
        S.ring[t % LV_RING] = v;
        mymax = max(mymax, v - 1u);
    }
    // same wave, in-order LDS: the ring entries land before the count
    if (lane == 0) __hip_atomic_store(&S.done, x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return true;
}

// DBG (a development instantiation, not launched by the product): s_memtime sums -- dbg[0] resolver cycles waiting for a slot, [1] its
// cycles from slot to published chunk, [2] chunks it waited > 100 cycles for, [3] helpers' cycles
// from "chunks <= x-3 final" to the slot's flag, [4] chunks staged
template <bool DBG>
__global__ __launch_bounds__((LS_HELPERS + 1) * 64) void lv_staged_kernel(uint32_t n, uint32_t nchunks,
                                                                        const uint32_t *__restrict__ rec,
                                                                        const uint32_t *__restrict__ pred_off,
                                                                        const uint32_t *__restrict__ preds,
                                                                        uint32_t *level, uint32_t *__restrict__ info,
                                                                        unsigned long long *dbg, uint32_t solo)
{
    __shared__ LsShared S;
    const uint32_t w = wave_id(), lane = lane_id();
    if (threadIdx.x == 0) { S.done = 0; S.abort_flag = 0; S.maxlv = 0; S.ring[LS_ZERO] = 0; }
    if (threadIdx.x < LS_K) { S.slot[threadIdx.x].ready = 0; S.slot[threadIdx.x].dready = 0; }
    __syncthreads();
    uint32_t mymax = 0;
    if (w == 0) {
        __builtin_amdgcn_s_setprio(3);
        unsigned long long tw = 0, tc = 0, ns = 0, tg = 0, tm = 0;
        for (uint32_t x = 0; x < nchunks; ++x) {
            unsigned long long t0 = 0, t1 = 0;
            if (DBG) {
                t0 = __builtin_amdgcn_s_memtime();
                if (!ls_spin<false, false>(&S.slot[x % LS_K].ready, &S.abort_flag, (x + 1) << 9)) break;
                t1 = __builtin_amdgcn_s_memtime();
            }
            if (!ls_resolve(S, n, nchunks, x, pred_off, preds, level, lane, mymax, DBG ? &tm : nullptr)) break;
            if (DBG) {
                const unsigned long long t2 = __builtin_amdgcn_s_memtime();
                tw += t1 - t0; tc += t2 - t1; ns += (t1 - t0 > 100) ? 1 : 0;
                tg += tm - t1;
            }
        }
        if (DBG && lane == 0) { dbg[0] = tw; dbg[1] = tc; dbg[2] = ns; dbg[5] = tg; }
    } else if (!(solo && w == 4)) {
        // solo: wave 4 (the resolver's SIMD, waves being placed round-robin) stays idle
        LvRec ra, rb;
        const uint32_t H = solo ? LS_HELPERS - 1 : LS_HELPERS;
        const uint32_t h = w - 1 - (solo && w > 4 ? 1u : 0u);
        unsigned long long tp = 0, *st = DBG ? &tp : nullptr;
        uint32_t cnt = 0;
        lv_load(rec, h, nchunks, lane, ra);
        for (uint32_t x = h; x < nchunks; x += 2 * H) {
            lv_load(rec, x + H, nchunks, lane, rb);      // the next record, in flight meanwhile
            if (!ls_stage(S, n, x, ra, pred_off, preds, level, lane, st)) break;
            ++cnt;
            if (x + H >= nchunks) break;
            lv_load(rec, x + 2 * H, nchunks, lane, ra);
            if (!ls_stage(S, n, x + H, rb, pred_off, preds, level, lane, st)) break;
            ++cnt;
        }
        if (DBG && lane == 0) { atomicAdd(&dbg[3], tp); atomicAdd(&dbg[4], (unsigned long long)cnt); }
    }
    atomicMax(&S.maxlv, mymax);
    __syncthreads();
    // the chunks no helper stage copied (the last three)
    const uint32_t c0 = nchunks > 3 ? nchunks - 3 : 0u;
    if (!S.abort_flag && c0 + w < nchunks) {
        const uint32_t c = (c0 + w) * LC + lane;
        if (c < n) level[c] = S.ring[c % LV_RING] - 1u;
    }
    if (threadIdx.x == 0) {
        if (S.abort_flag) info[0] = 1 + S.done;
        info[1] = S.maxlv;
    }
}

} // namespace

void launch_wo_words_count(uint32_t n, const uint32_t *kd_key_off, const uint32_t *rd_val_off, uint32_t *cnt,
                           hipStream_t s)
{
    if (n == 0) return;
    uint32_t b = (n + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(wo_words_count_kernel, dim3(b), dim3(256), 0, s, n, kd_key_off, rd_val_off, cnt);
}

void launch_wo_bits(uint32_t n, const uint32_t *kd_key_off, const uint32_t *rd_val_off, const uint32_t *wo_off,
                    unsigned long long *words, hipStream_t s)
{
    if (n == 0) return;
    uint32_t b = (n + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(wo_bits_kernel, dim3(b), dim3(256), 0, s, n, kd_key_off, rd_val_off, wo_off, words);
}

void launch_wo_preds_count(const WaitingOnParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t b = (p.n + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(wo_preds_kernel<false>, dim3(b), dim3(256), 0, s, p);
}

void launch_wo_preds_fill(const WaitingOnParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t b = (p.n + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(wo_preds_kernel<true>, dim3(b), dim3(256), 0, s, p);
}

size_t levels_temp_bytes(uint32_t n)
{
    const size_t chunks = (n + LC - 1) / LC;
    return chunks * RC_WORDS * 4 + 64;
}

void launch_levels(uint32_t n, const uint32_t *pred_off, const uint32_t *preds, uint32_t *level, uint32_t *info,
                   void *temp, hipStream_t s)
{
    if (n == 0) return;
    const uint32_t nchunks = (n + LC - 1) / LC;
    uint32_t *rec = (uint32_t *)temp;
    hipLaunchKernelGGL(lv_closure_kernel, dim3((nchunks + 3) / 4), dim3(256), 0, s, n, nchunks, pred_off, preds, rec,
                       info, 2u);
    // the resolver alone on its SIMD (wave 4, which round-robin placement puts there, idles): 48.3 ->
    // 44.7 ms on config 5 (profiles/r04_b/levels_staged_ab.txt)
    hipLaunchKernelGGL(lv_staged_kernel<false>, dim3(1), dim3((LS_HELPERS + 1) * 64), 0, s, n, nchunks, rec, pred_off,
                       preds, level, info, nullptr, 1u);
}

} // namespace accord
