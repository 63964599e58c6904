// Multi-GPU ownership by stream segments (config 4).
//
// The node's stream is cut into G consecutive segments of TxnIds; rank r owns segment r =
// positions [a_r, b_r) of EVERY CommandStore (all 8G EvenSplit stores, local/ShardDistributor.java:
// 46-157) and computes the node-level deps of its txns in full -- no partial deps travel.  What a
// txn needs from before its segment is the CommandsForKey state at a_r: under the status-at-time
// model a txn i on key k starts at maxCommittedBefore = the last Write j < i - W of the key
// (local/CommandsForKey.java:620-645), and every entry before it is pruned for good for later txns
// (the analogue of withRedundantBefore, :1654-1684).  So the state at a_r is, per key, the run
// from the last Write before a_r - W on -- the carry a resident store keeps between batches
// (resident.hip).  It is built from small per-segment summaries instead of the whole prefix:
//
//   summary(q) = per key, the entries of segment q from its last Write before b_q - W on (all of
//                them when it has none): what any later txn can still reach of segment q's txns;
//   carry(r)   = per key, walk back from summary(r-1) towards summary(0), keeping every entry, up
//                to and including the first Write before a_r - W -- i.e. every summary entry at or
//                after the key's last Write before a_r - W over all of them.
// Both stay in stream order (no key sort): the carry heads the compute's pairs, whose stable
// bucketing sort makes the history key-major with each key's entries in stream order.
//
// An entry the single-store run would still reach at a_r lies at or after the key's last Write
// before a_r - W, so no Write of the key lies between it and b_q - W <= a_r - W: its own summary
// kept it (oracle or_cfk_fold == or_cfk_reachable, tests/test_segments.py).  The summaries are a few
// hundred thousand 8-byte entries per segment (~2 MB at config 4), exchanged with one all-gather
// (bench.py, accord_amd.segment_exchange: torch.distributed over RCCL/xGMI); the compute is then the
// resident store's own pipeline over [carry | segment].
#include "store_impl.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace {

constexpr uint32_t SEG_MAX_PARTS = 64;

inline uint32_t grid_for(uint64_t n)
{
    uint64_t b = (n + 255) / 256;
    return (uint32_t)(b < 1 ? 1 : b > 65535 ? 65535 : b);
}

constexpr uint32_t SEG_T = 256;                    // txns (summary) / entries (fold) per block
constexpr uint32_t SEG_HASH = 2048;                 // LDS slots of a block's (key -> last Write) table
constexpr uint32_t SEG_EMPTY = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t l2_load(const uint32_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// exclusive sum over the block's 256 threads (4 waves); *total = the block's sum
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *total)
{
    __shared__ uint32_t wsum[SEG_T / 64];
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    const uint32_t inc = wave_incl_scan(v);
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t before = 0, all = 0;
#pragma unroll
    for (uint32_t u = 0; u < SEG_T / 64; ++u) {
        before += u < w ? wsum[u] : 0u;
        all += wsum[u];
    }
    *total = all;
    return before + inc - v;
}

// A block's txns and their (txn, key) pairs staged in LDS with coalesced loads: key ordinals sk[],
// the local txn of every pair st[], the txns' kinds.  (A thread per txn walking its own pairs issues
// one dependent global load per pair -- 8 round trips per thread -- and strides 32 bytes across the
// lanes: the first form of these kernels spent 30 us per launch on that.)  A block whose pairs
// exceed the stage takes the per-thread walk.
constexpr uint32_t SEG_STAGE = 4096, SEG_PER = SEG_STAGE / SEG_T;
struct SegTile {
    uint32_t t0, t1, p0, np;
    bool staged;
};
__device__ __forceinline__ SegTile seg_stage(uint32_t t0, uint32_t t1, const uint32_t *__restrict__ key_off,
                                             const uint32_t *__restrict__ key_ord, const uint64_t *__restrict__ lsb,
                                             uint32_t *sk, uint16_t *st, uint8_t *skind)
{
    SegTile g{t0, t1, key_off[t0], 0u, false};
    g.np = key_off[t1] - g.p0;
    g.staged = g.np <= SEG_STAGE;
    const uint32_t t = t0 + threadIdx.x;
    if (t < t1) skind[threadIdx.x] = (uint8_t)((lsb[t] >> 1) & 7u);
    if (g.staged) {
        for (uint32_t i = threadIdx.x; i < g.np; i += SEG_T) sk[i] = key_ord[g.p0 + i];
        if (t < t1)
            for (uint32_t p = key_off[t], e = key_off[t + 1]; p < e; ++p) st[p - g.p0] = (uint16_t)threadIdx.x;
    }
    __syncthreads();
    return g;
}

__device__ __forceinline__ void seg_hash_put(uint32_t *hk, uint32_t *hv, uint32_t k, uint32_t v, uint32_t *lastw)
{
    for (uint32_t probe = 0, h = (k * 2654435761u) >> 21; probe < 16; ++probe) {
        const uint32_t slot = (h + probe) & (SEG_HASH - 1);
        const uint32_t prev = atomicCAS(&hk[slot], SEG_EMPTY, k);
        if (prev == SEG_EMPTY || prev == k) { atomicMax(&hv[slot], v); return; }
    }
    if (l2_load(&lastw[k]) < v) atomicMax(&lastw[k], v);        // table full around h: directly
}

// (last Write position before thr) + 1 per key, 0 = none.  A block's Writes first meet in an LDS
// table (a hot key's Writes of the block become one entry) and each key of the table then raises
// the global word once, skipped when an L2-coherent read already shows a later Write (every Write of
// the hottest key going to the global atomic took 0.5 ms: half the grid is resident at once and
// reads the word before any of them raised it).  The segment is walked in launches from its end
// (the last eighth, the eighth before, the quarter before, the first half): most keys have a Write
// in the latest txns, and once it has landed the older Writes of the key are read and skipped.
__global__ __launch_bounds__(SEG_T) void seg_lastw_kernel(uint32_t t_lo, uint32_t t_hi, uint32_t base, uint32_t thr,
                                                          const uint64_t *__restrict__ lsb,
                                                          const uint32_t *__restrict__ key_off,
                                                          const uint32_t *__restrict__ key_ord, uint32_t key_lo,
                                                          uint32_t nkeys, uint32_t *lastw)
{
    __shared__ uint32_t hk[SEG_HASH], hv[SEG_HASH], sk[SEG_STAGE];
    __shared__ uint16_t st[SEG_STAGE];
    __shared__ uint8_t skind[SEG_T];
    for (uint32_t i = threadIdx.x; i < SEG_HASH; i += SEG_T) { hk[i] = SEG_EMPTY; hv[i] = 0u; }
    const uint32_t t1 = t_hi - blockIdx.x * SEG_T;                 // blocks from the range's end
    const uint32_t t0 = t1 - t_lo > SEG_T ? t1 - SEG_T : t_lo;
    const SegTile g = seg_stage(t0, t1, key_off, key_ord, lsb, sk, st, skind);
    if (g.staged) {
        for (uint32_t i = threadIdx.x; i < g.np; i += SEG_T) {
            const uint32_t lt = st[i], gp = base + t0 + lt, k = sk[i] - key_lo;
            if (skind[lt] == 1u && gp < thr && k < nkeys) seg_hash_put(hk, hv, k, gp + 1u, lastw);
        }
    } else {
        const uint32_t t = t0 + threadIdx.x, gp = base + t;
        if (t < t1 && skind[threadIdx.x] == 1u && gp < thr)          // Writes bound maxCommittedBefore
            for (uint32_t p = key_off[t], e = key_off[t + 1]; p < e; ++p) {
                const uint32_t k = key_ord[p] - key_lo;
                if (k < nkeys) seg_hash_put(hk, hv, k, gp + 1u, lastw);
            }
    }
    __syncthreads();
    uint32_t kk[SEG_HASH / SEG_T], vv[SEG_HASH / SEG_T], cur[SEG_HASH / SEG_T];
#pragma unroll
    for (uint32_t j = 0; j < SEG_HASH / SEG_T; ++j) { kk[j] = hk[threadIdx.x + j * SEG_T]; vv[j] = hv[threadIdx.x + j * SEG_T]; }
#pragma unroll
    for (uint32_t j = 0; j < SEG_HASH / SEG_T; ++j) cur[j] = kk[j] != SEG_EMPTY ? l2_load(&lastw[kk[j]]) : ~0u;
#pragma unroll
    for (uint32_t j = 0; j < SEG_HASH / SEG_T; ++j)
        if (kk[j] != SEG_EMPTY && cur[j] < vv[j]) atomicMax(&lastw[kk[j]], vv[j]);
}

// Per block of SEG_T txns: the pairs a later txn can still reach (at or after the key's last Write
// before thr), each thread a contiguous run of the block's pairs (stream order): its kept count,
// and with WRITE the kept pairs written at the block's offset + the block's exclusive scan.
template <bool WRITE>
__global__ __launch_bounds__(SEG_T) void seg_keep_kernel(uint32_t n, uint32_t base, const uint64_t *__restrict__ lsb,
                                                         const uint32_t *__restrict__ key_off,
                                                         const uint32_t *__restrict__ key_ord, uint32_t key_lo,
                                                         uint32_t nkeys, const uint32_t *__restrict__ lastw,
                                                         uint32_t *__restrict__ tile_cnt, const uint32_t *__restrict__ tile_off,
                                                         uint32_t *__restrict__ out_key, uint32_t *__restrict__ out_ent)
{
    __shared__ uint32_t sk[SEG_STAGE];
    __shared__ uint16_t st[SEG_STAGE];
    __shared__ uint8_t skind[SEG_T];
    const uint32_t t0 = blockIdx.x * SEG_T, t1 = min(n, t0 + SEG_T);
    const SegTile g = seg_stage(t0, t1, key_off, key_ord, lsb, sk, st, skind);
    uint32_t c = 0, tot;
    if (g.staged) {
        const uint32_t per = (g.np + SEG_T - 1) / SEG_T, i0 = threadIdx.x * per;
        uint32_t keep = 0;                                     // bit j: pair i0 + j is kept
        uint32_t lw[SEG_PER];
#pragma unroll
        for (uint32_t j = 0; j < SEG_PER; ++j) {               // every gather issued before any is used
            const uint32_t i = i0 + j;
            const uint32_t k = (j < per && i < g.np) ? sk[i] - key_lo : nkeys;
            lw[j] = k < nkeys ? lastw[k] : ~0u;
        }
#pragma unroll
        for (uint32_t j = 0; j < SEG_PER; ++j) {
            const uint32_t i = i0 + j;
            if (j < per && i < g.np && base + t0 + st[i] + 1u >= lw[j]) keep |= 1u << j;
        }
        c = __popc(keep);
        if (!WRITE) {
            (void)block_excl_scan(c, &tot);
        } else {
            uint32_t o = tile_off[blockIdx.x] + block_excl_scan(c, &tot);
            for (; keep; keep &= keep - 1) {
                const uint32_t i = i0 + __ffs(keep) - 1, lt = st[i];
                out_key[o] = sk[i] - key_lo;
                out_ent[o] = ((uint32_t)skind[lt] << ENT_KIND_SHIFT) | (base + t0 + lt);
                ++o;
            }
        }
    } else {                                                   // a thread per txn over its own pairs
        const uint32_t t = t0 + threadIdx.x;
        uint32_t a = 0, e = 0;
        if (t < t1) { a = key_off[t]; e = key_off[t + 1]; }
        for (uint32_t p = a; p < e; ++p) {
            const uint32_t k = key_ord[p] - key_lo;
            c += (k < nkeys && base + t + 1u >= lastw[k]) ? 1u : 0u;
        }
        if (!WRITE) {
            (void)block_excl_scan(c, &tot);
        } else {
            uint32_t o = tile_off[blockIdx.x] + block_excl_scan(c, &tot);
            for (uint32_t p = a; p < e && c; ++p) {
                const uint32_t k = key_ord[p] - key_lo;
                if (k < nkeys && base + t + 1u >= lastw[k]) {
                    out_key[o] = k;
                    out_ent[o] = ((uint32_t)skind[threadIdx.x] << ENT_KIND_SHIFT) | (base + t);
                    ++o;
                }
            }
        }
    }
    if (!WRITE && threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
}

struct SegParts {
    const uint32_t *key[SEG_MAX_PARTS];
    const uint32_t *ent[SEG_MAX_PARTS];
    uint32_t off[SEG_MAX_PARTS + 1];   // prefix of the parts' entry counts: a flat index space
    uint32_t np;
};

__device__ __forceinline__ uint32_t seg_part_of(const SegParts &P, uint32_t x)
{
    uint32_t q = 0;
    while (q + 1 < P.np && P.off[q + 1] <= x) ++q;
    return q;
}

// The fold, over the concatenated parts (stream order, each part in stream order): the entries
// kept are those at or after LW(k) = the key's last Write before thr over all parts -- a walk back
// from the newest part to that Write keeps exactly them -- written in stream order (the compute's
// stable bucketing sort makes them key-major).
//   lw: LW(k) + 1 per key;  count: kept entries per block;  write: tile offset + block scan
__global__ __launch_bounds__(SEG_T) void seg_fold_lw_kernel(SegParts P, uint32_t thr, uint32_t *__restrict__ lw)
{
    const uint32_t x = blockIdx.x * SEG_T + threadIdx.x;
    if (x >= P.off[P.np]) return;
    const uint32_t q = seg_part_of(P, x), j = x - P.off[q];
    const uint32_t e = P.ent[q][j];
    if ((e >> ENT_KIND_SHIFT) == 1u && (e & ENT_TXN_MASK) < thr) atomicMax(&lw[P.key[q][j]], (e & ENT_TXN_MASK) + 1u);
}

__device__ __forceinline__ bool seg_fold_kept(const SegParts &P, uint32_t x, const uint32_t *__restrict__ lw,
                                              uint32_t &k, uint32_t &e)
{
    if (x >= P.off[P.np]) return false;
    const uint32_t q = seg_part_of(P, x), j = x - P.off[q];
    k = P.key[q][j];
    e = P.ent[q][j];
    return (e & ENT_TXN_MASK) + 1u >= lw[k];
}

__global__ __launch_bounds__(SEG_T) void seg_fold_count_kernel(SegParts P, const uint32_t *__restrict__ lw,
                                                               uint32_t *__restrict__ tile_cnt)
{
    uint32_t k, e, tot;
    const bool kept = seg_fold_kept(P, blockIdx.x * SEG_T + threadIdx.x, lw, k, e);
    (void)block_excl_scan(kept ? 1u : 0u, &tot);
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SEG_T) void seg_fold_write_kernel(SegParts P, const uint32_t *__restrict__ lw,
                                                               const uint32_t *__restrict__ tile_off,
                                                               uint32_t *__restrict__ out_key, uint32_t *__restrict__ out_ent)
{
    uint32_t k = 0, e = 0, tot;
    const bool kept = seg_fold_kept(P, blockIdx.x * SEG_T + threadIdx.x, lw, k, e);
    const uint32_t o = tile_off[blockIdx.x] + block_excl_scan(kept ? 1u : 0u, &tot);
    if (kept) {
        out_key[o] = k;
        out_ent[o] = e;
    }
}

void seg_record(accord_store *s, int i)
{
    if (!s->events) return;
    if (!s->seg_ev_created) {
        for (hipEvent_t &e : s->seg_ev) (void)hipEventCreate(&e);
        s->seg_ev_created = true;
    }
    (void)hipEventRecord(s->seg_ev[i], s->stream);
}

float seg_elapsed(accord_store *s, int a, int b)
{
    float ms = 0;
    if (s->events && s->seg_ev_created) (void)hipEventElapsedTime(&ms, s->seg_ev[a], s->seg_ev[b]);
    return ms;
}

} // namespace

namespace accord_impl {

void segment_destroy(accord_store *s)
{
    DevBuf *bufs[] = {&s->sg_lastw, &s->sg_flag, &s->sg_off, &s->sg_key, &s->sg_ent, &s->sg_cnt, &s->sg_koff,
                      &s->sg_word, &s->sg_lw};
    for (DevBuf *b : bufs) b->release();
    if (s->seg_ev_created)
        for (hipEvent_t &e : s->seg_ev) (void)hipEventDestroy(e);
    s->seg_ev_created = false;
}

} // namespace accord_impl

extern "C" {

int32_t accord_segment_begin(accord_store *s, uint32_t seg_base)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (!s->resident || s->cfg.window == ACCORD_WINDOW_NONE)
        return fail(s, ACCORD_ERR_STATE, "stream segments need a resident store with a status-at-time window");
    if (seg_base >= (1u << 29)) return fail(s, ACCORD_ERR_CAPACITY, "segment base %u exceeds 2^29", seg_base);
    int32_t rc = accord_store_reset(s);
    if (rc) return rc;
    s->next_global = seg_base;
    s->seg_base = seg_base;
    s->seg_active = true;
    s->seg_sum_n = 0;
    s->seg_sum_ok = false;
    return ACCORD_OK;
}

int32_t accord_segment_summary(accord_store *s, accord_cfk_part *out)
{
    if (!s || !out) return fail(s, ACCORD_ERR_ARG, "null argument");
    std::memset(out, 0, sizeof(*out));
    if (!s->seg_active) return fail(s, ACCORD_ERR_STATE, "accord_segment_summary before accord_segment_begin");
    if (!s->has_batch) return fail(s, ACCORD_ERR_STATE, "accord_segment_summary before accord_batch_upload");
    if (s->R || s->n_range_txns || s->has_exec || s->user_txn_index)
        return fail(s, ACCORD_ERR_ARG, "stream segments take PreAccept batches of key txns (no ranges, executeAt or txn_index)");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    const uint32_t n = s->n, P = s->P, base = s->seg_base;
    const uint32_t nkeys = s->cfg.key_hi - s->cfg.key_lo;
    const uint32_t end = base + n;
    const uint32_t thr = end > s->cfg.window ? end - s->cfg.window : 0u;
    hipStream_t st = s->stream;
    seg_record(s, 0);
    const uint32_t tiles = (n + SEG_T - 1) / SEG_T;
    HIPCHECK(s, s->sg_lastw.ensure((size_t)nkeys * 4 + 4));
    HIPCHECK(s, s->sg_flag.ensure((size_t)tiles * 4 + 16));          // per block: kept pairs
    HIPCHECK(s, s->sg_off.ensure((size_t)tiles * 4 + 16));           // ... and their offsets
    HIPCHECK(s, s->sg_word.ensure(64));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(std::max(tiles, 1u)), st));
    unsigned long long *dtot = s->sg_word.as<unsigned long long>();
    uint64_t T = 0;
    if (n && P) {
        HIPCHECK(s, hipMemsetAsync(s->sg_lastw.p, 0, (size_t)nkeys * 4, st));
        const uint32_t cut[5] = {0u, n / 2, n / 4 * 3, n / 8 * 7, n};
        for (int c = 3; c >= 0; --c) {                 // from the segment's end
            if (cut[c + 1] <= cut[c]) continue;
            const uint32_t blocks = (cut[c + 1] - cut[c] + SEG_T - 1) / SEG_T;
            hipLaunchKernelGGL(seg_lastw_kernel, dim3(blocks), dim3(SEG_T), 0, st, cut[c], cut[c + 1], base, thr,
                               s->lsb.as<uint64_t>(), s->key_off.as<uint32_t>(), s->key_ord.as<uint32_t>(),
                               s->cfg.key_lo, nkeys, s->sg_lastw.as<uint32_t>());
        }
        hipLaunchKernelGGL(seg_keep_kernel<false>, dim3(tiles), dim3(SEG_T), 0, st, n, base, s->lsb.as<uint64_t>(),
                           s->key_off.as<uint32_t>(), s->key_ord.as<uint32_t>(), s->cfg.key_lo, nkeys,
                           s->sg_lastw.as<uint32_t>(), s->sg_flag.as<uint32_t>(), nullptr, nullptr, nullptr);
        accord::exclusive_scan_u32(s->sg_flag.as<uint32_t>(), s->sg_off.as<uint32_t>(), tiles, dtot, s->scan_tmp.p, st);
        HIPCHECK(s, hipMemcpyAsync(&s->pinned->totals[9], dtot, 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(s, hipStreamSynchronize(st));
        T = s->pinned->totals[9];
    }
    HIPCHECK(s, s->sg_key.ensure(T * 4 + 4));
    HIPCHECK(s, s->sg_ent.ensure(T * 4 + 4));
    if (T)   // in stream order (txn-major): the fold and the compute's stable sort need no key order
        hipLaunchKernelGGL(seg_keep_kernel<true>, dim3(tiles), dim3(SEG_T), 0, st, n, base, s->lsb.as<uint64_t>(),
                           s->key_off.as<uint32_t>(), s->key_ord.as<uint32_t>(), s->cfg.key_lo, nkeys,
                           s->sg_lastw.as<uint32_t>(), nullptr, s->sg_off.as<uint32_t>(), s->sg_key.as<uint32_t>(),
                           s->sg_ent.as<uint32_t>());
    seg_record(s, 1);
    // the summary may be read by another store's stream (one-GPU simulation) or a collective: ready
    HIPCHECK(s, hipStreamSynchronize(st));
    HIPCHECK(s, hipGetLastError());
    s->seg_sum_n = T;
    s->seg_sum_ok = true;
    s->seg_summary_ms = seg_elapsed(s, 0, 1);
    out->n = T;
    out->key = s->sg_key.as<uint32_t>();
    out->ent = s->sg_ent.as<uint32_t>();
    return ACCORD_OK;
}

int32_t accord_segment_summary_copy(accord_store *s, uint32_t *key_dst, uint32_t *ent_dst, uint64_t cap)
{
    if (!s || !key_dst || !ent_dst) return fail(s, ACCORD_ERR_ARG, "null argument");
    if (!s->seg_sum_ok) return fail(s, ACCORD_ERR_STATE, "accord_segment_summary_copy before accord_segment_summary");
    if (cap < s->seg_sum_n) return fail(s, ACCORD_ERR_CAPACITY, "summary of %llu entries, buffers of %llu",
                                        (unsigned long long)s->seg_sum_n, (unsigned long long)cap);
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    if (s->seg_sum_n) {
        // device or host destination (hipMemcpyDefault: a host-staged exchange takes host buffers)
        HIPCHECK(s, hipMemcpyAsync(key_dst, s->sg_key.p, s->seg_sum_n * 4, hipMemcpyDefault, s->stream));
        HIPCHECK(s, hipMemcpyAsync(ent_dst, s->sg_ent.p, s->seg_sum_n * 4, hipMemcpyDefault, s->stream));
    }
    HIPCHECK(s, hipStreamSynchronize(s->stream));
    return ACCORD_OK;
}

int32_t accord_segment_carry(accord_store *s, uint32_t nparts, const accord_cfk_part *parts)
{
    if (!s || (nparts && !parts)) return fail(s, ACCORD_ERR_ARG, "null argument");
    if (!s->seg_active) return fail(s, ACCORD_ERR_STATE, "accord_segment_carry before accord_segment_begin");
    if (!s->has_batch) return fail(s, ACCORD_ERR_STATE, "accord_segment_carry before accord_batch_upload");
    if (nparts > SEG_MAX_PARTS) return fail(s, ACCORD_ERR_CAPACITY, "%u earlier segments (up to %u)", nparts, SEG_MAX_PARTS);
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    const uint32_t nkeys = s->cfg.key_hi - s->cfg.key_lo;
    const uint32_t thr = s->seg_base > s->cfg.window ? s->seg_base - s->cfg.window : 0u;
    hipStream_t st = s->stream;
    SegParts sp{};
    uint64_t cap = 0;
    for (uint32_t q = 0; q < nparts; ++q) {
        if (parts[q].n && (!parts[q].key || !parts[q].ent)) return fail(s, ACCORD_ERR_ARG, "part %u without arrays", q);
        sp.key[q] = parts[q].key; sp.ent[q] = parts[q].ent; sp.off[q] = (uint32_t)cap;
        cap += parts[q].n;
        if (cap >= (1ull << 28)) return fail(s, ACCORD_ERR_CAPACITY, "carry of up to %llu entries exceeds 2^28",
                                             (unsigned long long)cap);
    }
    sp.off[nparts] = (uint32_t)cap;
    sp.np = nparts;
    seg_record(s, 2);
    const uint32_t tiles = (uint32_t)((cap + SEG_T - 1) / SEG_T);
    HIPCHECK(s, s->sg_lw.ensure((size_t)nkeys * 4 + 4));
    HIPCHECK(s, s->sg_cnt.ensure((size_t)tiles * 4 + 16));
    HIPCHECK(s, s->sg_koff.ensure((size_t)tiles * 4 + 16));
    HIPCHECK(s, s->sg_word.ensure(64));
    HIPCHECK(s, s->cy_key.ensure(cap * 4 + 4));
    HIPCHECK(s, s->cy_ent.ensure(cap * 4 + 4));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(std::max(tiles, 1u)), st));
    unsigned long long *dw = s->sg_word.as<unsigned long long>();   // [0] total, [1] kinds
    accord::FillList fl;
    fl.add(dw, 16, 0u);
    if (cap) fl.add(s->sg_lw.p, (size_t)nkeys * 4, 0u);
    accord::launch_fill_words(fl, st);
    if (cap) {
        hipLaunchKernelGGL(seg_fold_lw_kernel, dim3(tiles), dim3(SEG_T), 0, st, sp, thr, s->sg_lw.as<uint32_t>());
        hipLaunchKernelGGL(seg_fold_count_kernel, dim3(tiles), dim3(SEG_T), 0, st, sp, s->sg_lw.as<uint32_t>(),
                           s->sg_cnt.as<uint32_t>());
        accord::exclusive_scan_u32(s->sg_cnt.as<uint32_t>(), s->sg_koff.as<uint32_t>(), tiles, dw, s->scan_tmp.p, st);
        hipLaunchKernelGGL(seg_fold_write_kernel, dim3(tiles), dim3(SEG_T), 0, st, sp, s->sg_lw.as<uint32_t>(),
                           s->sg_koff.as<uint32_t>(), s->cy_key.as<uint32_t>(), s->cy_ent.as<uint32_t>());
    }
    seg_record(s, 3);
    HIPCHECK(s, hipMemcpyAsync(&s->pinned->totals[8], dw, 16, hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    HIPCHECK(s, hipGetLastError());
    // the store now stands at the start of its segment with the CommandsForKey state there; the
    // uploaded segment can be computed (again: a bench step repeats carry + compute)
    s->carry_n = cap ? (uint32_t)s->pinned->totals[8] : 0u;
    // every kind may be carried (kinds_present only selects range-txn kernels, which segments never run)
    s->hist_kinds = cap ? 0xFFu : 0u;
    s->next_global = s->seg_base;
    s->seg_carry_ok = true;
    s->has_prev = false;
    s->rc_n = 0;
    s->b_registered = false;
    s->computed = false;
    ++s->carry_version;
    s->seg_carry_ms = seg_elapsed(s, 2, 3);
    return ACCORD_OK;
}

int32_t accord_segment_timing(accord_store *s, float *summary_ms, float *carry_ms)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (summary_ms) *summary_ms = s->seg_summary_ms;
    if (carry_ms) *carry_ms = s->seg_carry_ms;
    return ACCORD_OK;
}

} // extern "C"
