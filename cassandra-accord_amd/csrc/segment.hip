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
//                to and including the first Write before a_r - W.
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

int bits_for(uint32_t maxval)
{
    int b = 0;
    while (b < 32 && (maxval >> b) != 0) ++b;
    return b < 1 ? 1 : b;
}

// (last Write position before thr) + 1 per key, 0 = none.  Txns are walked from the segment's end,
// so the newest Writes land first and older ones see a larger value and skip their atomic (the
// hottest key's Writes would otherwise all contend on one word).
__global__ __launch_bounds__(256) void seg_lastw_kernel(uint32_t n, uint32_t base, uint32_t thr,
                                                        const uint64_t *__restrict__ lsb,
                                                        const uint32_t *__restrict__ key_off,
                                                        const uint32_t *__restrict__ key_ord, uint32_t key_lo,
                                                        uint32_t nkeys, uint32_t *lastw)
{
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= n) return;
    const uint32_t t = n - 1 - x;
    const uint32_t gp = base + t;
    if (gp >= thr) return;
    if (((lsb[t] >> 1) & 7u) != 1u) return;          // Writes only bound maxCommittedBefore
    const uint32_t v = gp + 1;
    for (uint32_t p = key_off[t], e = key_off[t + 1]; p < e; ++p) {
        const uint32_t k = key_ord[p] - key_lo;
        if (k >= nkeys) continue;
        if (*(volatile const uint32_t *)&lastw[k] < v) atomicMax(&lastw[k], v);
    }
}

// per (txn, key) pair: kept in the summary iff at or after the key's last Write before thr
__global__ __launch_bounds__(256) void seg_flag_kernel(uint32_t n, uint32_t base, const uint32_t *__restrict__ key_off,
                                                       const uint32_t *__restrict__ key_ord, uint32_t key_lo,
                                                       uint32_t nkeys, const uint32_t *__restrict__ lastw,
                                                       uint32_t *__restrict__ flag)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t gp = base + t;
    for (uint32_t p = key_off[t], e = key_off[t + 1]; p < e; ++p) {
        const uint32_t k = key_ord[p] - key_lo;
        flag[p] = (k < nkeys && gp + 1 >= lastw[k]) ? 1u : 0u;
    }
}

__global__ __launch_bounds__(256) void seg_scatter_kernel(uint32_t n, uint32_t base, const uint64_t *__restrict__ lsb,
                                                          const uint32_t *__restrict__ key_off,
                                                          const uint32_t *__restrict__ key_ord, uint32_t key_lo,
                                                          const uint32_t *__restrict__ flag,
                                                          const uint32_t *__restrict__ off, uint32_t *__restrict__ out_key,
                                                          uint32_t *__restrict__ out_ent)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t ent = ((uint32_t)((lsb[t] >> 1) & 7u) << ENT_KIND_SHIFT) | (base + t);
    for (uint32_t p = key_off[t], e = key_off[t + 1]; p < e; ++p)
        if (flag[p]) {
            const uint32_t o = off[p];
            out_key[o] = key_ord[p] - key_lo;
            out_ent[o] = ent;
        }
}

struct SegParts {
    const uint32_t *key[SEG_MAX_PARTS];
    const uint32_t *ent[SEG_MAX_PARTS];
    uint32_t n[SEG_MAX_PARTS];
    uint32_t np;
};

// Per key: walk the parts from the newest back, keeping every entry, up to and including the first
// Write before thr.  Count pass (cnt) and fill pass (entries written backwards from off[k + 1], so
// they land in ascending position order).  kinds |= the entry kinds kept.
template <bool FILL>
__global__ __launch_bounds__(256) void seg_fold_kernel(SegParts P, uint32_t nkeys, uint32_t thr,
                                                       uint32_t *__restrict__ cnt, const uint32_t *__restrict__ off,
                                                       uint32_t *__restrict__ out_key, uint32_t *__restrict__ out_ent,
                                                       uint32_t *kinds)
{
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nkeys) return;
    uint32_t c = 0, w = FILL ? off[k + 1] : 0u, km = 0;
    bool done = false;
    for (int q = (int)P.np - 1; q >= 0 && !done; --q) {
        const uint32_t *K = P.key[q];
        uint32_t lo = 0, hi = P.n[q];
        while (lo < hi) {                              // first entry of key > k
            const uint32_t m = (lo + hi) >> 1;
            if (K[m] <= k) lo = m + 1; else hi = m;
        }
        const uint32_t *E = P.ent[q];
        for (uint32_t j = lo; j > 0 && K[j - 1] == k; --j) {
            const uint32_t e = E[j - 1];
            ++c;
            if (FILL) {
                --w;
                out_key[w] = k;
                out_ent[w] = e;
                km |= 1u << (e >> ENT_KIND_SHIFT);
            }
            if ((e >> ENT_KIND_SHIFT) == 1u && (e & ENT_TXN_MASK) < thr) { done = true; break; }
        }
    }
    if (!FILL) cnt[k] = c;
    else if (km) atomicOr(kinds, km);
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
    DevBuf *bufs[] = {&s->sg_lastw, &s->sg_flag, &s->sg_off, &s->sg_ckey, &s->sg_cent, &s->sg_key, &s->sg_ent,
                      &s->sg_tmp0, &s->sg_tmp1, &s->sg_tmp2, &s->sg_tmp3, &s->sg_radix, &s->sg_cnt, &s->sg_koff, &s->sg_word};
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
    HIPCHECK(s, s->sg_lastw.ensure((size_t)nkeys * 4 + 4));
    HIPCHECK(s, s->sg_flag.ensure((size_t)P * 4 + 16));
    HIPCHECK(s, s->sg_off.ensure((size_t)P * 4 + 16));
    HIPCHECK(s, s->sg_word.ensure(64));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(std::max(P, 1u)), st));
    unsigned long long *dtot = s->sg_word.as<unsigned long long>();
    uint64_t T = 0;
    if (n && P) {
        HIPCHECK(s, hipMemsetAsync(s->sg_lastw.p, 0, (size_t)nkeys * 4, st));
        hipLaunchKernelGGL(seg_lastw_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, base, thr, s->lsb.as<uint64_t>(),
                           s->key_off.as<uint32_t>(), s->key_ord.as<uint32_t>(), s->cfg.key_lo, nkeys,
                           s->sg_lastw.as<uint32_t>());
        hipLaunchKernelGGL(seg_flag_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, base, s->key_off.as<uint32_t>(),
                           s->key_ord.as<uint32_t>(), s->cfg.key_lo, nkeys, s->sg_lastw.as<uint32_t>(),
                           s->sg_flag.as<uint32_t>());
        accord::exclusive_scan_u32(s->sg_flag.as<uint32_t>(), s->sg_off.as<uint32_t>(), P, dtot, s->scan_tmp.p, st);
        HIPCHECK(s, hipMemcpyAsync(&s->pinned->totals[9], dtot, 8, hipMemcpyDeviceToHost, st));
        HIPCHECK(s, hipStreamSynchronize(st));
        T = s->pinned->totals[9];
    }
    HIPCHECK(s, s->sg_ckey.ensure(T * 4 + 4)); HIPCHECK(s, s->sg_cent.ensure(T * 4 + 4));
    HIPCHECK(s, s->sg_key.ensure(T * 4 + 4)); HIPCHECK(s, s->sg_ent.ensure(T * 4 + 4));
    HIPCHECK(s, s->sg_tmp0.ensure(T * 4 + 4)); HIPCHECK(s, s->sg_tmp1.ensure(T * 4 + 4));
    HIPCHECK(s, s->sg_tmp2.ensure(T * 4 + 4)); HIPCHECK(s, s->sg_tmp3.ensure(T * 4 + 4));
    if (T) {
        hipLaunchKernelGGL(seg_scatter_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, base, s->lsb.as<uint64_t>(),
                           s->key_off.as<uint32_t>(), s->key_ord.as<uint32_t>(), s->cfg.key_lo,
                           s->sg_flag.as<uint32_t>(), s->sg_off.as<uint32_t>(), s->sg_ckey.as<uint32_t>(),
                           s->sg_cent.as<uint32_t>());
        // key-major, positions ascending within a key: a stable sort by key of the txn-major entries
        HIPCHECK(s, s->sg_radix.ensure(accord::radix_sort_temp_bytes((uint32_t)T)));
        HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(std::max<uint32_t>(
                                                  P, accord::radix_sort_scan_len((uint32_t)T))), st));
        accord::radix_sort_pairs(s->sg_ckey.as<uint32_t>(), nullptr, s->sg_key.as<uint32_t>(), s->sg_tmp0.as<uint32_t>(),
                                 s->sg_tmp1.as<uint32_t>(), s->sg_tmp2.as<uint32_t>(), s->sg_cent.as<uint32_t>(),
                                 s->sg_ent.as<uint32_t>(), s->sg_tmp3.as<uint32_t>(), (uint32_t)T, bits_for(nkeys - 1),
                                 s->sg_radix.p, s->scan_tmp.p, st);
    }
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
        if (parts[q].n >= (1ull << 32)) return fail(s, ACCORD_ERR_CAPACITY, "part %u over 2^32 entries", q);
        sp.key[q] = parts[q].key; sp.ent[q] = parts[q].ent; sp.n[q] = (uint32_t)parts[q].n;
        cap += parts[q].n;
    }
    sp.np = nparts;
    if (cap >= (1ull << 28)) return fail(s, ACCORD_ERR_CAPACITY, "carry of up to %llu entries exceeds 2^28",
                                         (unsigned long long)cap);
    seg_record(s, 2);
    HIPCHECK(s, s->sg_cnt.ensure((size_t)nkeys * 4 + 4));
    HIPCHECK(s, s->sg_koff.ensure(((size_t)nkeys + 1) * 4));
    HIPCHECK(s, s->sg_word.ensure(64));
    HIPCHECK(s, s->cy_key.ensure(cap * 4 + 4));
    HIPCHECK(s, s->cy_ent.ensure(cap * 4 + 4));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(nkeys), st));
    unsigned long long *dw = s->sg_word.as<unsigned long long>();   // [0] total, [1] kinds
    HIPCHECK(s, hipMemsetAsync(dw, 0, 16, st));
    if (nparts) {
        hipLaunchKernelGGL(seg_fold_kernel<false>, dim3(grid_for(nkeys)), dim3(256), 0, st, sp, nkeys, thr,
                           s->sg_cnt.as<uint32_t>(), nullptr, nullptr, nullptr, nullptr);
        accord::exclusive_scan_u32(s->sg_cnt.as<uint32_t>(), s->sg_koff.as<uint32_t>(), nkeys, dw, s->scan_tmp.p, st);
        hipLaunchKernelGGL(seg_fold_kernel<true>, dim3(grid_for(nkeys)), dim3(256), 0, st, sp, nkeys, thr,
                           s->sg_cnt.as<uint32_t>(), s->sg_koff.as<uint32_t>(), s->cy_key.as<uint32_t>(),
                           s->cy_ent.as<uint32_t>(), (uint32_t *)(dw + 1));
    }
    seg_record(s, 3);
    HIPCHECK(s, hipMemcpyAsync(&s->pinned->totals[8], dw, 16, hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    HIPCHECK(s, hipGetLastError());
    // the store now stands at the start of its segment with the CommandsForKey state there; the
    // uploaded segment can be computed (again: a bench step repeats carry + compute)
    s->carry_n = nparts ? (uint32_t)s->pinned->totals[8] : 0u;
    s->hist_kinds = nparts ? (uint32_t)s->pinned->totals[9] : 0u;
    s->next_global = s->seg_base;
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
