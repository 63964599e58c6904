// Multi-store / multi-GPU union of per-store PartialDeps.
//
// accord_deps_merge       : union of G per-store partial KeyDeps of the same txns (device views,
//                           e.g. several stores on one GPU) -- PreAccept.reduce
//                           (messages/PreAccept.java:140-156) for key-disjoint stores.
// accord_deps_exchange_merge : the multi-GPU form.  Every rank (one GPU, a contiguous block of the
//                           8*G EvenSplit stores, local/ShardDistributor.java:46-157) has computed
//                           its stores' partial KeyDeps for the txns intersecting them; txn i's
//                           union is owned by rank floor(i*G/N).  One RCCL exchange (grouped
//                           send/recv over xGMI) moves every partial to its owner, which unions
//                           the G parts on device.
#include "store_impl.h"

#include <rccl/rccl.h>

#include <array>
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

namespace {

struct Part {
    const uint32_t *key_off, *keys, *val_off, *vals, *k2v_off;
    const int32_t *k2v;
};

} // namespace

struct ShardComm {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    DevBuf ind, cscan, exp[6], bnd, counts, allcounts, recv;
    unsigned long long *total = nullptr;
    DevBuf total_buf, flag;
};

namespace accord_impl {

void shard_comm_destroy(accord_store *s)
{
    if (!s || !s->comm) return;
    ShardComm *c = s->comm;
    if (c->comm) (void)ncclCommDestroy(c->comm);
    DevBuf *bufs[] = {&c->ind, &c->cscan, &c->exp[0], &c->exp[1], &c->exp[2], &c->exp[3], &c->exp[4], &c->exp[5],
                      &c->bnd, &c->counts, &c->allcounts, &c->recv, &c->total_buf, &c->flag};
    for (DevBuf *b : bufs) b->release();
    delete c;
    s->comm = nullptr;
}

} // namespace accord_impl

namespace {

// Union of G aligned parts of n txns (global positions txn_lo..txn_lo+n-1) into s->m_*.
int32_t merge_parts(accord_store *s, const std::vector<Part> &parts, uint32_t n, uint32_t txn_lo)
{
    const uint32_t G = (uint32_t)parts.size();
    if (G == 0 || G > 64) return fail(s, ACCORD_ERR_CAPACITY, "merge of %u parts (1..64 supported)", G);
    hipStream_t st = s->stream;
    const size_t n1 = (size_t)n + 1;
    HIPCHECK(s, s->m_ptrs.ensure((size_t)6 * G * sizeof(void *)));
    HIPCHECK(s, s->m_cnt_keys.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->m_cnt_vals.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->m_cnt_k2v.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->m_key_off.ensure(n1 * 4));
    HIPCHECK(s, s->m_val_off.ensure(n1 * 4));
    HIPCHECK(s, s->m_k2v_off.ensure(n1 * 4));
    HIPCHECK(s, s->m_zero.ensure(n1 * 4));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(n), s->stream));
    HIPCHECK(s, s->status_totals.ensure(sizeof(HostTotals)));
    std::vector<const void *> tbl(6 * (size_t)G);
    for (uint32_t g = 0; g < G; ++g) {
        tbl[0 * G + g] = parts[g].key_off; tbl[1 * G + g] = parts[g].keys;
        tbl[2 * G + g] = parts[g].val_off; tbl[3 * G + g] = parts[g].vals;
        tbl[4 * G + g] = parts[g].k2v_off; tbl[5 * G + g] = parts[g].k2v;
    }
    HIPCHECK(s, hipMemcpyAsync(s->m_ptrs.p, tbl.data(), tbl.size() * sizeof(void *), hipMemcpyHostToDevice, st));
    const void *const *ptab = (const void *const *)s->m_ptrs.p;
    accord::MergeParams mp{};
    mp.n = n; mp.G = G; mp.txn_lo = txn_lo;
    mp.key_off = (const uint32_t *const *)(ptab + 0 * G); mp.keys = (const uint32_t *const *)(ptab + 1 * G);
    mp.val_off = (const uint32_t *const *)(ptab + 2 * G); mp.vals = (const uint32_t *const *)(ptab + 3 * G);
    mp.k2v_off = (const uint32_t *const *)(ptab + 4 * G); mp.k2v = (const int32_t *const *)(ptab + 5 * G);
    mp.cnt_keys = s->m_cnt_keys.as<uint32_t>(); mp.cnt_vals = s->m_cnt_vals.as<uint32_t>(); mp.cnt_k2v = s->m_cnt_k2v.as<uint32_t>();
    HostTotals *dev = s->status_totals.as<HostTotals>();
    mp.status = &dev->status;
    HIPCHECK(s, hipMemsetAsync(dev, 0xFF, sizeof(HostTotals), st));
    HIPCHECK(s, hipMemsetAsync(&dev->status.overflow, 0, sizeof(uint32_t), st));
    HIPCHECK(s, hipMemsetAsync(s->m_zero.p, 0, n1 * 4, st));
    accord::launch_merge_count(mp, st);
    accord::exclusive_scan_u32(mp.cnt_keys, s->m_key_off.as<uint32_t>(), n, &dev->totals[0], s->scan_tmp.p, st);
    accord::exclusive_scan_u32(mp.cnt_vals, s->m_val_off.as<uint32_t>(), n, &dev->totals[1], s->scan_tmp.p, st);
    accord::exclusive_scan_u32(mp.cnt_k2v, s->m_k2v_off.as<uint32_t>(), n, &dev->totals[2], s->scan_tmp.p, st);
    HIPCHECK(s, hipMemcpyAsync(s->pinned, dev, sizeof(HostTotals), hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    const HostTotals &h = *s->pinned;
    if (h.status.first != ~0ull) {
        const uint32_t where = (uint32_t)(h.status.first >> 32);
        const int32_t code = -(int32_t)(uint32_t)(h.status.first & 0xFFFFFFFFu);
        return fail(s, code, "merge: parts have overlapping or unordered keys (txn %u)", where);
    }
    if (h.status.overflow)
        return fail(s, ACCORD_ERR_CAPACITY, "merge: %u txns exceed the union capacity (first: txn %u)",
                    h.status.overflow, h.status.overflow_first);
    s->m_tot_keys = h.totals[0]; s->m_tot_vals = h.totals[1]; s->m_tot_k2v = h.totals[2];
    HIPCHECK(s, s->m_keys.ensure(s->m_tot_keys * 4));
    HIPCHECK(s, s->m_vals.ensure(s->m_tot_vals * 4));
    HIPCHECK(s, s->m_k2v.ensure(s->m_tot_k2v * 4));
    mp.out_key_off = s->m_key_off.as<uint32_t>(); mp.out_val_off = s->m_val_off.as<uint32_t>();
    mp.out_k2v_off = s->m_k2v_off.as<uint32_t>();
    mp.out_keys = s->m_keys.as<uint32_t>(); mp.out_vals = s->m_vals.as<uint32_t>(); mp.out_k2v = s->m_k2v.as<int32_t>();
    accord::launch_merge_fill(mp, st);
    HIPCHECK(s, hipStreamSynchronize(st));
    HIPCHECK(s, hipGetLastError());
    s->m_n = n;
    s->m_txn_lo = txn_lo;
    s->merged = true;
    s->ds_cur = -1;
    s->wo_done = false;
    s->computed = true;
    return ACCORD_OK;
}

// Parts with RangeDeps: the stores' RangeDeps share range keys (a range txn intersecting several
// stores' key blocks appears in each), so their union is RelationMultiMap.linearUnion, not the
// concatenation the key-disjoint merge relies on.  Both sides go through accord_deps_union; the
// result becomes the store's current deps.
int32_t union_general(accord_store *s, uint32_t nparts, const accord_deps *parts)
{
    const int32_t rc = accord_deps_union(s, nparts, parts);
    if (rc) return rc;
    s->merged = true;
    return ACCORD_OK;
}

#define NCCLGROUPCHECK(s, expr)                                                                  \
    do {                                                                                         \
        ncclResult_t r_ = (expr);                                                                \
        if (r_ != ncclSuccess) {                                                                 \
            (void)ncclGroupEnd();                                                                \
            return fail((s), ACCORD_ERR_HIP, "%s: %s", #expr, ncclGetErrorString(r_));           \
        }                                                                                        \
    } while (0)

#define NCCLCHECK(s, expr)                                                                       \
    do {                                                                                         \
        ncclResult_t r_ = (expr);                                                                \
        if (r_ != ncclSuccess) return fail((s), ACCORD_ERR_HIP, "%s: %s", #expr, ncclGetErrorString(r_)); \
    } while (0)

} // namespace

extern "C" {

int32_t accord_deps_merge(accord_store *s, uint32_t nparts, const accord_deps *parts, uint32_t txn_lo)
{
    if (!s || !parts || nparts == 0) return fail(s, ACCORD_ERR_ARG, "accord_deps_merge: bad arguments");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    const uint32_t n = parts[0].n;
    std::vector<Part> ps(nparts);
    bool ranges = false;
    for (uint32_t g = 0; g < nparts; ++g) {
        if (parts[g].n != n) return fail(s, ACCORD_ERR_ARG, "merge parts cover different txn counts");
        ranges = ranges || parts[g].rd_rngs_total || parts[g].rd_vals_total;
        ps[g] = Part{parts[g].kd_key_off, parts[g].kd_keys, parts[g].kd_val_off, parts[g].kd_vals,
                     parts[g].kd_k2v_off, parts[g].kd_k2v};
    }
    // RangeDeps, more parts than the merge kernel's lanes, or a txn past its union capacity: the
    // general union (linearUnion on both sides gives the same sets for key-disjoint parts)
    if (ranges || nparts > 64) return union_general(s, nparts, parts);
    const int32_t rc = merge_parts(s, ps, n, txn_lo);
    if (rc == ACCORD_ERR_CAPACITY) return union_general(s, nparts, parts);
    return rc;
}

int32_t accord_comm_unique_id(void *id128)
{
    if (!id128) return fail(nullptr, ACCORD_ERR_ARG, "null id");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(nullptr, ACCORD_ERR_HIP, "ncclGetUniqueId: %s", ncclGetErrorString(r));
    std::memcpy(id128, &id, sizeof(id));
    return ACCORD_OK;
}

int32_t accord_comm_init(accord_store *s, int32_t nranks, int32_t rank, const void *id128)
{
    if (!s || !id128 || nranks < 1 || rank < 0 || rank >= nranks) return fail(s, ACCORD_ERR_ARG, "accord_comm_init: bad arguments");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    accord_impl::shard_comm_destroy(s);
    ShardComm *c = new (std::nothrow) ShardComm();
    if (!c) return fail(s, ACCORD_ERR_OOM, "out of host memory");
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof(id));
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        delete c;
        return fail(s, ACCORD_ERR_HIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    if (c->flag.ensure(16) != hipSuccess) {
        (void)ncclCommDestroy(c->comm);
        delete c;
        return fail(s, ACCORD_ERR_OOM, "accord_comm_init: flag buffer");
    }
    c->nranks = nranks;
    c->rank = rank;
    s->comm = c;
    return ACCORD_OK;
}

int32_t accord_deps_exchange_merge(accord_store *s, uint32_t n_total)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (!s->comm) return fail(s, ACCORD_ERR_STATE, "accord_deps_exchange_merge before accord_comm_init");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    ShardComm *c = s->comm;
    const uint32_t G = (uint32_t)c->nranks, me = (uint32_t)c->rank, n = s->n;
    hipStream_t st = s->stream;
    // Offset arrays (KeyDeps keys / values / keysToTxnIds, RangeDeps ranges / values /
    // rangesToTxnIds) and the data arrays each indexes (ranges: starts and ends).
    constexpr int NA = 6, ND = 7;
    static const int grp[ND] = {0, 1, 2, 3, 3, 4, 5};

    // Every rank must reach the same collectives: the local checks and allocations run first, then
    // one all-reduce (max) of their status agrees whether every rank goes ahead; a rank that failed
    // keeps its own message, the others report that a peer failed.
    std::vector<uint32_t> bnd(NA * (G + 1));
    uint32_t *exp_off[NA] = {};
    auto prepare = [&]() -> int32_t {
        if (!s->computed || s->merged) return fail(s, ACCORD_ERR_STATE, "exchange needs a freshly computed partial");
        if (!s->has_txn_index && s->n != n_total) return fail(s, ACCORD_ERR_ARG, "batch without txn_index must be the whole stream");
        // 1. partial offsets expanded to every global txn position
        HIPCHECK(s, c->ind.ensure((size_t)n_total * 4 + 4));
        HIPCHECK(s, c->cscan.ensure(((size_t)n_total + 1) * 4));
        for (int a = 0; a < NA; ++a) HIPCHECK(s, c->exp[a].ensure(((size_t)n_total + 1) * 4));
        HIPCHECK(s, c->bnd.ensure((size_t)NA * (G + 1) * 4));
        HIPCHECK(s, c->total_buf.ensure(16));
        HIPCHECK(s, c->counts.ensure(2 * NA * (size_t)G * 8));
        HIPCHECK(s, c->allcounts.ensure(2 * NA * (size_t)G * 8 * G));
        HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(n_total), s->stream));
        return ACCORD_OK;
    };
    // flag buffer: allocated by accord_comm_init, so agreeing cannot itself fail on one rank only
    auto agree = [&](int32_t local_rc) -> int32_t {
        const int32_t flag = local_rc ? 1 : 0;
        int32_t *dflag = (int32_t *)c->flag.p;
        int32_t any = 0;
        if (hipMemcpyAsync(dflag, &flag, 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            ncclAllReduce(dflag, dflag, 1, ncclInt32, ncclMax, c->comm, st) != ncclSuccess ||
            hipMemcpyAsync(&any, dflag, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return fail(s, ACCORD_ERR_HIP, "accord_deps_exchange_merge: status all-reduce failed");
        if (local_rc) return local_rc;
        if (any) return fail(s, ACCORD_ERR_STATE, "accord_deps_exchange_merge: a peer rank rejected the exchange");
        return ACCORD_OK;
    };
    {
        int32_t rc = agree(prepare());
        if (rc) return rc;
    }
    if (s->events) (void)hipEventRecord(s->ev[EV_XCHG_START], st);
    const uint32_t *off[NA] = {s->kd_key_off.as<uint32_t>(), s->kd_val_off.as<uint32_t>(), s->kd_k2v_off.as<uint32_t>(),
                               s->rd_rng_off.as<uint32_t>(), s->rd_val_off.as<uint32_t>(), s->rd_r2v_off.as<uint32_t>()};
    for (int a = 0; a < NA; ++a) exp_off[a] = c->exp[a].as<uint32_t>();
    for (int h = 0; h < 2; ++h) {          // KeyDeps side, RangeDeps side
        if (s->has_txn_index) {
            accord::launch_expand_offsets(n, n_total, s->txn_index.as<uint32_t>(), c->ind.as<uint32_t>(),
                                          c->cscan.as<uint32_t>(), off + 3 * h, exp_off + 3 * h, s->scan_tmp.p,
                                          c->total_buf.as<unsigned long long>(), st);
        } else {
            for (int a = 3 * h; a < 3 * h + 3; ++a)
                HIPCHECK(s, hipMemcpyAsync(exp_off[a], off[a], ((size_t)n_total + 1) * 4, hipMemcpyDeviceToDevice, st));
        }
        accord::launch_boundaries(G, n_total, exp_off + 3 * h, c->bnd.as<uint32_t>() + 3 * h * (G + 1), st);
    }
    HIPCHECK(s, hipMemcpyAsync(bnd.data(), c->bnd.p, bnd.size() * 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));

    // 2. per destination: element counts and start offsets of what I send; all-gather the G x G matrix
    auto home_lo = [&](uint32_t d) { return (uint32_t)(((unsigned long long)d * n_total) / G); };
    const size_t W = 2 * NA;
    std::vector<unsigned long long> mine(W * (size_t)G);
    for (uint32_t d = 0; d < G; ++d)
        for (int a = 0; a < NA; ++a) {
            mine[W * d + a] = bnd[a * (G + 1) + d + 1] - bnd[a * (G + 1) + d];
            mine[W * d + NA + a] = bnd[a * (G + 1) + d];
        }
    HIPCHECK(s, hipMemcpyAsync(c->counts.p, mine.data(), mine.size() * 8, hipMemcpyHostToDevice, st));
    NCCLCHECK(s, ncclAllGather(c->counts.p, c->allcounts.p, mine.size(), ncclUint64, c->comm, st));
    std::vector<unsigned long long> all(mine.size() * G);
    HIPCHECK(s, hipMemcpyAsync(all.data(), c->allcounts.p, all.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));

    // 3. receive layout: per source [NA offset arrays (nh+1 each)][ND data arrays]
    const uint32_t my_lo = home_lo(me), nh = home_lo(me + 1) - my_lo;
    std::vector<size_t> rbase(G + 1);
    rbase[0] = 0;
    bool ranges = false;
    for (uint32_t src = 0; src < G; ++src) {
        const unsigned long long *cnt = &all[(size_t)src * W * G + W * me];
        size_t sz = NA * ((size_t)nh + 1);
        for (int k = 0; k < ND; ++k) sz += cnt[grp[k]];
        rbase[src + 1] = rbase[src] + sz;
        ranges = ranges || cnt[3] || cnt[4];
    }
    {
        const hipError_t e = c->recv.ensure(rbase[G] * 4 + 16);
        int32_t rc = agree(e == hipSuccess ? ACCORD_OK
                                           : fail(s, ACCORD_ERR_OOM, "exchange receive buffer: %s", hipGetErrorString(e)));
        if (rc) return rc;
    }
    uint32_t *R = c->recv.as<uint32_t>();
    std::vector<std::array<uint32_t *, NA>> roff(G);
    std::vector<std::array<uint32_t *, ND>> rdat(G);
    for (uint32_t src = 0; src < G; ++src) {
        const unsigned long long *cnt = &all[(size_t)src * W * G + W * me];
        uint32_t *b = R + rbase[src];
        for (int a = 0; a < NA; ++a) roff[src][a] = b + (size_t)a * (nh + 1);
        uint32_t *p = b + (size_t)NA * (nh + 1);
        for (int k = 0; k < ND; ++k) { rdat[src][k] = p; p += cnt[grp[k]]; }
    }
    const uint32_t *data[ND] = {s->kd_keys.as<uint32_t>(), s->kd_vals.as<uint32_t>(), (const uint32_t *)s->kd_k2v.p,
                                s->rd_rng_start.as<uint32_t>(), s->rd_rng_end.as<uint32_t>(), s->rd_vals.as<uint32_t>(),
                                (const uint32_t *)s->rd_r2v.p};
    NCCLCHECK(s, ncclGroupStart());
    for (uint32_t d = 0; d < G; ++d) {
        const uint32_t lo = home_lo(d), nd = home_lo(d + 1) - lo;
        for (int a = 0; a < NA; ++a) {
            const uint32_t *so = exp_off[a] + lo;
            if (d == me) {
                if (hipMemcpyAsync(roff[me][a], so, ((size_t)nd + 1) * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) {
                    (void)ncclGroupEnd();
                    return fail(s, ACCORD_ERR_HIP, "local exchange copy failed");
                }
            } else {
                NCCLGROUPCHECK(s, ncclSend(so, (size_t)nd + 1, ncclUint32, (int)d, c->comm, st));
            }
        }
        for (int k = 0; k < ND; ++k) {
            const int a = grp[k];
            const size_t dc = mine[W * d + a];
            if (!dc) continue;
            const uint32_t *sd = data[k] + bnd[a * (G + 1) + d];
            if (d == me) {
                if (hipMemcpyAsync(rdat[me][k], sd, dc * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) {
                    (void)ncclGroupEnd();
                    return fail(s, ACCORD_ERR_HIP, "local exchange copy failed");
                }
            } else {
                NCCLGROUPCHECK(s, ncclSend(sd, dc, ncclUint32, (int)d, c->comm, st));
            }
        }
    }
    for (uint32_t src = 0; src < G; ++src) {
        if (src == me) continue;
        const unsigned long long *cnt = &all[(size_t)src * W * G + W * me];
        for (int a = 0; a < NA; ++a) NCCLGROUPCHECK(s, ncclRecv(roff[src][a], (size_t)nh + 1, ncclUint32, (int)src, c->comm, st));
        for (int k = 0; k < ND; ++k)
            if (cnt[grp[k]]) NCCLGROUPCHECK(s, ncclRecv(rdat[src][k], cnt[grp[k]], ncclUint32, (int)src, c->comm, st));
    }
    NCCLCHECK(s, ncclGroupEnd());
    if (s->events) (void)hipEventRecord(s->ev[EV_XCHG_END], st);

    // 4. union of the G parts of my txns.  Received offsets are the sender's (not rebased): the
    // key-disjoint merge reads them relative to their first entry; the general union gets data
    // pointers shifted back by the sender's start offset so the offsets index them directly.
    int32_t rc;
    if (!ranges) {
        std::vector<Part> parts(G);
        for (uint32_t src = 0; src < G; ++src)
            parts[src] = Part{roff[src][0], rdat[src][0], roff[src][1], rdat[src][1], roff[src][2],
                              (const int32_t *)rdat[src][2]};
        rc = merge_parts(s, parts, nh, my_lo);
    } else {
        std::vector<accord_deps> views(G);
        for (uint32_t src = 0; src < G; ++src) {
            const unsigned long long *cnt = &all[(size_t)src * W * G + W * me];
            const unsigned long long *start = cnt + NA;
            auto back = [&](uint32_t *p, int a) { return (uint32_t *)((uintptr_t)p - (uintptr_t)(start[a] * 4)); };
            accord_deps &v = views[src];
            std::memset(&v, 0, sizeof(v));
            v.n = nh;
            v.kd_keys_total = cnt[0]; v.kd_vals_total = cnt[1]; v.kd_k2v_total = cnt[2];
            v.rd_rngs_total = cnt[3]; v.rd_vals_total = cnt[4]; v.rd_r2v_total = cnt[5];
            v.kd_key_off = roff[src][0]; v.kd_keys = back(rdat[src][0], 0);
            v.kd_val_off = roff[src][1]; v.kd_vals = back(rdat[src][1], 1);
            v.kd_k2v_off = roff[src][2]; v.kd_k2v = (int32_t *)back(rdat[src][2], 2);
            v.rd_rng_off = roff[src][3]; v.rd_rng_start = back(rdat[src][3], 3); v.rd_rng_end = back(rdat[src][4], 3);
            v.rd_val_off = roff[src][4]; v.rd_vals = back(rdat[src][5], 4);
            v.rd_r2v_off = roff[src][5]; v.rd_r2v = (int32_t *)back(rdat[src][6], 5);
        }
        rc = union_general(s, G, views.data());
    }
    if (rc) return rc;
    if (s->events) {
        (void)hipEventRecord(s->ev[EV_MERGE_END], st);
        (void)hipEventSynchronize(s->ev[EV_MERGE_END]);
        (void)hipEventElapsedTime(&s->xchg_ms, s->ev[EV_XCHG_START], s->ev[EV_XCHG_END]);
        (void)hipEventElapsedTime(&s->merge_ms, s->ev[EV_XCHG_END], s->ev[EV_MERGE_END]);
    }
    return ACCORD_OK;
}

int32_t accord_shard_timing(accord_store *s, float *exchange_ms, float *merge_ms)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (exchange_ms) *exchange_ms = s->xchg_ms;
    if (merge_ms) *merge_ms = s->merge_ms;
    return ACCORD_OK;
}

} // extern "C"
