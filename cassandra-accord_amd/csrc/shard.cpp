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
    DevBuf ind, cscan, exp[3], bnd, counts, allcounts, recv;
    unsigned long long *total = nullptr;
    DevBuf total_buf, flag;
};

namespace accord_impl {

void shard_comm_destroy(accord_store *s)
{
    if (!s || !s->comm) return;
    ShardComm *c = s->comm;
    if (c->comm) (void)ncclCommDestroy(c->comm);
    DevBuf *bufs[] = {&c->ind, &c->cscan, &c->exp[0], &c->exp[1], &c->exp[2], &c->bnd, &c->counts, &c->allcounts,
                      &c->recv, &c->total_buf, &c->flag};
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
    for (uint32_t g = 0; g < nparts; ++g) {
        if (parts[g].n != n) return fail(s, ACCORD_ERR_ARG, "merge parts cover different txn counts");
        if (parts[g].rd_rngs_total || parts[g].rd_vals_total)
            return fail(s, ACCORD_ERR_STATE, "merge of RangeDeps is not supported by this build");
        ps[g] = Part{parts[g].kd_key_off, parts[g].kd_keys, parts[g].kd_val_off, parts[g].kd_vals,
                     parts[g].kd_k2v_off, parts[g].kd_k2v};
    }
    return merge_parts(s, ps, n, txn_lo);
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

    // Every rank must reach the same collectives: the local checks and allocations run first, then
    // one all-reduce (max) of their status agrees whether every rank goes ahead; a rank that failed
    // keeps its own message, the others report that a peer failed.
    std::vector<uint32_t> bnd(3 * (G + 1));
    uint32_t *exp_off[3] = {nullptr, nullptr, nullptr};
    auto prepare = [&]() -> int32_t {
        if (!s->computed || s->merged) return fail(s, ACCORD_ERR_STATE, "exchange needs a freshly computed partial");
        if (s->tot_rngs || s->tot_rvals) return fail(s, ACCORD_ERR_STATE, "exchange of RangeDeps is not supported by this build");
        if (!s->has_txn_index && s->n != n_total) return fail(s, ACCORD_ERR_ARG, "batch without txn_index must be the whole stream");
        // 1. partial offsets expanded to every global txn position
        HIPCHECK(s, c->ind.ensure((size_t)n_total * 4 + 4));
        HIPCHECK(s, c->cscan.ensure(((size_t)n_total + 1) * 4));
        for (int a = 0; a < 3; ++a) HIPCHECK(s, c->exp[a].ensure(((size_t)n_total + 1) * 4));
        HIPCHECK(s, c->bnd.ensure((size_t)3 * (G + 1) * 4));
        HIPCHECK(s, c->total_buf.ensure(16));
        HIPCHECK(s, c->counts.ensure(3 * (size_t)G * 8));
        HIPCHECK(s, c->allcounts.ensure(3 * (size_t)G * 8 * G));
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
    const uint32_t *off[3] = {s->kd_key_off.as<uint32_t>(), s->kd_val_off.as<uint32_t>(), s->kd_k2v_off.as<uint32_t>()};
    for (int a = 0; a < 3; ++a) exp_off[a] = c->exp[a].as<uint32_t>();
    if (s->has_txn_index) {
        accord::launch_expand_offsets(n, n_total, s->txn_index.as<uint32_t>(), c->ind.as<uint32_t>(),
                                      c->cscan.as<uint32_t>(), off, exp_off, s->scan_tmp.p,
                                      c->total_buf.as<unsigned long long>(), st);
    } else {
        for (int a = 0; a < 3; ++a)
            HIPCHECK(s, hipMemcpyAsync(exp_off[a], off[a], ((size_t)n_total + 1) * 4, hipMemcpyDeviceToDevice, st));
    }
    accord::launch_boundaries(G, n_total, exp_off, c->bnd.as<uint32_t>(), st);
    HIPCHECK(s, hipMemcpyAsync(bnd.data(), c->bnd.p, bnd.size() * 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));

    // 2. element counts I send to every rank; all-gather the G x G x 3 matrix
    auto home_lo = [&](uint32_t d) { return (uint32_t)(((unsigned long long)d * n_total) / G); };
    std::vector<unsigned long long> mine(3 * (size_t)G);
    for (uint32_t d = 0; d < G; ++d)
        for (int a = 0; a < 3; ++a) mine[3 * d + a] = bnd[a * (G + 1) + d + 1] - bnd[a * (G + 1) + d];
    HIPCHECK(s, hipMemcpyAsync(c->counts.p, mine.data(), mine.size() * 8, hipMemcpyHostToDevice, st));
    NCCLCHECK(s, ncclAllGather(c->counts.p, c->allcounts.p, mine.size(), ncclUint64, c->comm, st));
    std::vector<unsigned long long> all(mine.size() * G);
    HIPCHECK(s, hipMemcpyAsync(all.data(), c->allcounts.p, all.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));

    // 3. receive layout: per source [off_key|off_val|off_k2v (nh+1 each)][keys][vals][k2v]
    const uint32_t my_lo = home_lo(me), nh = home_lo(me + 1) - my_lo;
    std::vector<size_t> rbase(G + 1);
    rbase[0] = 0;
    for (uint32_t src = 0; src < G; ++src) {
        const unsigned long long *cnt = &all[(size_t)src * 3 * G + 3 * me];
        rbase[src + 1] = rbase[src] + 3 * ((size_t)nh + 1) + cnt[0] + cnt[1] + cnt[2];
    }
    {
        const hipError_t e = c->recv.ensure(rbase[G] * 4 + 16);
        int32_t rc = agree(e == hipSuccess ? ACCORD_OK
                                           : fail(s, ACCORD_ERR_OOM, "exchange receive buffer: %s", hipGetErrorString(e)));
        if (rc) return rc;
    }
    uint32_t *R = c->recv.as<uint32_t>();
    std::vector<Part> parts(G);
    for (uint32_t src = 0; src < G; ++src) {
        const unsigned long long *cnt = &all[(size_t)src * 3 * G + 3 * me];
        uint32_t *b = R + rbase[src];
        Part &p = parts[src];
        p.key_off = b; p.val_off = b + (nh + 1); p.k2v_off = b + 2 * (nh + 1);
        p.keys = b + 3 * (nh + 1); p.vals = p.keys + cnt[0]; p.k2v = (const int32_t *)(p.vals + cnt[1]);
    }
    const uint32_t *data[3] = {s->kd_keys.as<uint32_t>(), s->kd_vals.as<uint32_t>(), (const uint32_t *)s->kd_k2v.p};
    NCCLCHECK(s, ncclGroupStart());
    for (uint32_t d = 0; d < G; ++d) {
        const uint32_t lo = home_lo(d), nd = home_lo(d + 1) - lo;
        for (int a = 0; a < 3; ++a) {
            const uint32_t *so = exp_off[a] + lo;
            const uint32_t *sd = data[a] + bnd[a * (G + 1) + d];
            const size_t dc = mine[3 * d + a];
            if (d == me) {
                uint32_t *ro = (uint32_t *)(a == 0 ? parts[me].key_off : a == 1 ? parts[me].val_off : parts[me].k2v_off);
                uint32_t *rd = (uint32_t *)(a == 0 ? parts[me].keys : a == 1 ? parts[me].vals : (const uint32_t *)parts[me].k2v);
                if (hipMemcpyAsync(ro, so, ((size_t)nd + 1) * 4, hipMemcpyDeviceToDevice, st) != hipSuccess ||
                    (dc && hipMemcpyAsync(rd, sd, dc * 4, hipMemcpyDeviceToDevice, st) != hipSuccess)) {
                    (void)ncclGroupEnd();
                    return fail(s, ACCORD_ERR_HIP, "local exchange copy failed");
                }
            } else {
                NCCLGROUPCHECK(s, ncclSend(so, (size_t)nd + 1, ncclUint32, (int)d, c->comm, st));
                if (dc) NCCLGROUPCHECK(s, ncclSend(sd, dc, ncclUint32, (int)d, c->comm, st));
            }
        }
    }
    for (uint32_t src = 0; src < G; ++src) {
        if (src == me) continue;
        const unsigned long long *cnt = &all[(size_t)src * 3 * G + 3 * me];
        for (int a = 0; a < 3; ++a) {
            uint32_t *ro = (uint32_t *)(a == 0 ? parts[src].key_off : a == 1 ? parts[src].val_off : parts[src].k2v_off);
            uint32_t *rd = (uint32_t *)(a == 0 ? parts[src].keys : a == 1 ? parts[src].vals : (const uint32_t *)parts[src].k2v);
            NCCLGROUPCHECK(s, ncclRecv(ro, (size_t)nh + 1, ncclUint32, (int)src, c->comm, st));
            if (cnt[a]) NCCLGROUPCHECK(s, ncclRecv(rd, cnt[a], ncclUint32, (int)src, c->comm, st));
        }
    }
    NCCLCHECK(s, ncclGroupEnd());
    if (s->events) (void)hipEventRecord(s->ev[EV_XCHG_END], st);

    // 4. union of the G parts of my txns
    int32_t rc = merge_parts(s, parts, nh, my_lo);
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
