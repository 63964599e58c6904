// Multi-store / multi-GPU union of per-store PartialDeps.
//
// accord_deps_merge          : union of G per-store partial KeyDeps of the same txns (device views,
//                              e.g. several stores on one GPU) -- PreAccept.reduce
//                              (messages/PreAccept.java:140-156) for key-disjoint stores.
// accord_deps_exchange_merge : the multi-GPU form.  Every rank (one GPU, a contiguous block of the
//                              8*G EvenSplit stores, local/ShardDistributor.java:46-157) has computed
//                              its stores' partial deps for the txns intersecting them
//                              (CommandStores.mapReduce fan-out, local/CommandStores.java:575-592);
//                              txn g's union is owned by rank floor(g*G/n_total).
//
// The exchange is three parts, and only the middle one differs between a real multi-GPU run and the
// one-GPU simulation (accord_deps_exchange_local) that the tests drive:
//   plan      : per rank, the expanded offset arrays (a store holding a subset of the stream maps its
//               offsets onto every global position) and, per destination rank, the element count and
//               first element of the 6 offset + 7 data arrays it sends (device, no host sync); the
//               G x G table of those counts (one all-gather) gives every rank the receive layout of
//               every rank -- the only host read of the exchange.
//   transport : the segment lists of the plan moved sender -> receiver: one grouped RCCL send/recv
//               over xGMI (product), or device copies between the G stores of one GPU (simulation).
//   union     : the G received parts of the owner's txns unioned on device -- the key-disjoint merge
//               (merge.hip) when no part holds RangeDeps, else RelationMultiMap.linearUnion
//               (accord_deps_union); output sizes are bounded by the received counts, so it runs
//               without a host sync (totals and the error word are read when the result is).
#include "store_impl.h"

#include <rccl/rccl.h>

#include <array>
#include <cstdint>
#include <cstring>
#include <new>
#include <utility>
#include <vector>

namespace {

constexpr int NA = accord::XCHG_NA;     // offset arrays
constexpr int ND = 7;                   // data arrays (range starts and ends share offset array 3)
constexpr size_t W = 2 * NA;            // per destination: NA counts, NA first elements
const int kGrp[ND] = {0, 1, 2, 3, 3, 4, 5};

#define RC_FORWARD(expr)                 \
    do {                                 \
        const int32_t rc_ = (expr);      \
        if (rc_) return rc_;             \
    } while (0)

struct Part {
    const uint32_t *key_off, *keys, *val_off, *vals, *k2v_off;
    const int32_t *k2v;
    const uint32_t *val_cnt;          // gapped txnIds: per-txn counts (nullptr: dense)
};

} // namespace

struct ShardComm {
    ncclComm_t comm = nullptr;          // null: a simulated rank of accord_deps_exchange_local
    int nranks = 1, rank = 0;
    DevBuf ind, cscan, exp[NA], total_buf, flag, counts, allcounts, recv;
    unsigned long long *h_all = nullptr;    // pinned host copy of the all-gathered counts
    // receive capacity (words) of every rank's buffer; every rank derives the same values from the
    // same count tables, so all agree whether any rank had to grow (and must confirm it succeeded)
    std::vector<size_t> peer_cap;
    // the exchange in flight
    uint32_t n_total = 0, my_lo = 0, nh = 0;
    bool ranges = false, grew = false, timed = false;
    accord::XchgOffsets eoff{};
    std::vector<size_t> rbase;
    size_t row() const { return W * (size_t)nranks + 1; }      // one rank's count row (+ status)
    const unsigned long long *cnt(uint32_t src, uint32_t dst) const { return h_all + src * row() + W * dst; }
};

namespace accord_impl {

void shard_comm_destroy(accord_store *s)
{
    if (!s || !s->comm) return;
    ShardComm *c = s->comm;
    if (c->comm) (void)ncclCommDestroy(c->comm);
    DevBuf *bufs[] = {&c->ind, &c->cscan, &c->exp[0], &c->exp[1], &c->exp[2], &c->exp[3], &c->exp[4], &c->exp[5],
                      &c->total_buf, &c->flag, &c->counts, &c->allcounts, &c->recv};
    for (DevBuf *b : bufs) b->release();
    if (c->h_all) (void)hipHostFree(c->h_all);
    delete c;
    s->comm = nullptr;
}

// the merged result's totals and error word, read when the result is first used (exchange path)
int32_t merge_finalize(accord_store *s)
{
    if (!s->m_pending) return ACCORD_OK;
    HIPCHECK(s, hipStreamSynchronize(s->stream));
    s->m_pending = false;
    const HostTotals &h = *s->pinned;
    if (h.status.first != ~0ull) {
        s->merged = false; s->computed = false;
        return fail(s, -(int32_t)(uint32_t)(h.status.first & 0xFFFFFFFFu),
                    "merge: parts have overlapping or unordered keys (txn %u)", (uint32_t)(h.status.first >> 32));
    }
    if (h.status.overflow) {
        s->merged = false; s->computed = false;
        return fail(s, ACCORD_ERR_CAPACITY, "merge: %u txns exceed the union capacity (first: txn %u)",
                    h.status.overflow, h.status.overflow_first);
    }
    s->m_tot_keys = h.totals[0]; s->m_tot_vals = h.totals[1]; s->m_tot_k2v = h.totals[2];
    return ACCORD_OK;
}

} // namespace accord_impl

namespace {

// Union of G aligned parts of n txns (global positions txn_lo..txn_lo+n-1) into s->m_*.
// bounds (keys, txnIds, keysToTxnIds upper bounds of the union) known: outputs sized by them and
// no host sync (totals pending, accord_impl::merge_finalize); else the exact totals are read first.
int32_t merge_parts(accord_store *s, const std::vector<Part> &parts, uint32_t n, uint32_t txn_lo,
                    const uint64_t *bounds = nullptr)
{
    const uint32_t G = (uint32_t)parts.size();
    if (G == 0 || G > 64) return fail(s, ACCORD_ERR_CAPACITY, "merge of %u parts (1..64 supported)", G);
    hipStream_t st = s->stream;
    const size_t n1 = (size_t)n + 1;
    HIPCHECK(s, s->m_ptrs.ensure((size_t)7 * G * sizeof(void *)));
    HIPCHECK(s, s->m_cnt_keys.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->m_cnt_vals.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->m_cnt_k2v.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->m_key_off.ensure(n1 * 4));
    HIPCHECK(s, s->m_val_off.ensure(n1 * 4));
    HIPCHECK(s, s->m_k2v_off.ensure(n1 * 4));
    HIPCHECK(s, s->m_zero.ensure(n1 * 4));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(n), s->stream));
    HIPCHECK(s, s->status_totals.ensure(sizeof(HostTotals)));
    if (bounds) {
        HIPCHECK(s, s->m_keys.ensure(bounds[0] * 4));
        HIPCHECK(s, s->m_vals.ensure(bounds[1] * 4));
        HIPCHECK(s, s->m_k2v.ensure(bounds[2] * 4));
    }
    // the pointer table (a pageable source: HIP stages the copy before returning, so the vector
    // may go out of scope right after)
    std::vector<const void *> tbl(7 * (size_t)G);
    for (uint32_t g = 0; g < G; ++g) {
        tbl[0 * G + g] = parts[g].key_off; tbl[1 * G + g] = parts[g].keys;
        tbl[2 * G + g] = parts[g].val_off; tbl[3 * G + g] = parts[g].vals;
        tbl[4 * G + g] = parts[g].k2v_off; tbl[5 * G + g] = parts[g].k2v;
        tbl[6 * G + g] = parts[g].val_cnt;
    }
    HIPCHECK(s, hipMemcpyAsync(s->m_ptrs.p, tbl.data(), tbl.size() * sizeof(void *), hipMemcpyHostToDevice, st));
    const void *const *ptab = (const void *const *)s->m_ptrs.p;
    accord::MergeParams mp{};
    mp.n = n; mp.G = G; mp.txn_lo = txn_lo;
    mp.key_off = (const uint32_t *const *)(ptab + 0 * G); mp.keys = (const uint32_t *const *)(ptab + 1 * G);
    mp.val_off = (const uint32_t *const *)(ptab + 2 * G); mp.vals = (const uint32_t *const *)(ptab + 3 * G);
    mp.k2v_off = (const uint32_t *const *)(ptab + 4 * G); mp.k2v = (const int32_t *const *)(ptab + 5 * G);
    mp.val_cnt = (const uint32_t *const *)(ptab + 6 * G);
    mp.cnt_keys = s->m_cnt_keys.as<uint32_t>(); mp.cnt_vals = s->m_cnt_vals.as<uint32_t>(); mp.cnt_k2v = s->m_cnt_k2v.as<uint32_t>();
    HostTotals *dev = s->status_totals.as<HostTotals>();
    mp.status = &dev->status;
    HIPCHECK(s, hipMemsetAsync(dev, 0xFF, sizeof(HostTotals), st));
    HIPCHECK(s, hipMemsetAsync(&dev->status.overflow, 0, sizeof(uint32_t), st));
    HIPCHECK(s, hipMemsetAsync(s->m_zero.p, 0, n1 * 4, st));
    accord::launch_merge_count(mp, st);
    {
        const uint32_t *in[3] = {mp.cnt_keys, mp.cnt_vals, mp.cnt_k2v};
        uint32_t *out[3] = {s->m_key_off.as<uint32_t>(), s->m_val_off.as<uint32_t>(), s->m_k2v_off.as<uint32_t>()};
        unsigned long long *tot[3] = {&dev->totals[0], &dev->totals[1], &dev->totals[2]};
        accord::exclusive_scan_multi(3, in, out, tot, n, s->scan_tmp.p, st);
    }
    mp.out_key_off = s->m_key_off.as<uint32_t>(); mp.out_val_off = s->m_val_off.as<uint32_t>();
    mp.out_k2v_off = s->m_k2v_off.as<uint32_t>();
    s->m_n = n;
    s->m_txn_lo = txn_lo;
    s->ds_cur = -1;
    s->wo_done = false;
    if (bounds) {
        mp.out_keys = s->m_keys.as<uint32_t>(); mp.out_vals = s->m_vals.as<uint32_t>(); mp.out_k2v = s->m_k2v.as<int32_t>();
        accord::launch_merge_fill(mp, st);
        HIPCHECK(s, hipMemcpyAsync(s->pinned, dev, sizeof(HostTotals), hipMemcpyDeviceToHost, st));
        HIPCHECK(s, hipGetLastError());
        s->m_pending = true;
        s->merged = true;
        s->computed = true;
        return ACCORD_OK;
    }
    HIPCHECK(s, hipMemcpyAsync(s->pinned, dev, sizeof(HostTotals), hipMemcpyDeviceToHost, st));
    s->m_pending = true;
    s->merged = true;
    s->computed = true;
    {
        const int32_t rc = accord_impl::merge_finalize(s);
        if (rc) return rc;
    }
    HIPCHECK(s, s->m_keys.ensure(s->m_tot_keys * 4));
    HIPCHECK(s, s->m_vals.ensure(s->m_tot_vals * 4));
    HIPCHECK(s, s->m_k2v.ensure(s->m_tot_k2v * 4));
    mp.out_keys = s->m_keys.as<uint32_t>(); mp.out_vals = s->m_vals.as<uint32_t>(); mp.out_k2v = s->m_k2v.as<int32_t>();
    accord::launch_merge_fill(mp, st);
    HIPCHECK(s, hipStreamSynchronize(st));
    HIPCHECK(s, hipGetLastError());
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

uint32_t home_lo(uint32_t d, uint32_t n_total, uint32_t G) { return (uint32_t)(((unsigned long long)d * n_total) / G); }

// ---------------------------------------------------------------- plan
// The exchange state of a store as rank `rank` of `G` (comm: the RCCL communicator, or null for a
// simulated rank).  The count buffers depend on G only.
int32_t xchg_state(accord_store *s, int G, int rank, ncclComm_t comm)
{
    ShardComm *c = new (std::nothrow) ShardComm();
    if (!c) return fail(s, ACCORD_ERR_OOM, "out of host memory");
    c->comm = comm;
    c->nranks = G;
    c->rank = rank;
    c->peer_cap.assign((size_t)G, 0);
    const size_t row = c->row();
    if (c->flag.ensure(16) != hipSuccess || c->counts.ensure(row * 8) != hipSuccess ||
        c->allcounts.ensure(row * G * 8) != hipSuccess ||
        hipHostMalloc((void **)&c->h_all, row * G * 8, hipHostMallocDefault) != hipSuccess) {
        c->comm = nullptr;                      // the caller still owns comm on failure
        s->comm = c;
        accord_impl::shard_comm_destroy(s);
        return fail(s, ACCORD_ERR_OOM, "exchange state for %d ranks", G);
    }
    s->comm = c;
    return ACCORD_OK;
}

// local checks and allocations of the plan
int32_t xchg_prepare(accord_store *s, uint32_t n_total)
{
    ShardComm *c = s->comm;
    if (!s->computed || s->merged) return fail(s, ACCORD_ERR_STATE, "exchange needs a freshly computed partial");
    if (!s->has_txn_index && s->n != n_total) return fail(s, ACCORD_ERR_ARG, "batch without txn_index must be the whole stream");
    if (s->ds_cur >= 0) return fail(s, ACCORD_ERR_STATE, "exchange of a store holding a deps-set result");
    // the partials travel dense: the compute's gapped txnIds are compacted first (kd_val_off / kd_vals)
    RC_FORWARD(accord_impl::store_dense_keydeps(s));
    if (s->has_txn_index) {
        HIPCHECK(s, c->ind.ensure((size_t)n_total * 4 + 4));
        HIPCHECK(s, c->cscan.ensure(((size_t)n_total + 1) * 4));
        for (int a = 0; a < NA; ++a) HIPCHECK(s, c->exp[a].ensure(((size_t)n_total + 1) * 4));
        HIPCHECK(s, c->total_buf.ensure(16));
        HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(n_total), s->stream));
    }
    return ACCORD_OK;
}

// device part of the plan: expanded offsets and this rank's count row; a rank whose prepare failed
// publishes a row with its status word set instead, so every rank still reaches the all-gather
int32_t xchg_plan(accord_store *s, uint32_t n_total, int32_t prepared)
{
    ShardComm *c = s->comm;
    hipStream_t st = s->stream;
    const uint32_t G = (uint32_t)c->nranks;
    c->n_total = n_total;
    if (prepared != ACCORD_OK) {
        std::vector<unsigned long long> row(c->row(), 0ull);
        row.back() = 1ull;
        HIPCHECK(s, hipMemcpy(c->counts.p, row.data(), row.size() * 8, hipMemcpyHostToDevice));
        return prepared;
    }
    const accord::XchgOffsets own{{s->kd_key_off.as<uint32_t>(), s->kd_val_off.as<uint32_t>(), s->kd_k2v_off.as<uint32_t>(),
                                   s->rd_rng_off.as<uint32_t>(), s->rd_val_off.as<uint32_t>(), s->rd_r2v_off.as<uint32_t>()}};
    if (s->has_txn_index) {
        accord::launch_expand_index(s->n, n_total, s->txn_index.as<uint32_t>(), c->ind.as<uint32_t>(),
                                    c->cscan.as<uint32_t>(), s->scan_tmp.p, c->total_buf.as<unsigned long long>(), st);
        for (int a = 0; a < NA; ++a) c->eoff.p[a] = c->exp[a].as<uint32_t>();
        accord::launch_expand_offsets(n_total, c->cscan.as<uint32_t>(), own, c->eoff, st);
    } else {
        c->eoff = own;                              // the store holds every txn of the stream
    }
    accord::launch_xchg_counts(G, n_total, c->eoff, c->counts.as<unsigned long long>(), st);
    HIPCHECK(s, hipGetLastError());
    return ACCORD_OK;
}

// the all-gathered count table read back (the exchange's one host sync); any rank's status word
// stops every rank here
int32_t xchg_read_counts(accord_store *s, int32_t own_rc)
{
    ShardComm *c = s->comm;
    const size_t bytes = c->row() * (size_t)c->nranks * 8;
    HIPCHECK(s, hipMemcpyAsync(c->h_all, c->allcounts.p, bytes, hipMemcpyDeviceToHost, s->stream));
    HIPCHECK(s, hipStreamSynchronize(s->stream));
    if (own_rc) return own_rc;
    for (int r = 0; r < c->nranks; ++r)
        if (c->h_all[(size_t)r * c->row() + W * c->nranks])
            return fail(s, ACCORD_ERR_STATE, "accord_deps_exchange_merge: rank %d rejected the exchange", r);
    return ACCORD_OK;
}

// receive layout of every rank from the table: per source [NA offset arrays (nh+1 each)][ND data
// arrays]; this rank's buffer grows when needed (c->grew: some rank's did)
size_t recv_words(const ShardComm *c, uint32_t me)
{
    const uint32_t G = (uint32_t)c->nranks;
    const uint32_t nh = home_lo(me + 1, c->n_total, G) - home_lo(me, c->n_total, G);
    size_t sz = 0;
    for (uint32_t src = 0; src < G; ++src) {
        sz += NA * ((size_t)nh + 1);
        for (int k = 0; k < ND; ++k) sz += c->cnt(src, me)[kGrp[k]];
    }
    return sz;
}

int32_t xchg_layout(accord_store *s)
{
    ShardComm *c = s->comm;
    const uint32_t G = (uint32_t)c->nranks, me = (uint32_t)c->rank;
    c->my_lo = home_lo(me, c->n_total, G);
    c->nh = home_lo(me + 1, c->n_total, G) - c->my_lo;
    c->rbase.assign(G + 1, 0);
    c->ranges = false;
    for (uint32_t src = 0; src < G; ++src) {
        const unsigned long long *cnt = c->cnt(src, me);
        size_t sz = NA * ((size_t)c->nh + 1);
        for (int k = 0; k < ND; ++k) sz += cnt[kGrp[k]];
        c->rbase[src + 1] = c->rbase[src] + sz;
        c->ranges = c->ranges || cnt[3] || cnt[4];
    }
    c->grew = false;
    for (uint32_t r = 0; r < G; ++r) {
        const size_t need = recv_words(c, r);
        if (need > c->peer_cap[r]) { c->peer_cap[r] = need + need / 8 + 64; c->grew = true; }
    }
    HIPCHECK(s, c->recv.ensure(c->peer_cap[me] * 4 + 16));
    return ACCORD_OK;
}

// what rank `me` sends to d / receives from src, as matching ordered segment lists (words)
using SendSeg = std::pair<const uint32_t *, size_t>;
using RecvSeg = std::pair<uint32_t *, size_t>;

void send_segs(const accord_store *s, uint32_t d, std::vector<SendSeg> &out)
{
    const ShardComm *c = s->comm;
    const uint32_t G = (uint32_t)c->nranks, me = (uint32_t)c->rank;
    const uint32_t lo = home_lo(d, c->n_total, G), nd = home_lo(d + 1, c->n_total, G) - lo;
    const unsigned long long *mine = c->cnt(me, d);
    const uint32_t *data[ND] = {s->kd_keys.as<uint32_t>(), s->kd_vals.as<uint32_t>(), (const uint32_t *)s->kd_k2v.p,
                                s->rd_rng_start.as<uint32_t>(), s->rd_rng_end.as<uint32_t>(), s->rd_vals.as<uint32_t>(),
                                (const uint32_t *)s->rd_r2v.p};
    out.clear();
    for (int a = 0; a < NA; ++a) out.emplace_back(c->eoff.p[a] + lo, (size_t)nd + 1);
    for (int k = 0; k < ND; ++k) {
        const int a = kGrp[k];
        if (mine[a]) out.emplace_back(data[k] + mine[NA + a], (size_t)mine[a]);
    }
}

struct RecvView {
    std::array<uint32_t *, NA> off;
    std::array<uint32_t *, ND> dat;
};

RecvView recv_view(const accord_store *s, uint32_t src)
{
    const ShardComm *c = s->comm;
    const unsigned long long *cnt = c->cnt(src, (uint32_t)c->rank);
    RecvView v;
    uint32_t *b = c->recv.as<uint32_t>() + c->rbase[src];
    for (int a = 0; a < NA; ++a) v.off[a] = b + (size_t)a * (c->nh + 1);
    uint32_t *p = b + (size_t)NA * (c->nh + 1);
    for (int k = 0; k < ND; ++k) { v.dat[k] = p; p += cnt[kGrp[k]]; }
    return v;
}

void recv_segs(const accord_store *s, uint32_t src, std::vector<RecvSeg> &out)
{
    const ShardComm *c = s->comm;
    const unsigned long long *cnt = c->cnt(src, (uint32_t)c->rank);
    const RecvView v = recv_view(s, src);
    out.clear();
    for (int a = 0; a < NA; ++a) out.emplace_back(v.off[a], (size_t)c->nh + 1);
    for (int k = 0; k < ND; ++k)
        if (cnt[kGrp[k]]) out.emplace_back(v.dat[k], (size_t)cnt[kGrp[k]]);
}

// ---------------------------------------------------------------- union
// Received offsets are the sender's (not rebased); both unions read a part's data relative to its
// first offset (element of txn t at off[t] - off[0]), so the received data arrays are used as they
// are.
int32_t xchg_union(accord_store *s)
{
    ShardComm *c = s->comm;
    const uint32_t G = (uint32_t)c->nranks, me = (uint32_t)c->rank;
    if (!c->ranges) {
        std::vector<Part> parts(G);
        uint64_t bounds[3] = {0, 0, 0};
        for (uint32_t src = 0; src < G; ++src) {
            const RecvView v = recv_view(s, src);
            parts[src] = Part{v.off[0], v.dat[0], v.off[1], v.dat[1], v.off[2], (const int32_t *)v.dat[2], nullptr};
            for (int a = 0; a < 3; ++a) bounds[a] += c->cnt(src, me)[a];
        }
        return merge_parts(s, parts, c->nh, c->my_lo, bounds);
    }
    std::vector<accord_deps> views(G);
    for (uint32_t src = 0; src < G; ++src) {
        const unsigned long long *cnt = c->cnt(src, me);
        const RecvView rv = recv_view(s, src);
        accord_deps &v = views[src];
        std::memset(&v, 0, sizeof(v));
        v.n = c->nh;
        v.kd_keys_total = cnt[0]; v.kd_vals_total = cnt[1]; v.kd_k2v_total = cnt[2];
        v.rd_rngs_total = cnt[3]; v.rd_vals_total = cnt[4]; v.rd_r2v_total = cnt[5];
        v.kd_key_off = rv.off[0]; v.kd_keys = rv.dat[0];
        v.kd_val_off = rv.off[1]; v.kd_vals = rv.dat[1];
        v.kd_k2v_off = rv.off[2]; v.kd_k2v = (int32_t *)rv.dat[2];
        v.rd_rng_off = rv.off[3]; v.rd_rng_start = rv.dat[3]; v.rd_rng_end = rv.dat[4];
        v.rd_val_off = rv.off[4]; v.rd_vals = rv.dat[5];
        v.rd_r2v_off = rv.off[5]; v.rd_r2v = (int32_t *)rv.dat[6];
    }
    return union_general(s, G, views.data());
}

void mark(accord_store *s, int ev)
{
    if (s->events) (void)hipEventRecord(s->ev[ev], s->stream);
}

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
                     parts[g].kd_k2v_off, parts[g].kd_k2v, parts[g].kd_val_cnt};
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

int32_t accord_comm_size(accord_store *s, int32_t *nranks, int32_t *rank)
{
    if (!s || !nranks || !rank) return fail(s, ACCORD_ERR_ARG, "accord_comm_size: null argument");
    if (!s->comm || !s->comm->comm) return fail(s, ACCORD_ERR_STATE, "accord_comm_size before accord_comm_init");
    int cnt = 0, me = 0;
    ncclResult_t r = ncclCommCount(s->comm->comm, &cnt);
    if (r == ncclSuccess) r = ncclCommUserRank(s->comm->comm, &me);
    if (r != ncclSuccess) return fail(s, ACCORD_ERR_HIP, "ncclCommCount: %s", ncclGetErrorString(r));
    *nranks = cnt; *rank = me;
    return ACCORD_OK;
}

int32_t accord_comm_init(accord_store *s, int32_t nranks, int32_t rank, const void *id128)
{
    if (!s || !id128 || nranks < 1 || rank < 0 || rank >= nranks) return fail(s, ACCORD_ERR_ARG, "accord_comm_init: bad arguments");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    accord_impl::shard_comm_destroy(s);
    ncclUniqueId id;
    std::memcpy(&id, id128, sizeof(id));
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclCommInitRank(&comm, nranks, id, rank);
    if (r != ncclSuccess) return fail(s, ACCORD_ERR_HIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
    const int32_t rc = xchg_state(s, nranks, rank, comm);
    if (rc) (void)ncclCommDestroy(comm);
    return rc;
}

int32_t accord_deps_exchange_merge(accord_store *s, uint32_t n_total)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (!s->comm || !s->comm->comm) return fail(s, ACCORD_ERR_STATE, "accord_deps_exchange_merge before accord_comm_init");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    ShardComm *c = s->comm;
    const uint32_t G = (uint32_t)c->nranks, me = (uint32_t)c->rank;
    hipStream_t st = s->stream;
    c->timed = false;

    // 1. plan: every rank reaches the all-gather, a rank that failed locally with its status set
    mark(s, EV_XCHG_START);
    int32_t rc = xchg_prepare(s, n_total);
    {
        const int32_t prc = xchg_plan(s, n_total, rc);
        if (!rc) rc = prc;
    }
    NCCLCHECK(s, ncclAllGather(c->counts.p, c->allcounts.p, c->row(), ncclUint64, c->comm, st));
    rc = xchg_read_counts(s, rc);
    if (rc) return rc;
    // every rank computes the same `grew`: only then do all confirm the allocation succeeded
    rc = xchg_layout(s);
    if (c->grew) {
        const int32_t flag = rc ? 1 : 0;
        int32_t *dflag = (int32_t *)c->flag.p;
        int32_t any = 0;
        if (hipMemcpyAsync(dflag, &flag, 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            ncclAllReduce(dflag, dflag, 1, ncclInt32, ncclMax, c->comm, st) != ncclSuccess ||
            hipMemcpyAsync(&any, dflag, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return fail(s, ACCORD_ERR_HIP, "accord_deps_exchange_merge: status all-reduce failed");
        if (rc) return rc;
        if (any) return fail(s, ACCORD_ERR_STATE, "accord_deps_exchange_merge: a peer rank could not size its receive buffer");
    } else if (rc) {
        return rc;
    }

    // 2. transport: one grouped send/recv; the part a rank keeps is a device copy
    std::vector<SendSeg> out;
    std::vector<RecvSeg> in;
    NCCLCHECK(s, ncclGroupStart());
    for (uint32_t d = 0; d < G; ++d) {
        send_segs(s, d, out);
        if (d == me) {
            recv_segs(s, me, in);
            for (size_t i = 0; i < out.size(); ++i)
                if (hipMemcpyAsync(in[i].first, out[i].first, out[i].second * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) {
                    (void)ncclGroupEnd();
                    return fail(s, ACCORD_ERR_HIP, "local exchange copy failed");
                }
            continue;
        }
        for (const SendSeg &g : out) NCCLGROUPCHECK(s, ncclSend(g.first, g.second, ncclUint32, (int)d, c->comm, st));
    }
    for (uint32_t src = 0; src < G; ++src) {
        if (src == me) continue;
        recv_segs(s, src, in);
        for (const RecvSeg &g : in) NCCLGROUPCHECK(s, ncclRecv(g.first, g.second, ncclUint32, (int)src, c->comm, st));
    }
    NCCLCHECK(s, ncclGroupEnd());
    mark(s, EV_XCHG_END);

    // 3. union of the G parts of my txns
    rc = xchg_union(s);
    if (rc) return rc;
    mark(s, EV_MERGE_END);
    c->timed = s->events;
    return ACCORD_OK;
}

int32_t accord_deps_exchange_local(accord_store *const *stores, uint32_t G, uint32_t n_total)
{
    if (!stores || G == 0 || G > 64) return fail(nullptr, ACCORD_ERR_ARG, "accord_deps_exchange_local: bad arguments");
    for (uint32_t r = 0; r < G; ++r) {
        accord_store *s = stores[r];
        if (!s) return fail(nullptr, ACCORD_ERR_ARG, "accord_deps_exchange_local: null store %u", r);
        if (s->cfg.device != stores[0]->cfg.device) return fail(s, ACCORD_ERR_ARG, "simulated ranks must share a device");
        if (s->comm && s->comm->comm) return fail(s, ACCORD_ERR_STATE, "store %u holds an RCCL communicator", r);
        if (!s->comm || s->comm->nranks != (int)G || s->comm->rank != (int)r) {
            accord_impl::shard_comm_destroy(s);
            RC_FORWARD(xchg_state(s, (int)G, (int)r, nullptr));
        }
    }
    HIPCHECK(stores[0], hipSetDevice(stores[0]->cfg.device));
    // 1. plan on every simulated rank, then the all-gather of their count rows
    for (uint32_t r = 0; r < G; ++r) {
        accord_store *s = stores[r];
        s->comm->timed = false;
        mark(s, EV_XCHG_START);
        RC_FORWARD(xchg_prepare(s, n_total));
        RC_FORWARD(xchg_plan(s, n_total, ACCORD_OK));
    }
    for (uint32_t r = 0; r < G; ++r) HIPCHECK(stores[r], hipStreamSynchronize(stores[r]->stream));
    for (uint32_t r = 0; r < G; ++r) {
        ShardComm *c = stores[r]->comm;
        for (uint32_t src = 0; src < G; ++src)
            HIPCHECK(stores[r], hipMemcpyAsync(c->allcounts.as<unsigned long long>() + src * c->row(), stores[src]->comm->counts.p,
                                               c->row() * 8, hipMemcpyDeviceToDevice, stores[r]->stream));
        RC_FORWARD(xchg_read_counts(stores[r], ACCORD_OK));
        RC_FORWARD(xchg_layout(stores[r]));
    }
    // 2. transport: the sender's segment list copied into the receiver's matching list
    std::vector<SendSeg> out;
    std::vector<RecvSeg> in;
    for (uint32_t d = 0; d < G; ++d) {
        accord_store *dst = stores[d];
        for (uint32_t src = 0; src < G; ++src) {
            send_segs(stores[src], d, out);
            recv_segs(dst, src, in);
            if (out.size() != in.size()) return fail(dst, ACCORD_ERR_STATE, "exchange plan mismatch (%u -> %u)", src, d);
            for (size_t i = 0; i < out.size(); ++i) {
                if (out[i].second != in[i].second) return fail(dst, ACCORD_ERR_STATE, "exchange segment size mismatch");
                HIPCHECK(dst, hipMemcpyAsync(in[i].first, out[i].first, out[i].second * 4, hipMemcpyDeviceToDevice, dst->stream));
            }
        }
        mark(dst, EV_XCHG_END);
    }
    // the senders' buffers are read by the receivers' streams: every copy completes before any
    // sender may reuse them (and before the union below overwrites nothing a copy still reads)
    for (uint32_t r = 0; r < G; ++r) HIPCHECK(stores[r], hipStreamSynchronize(stores[r]->stream));
    // 3. union on every simulated rank
    for (uint32_t r = 0; r < G; ++r) {
        RC_FORWARD(xchg_union(stores[r]));
        mark(stores[r], EV_MERGE_END);
        stores[r]->comm->timed = stores[r]->events;
    }
    return ACCORD_OK;
}

int32_t accord_shard_timing(accord_store *s, float *exchange_ms, float *merge_ms)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (s->comm && s->comm->timed) {
        HIPCHECK(s, hipEventSynchronize(s->ev[EV_MERGE_END]));
        (void)hipEventElapsedTime(&s->xchg_ms, s->ev[EV_XCHG_START], s->ev[EV_XCHG_END]);
        (void)hipEventElapsedTime(&s->merge_ms, s->ev[EV_XCHG_END], s->ev[EV_MERGE_END]);
        s->comm->timed = false;
    }
    if (exchange_ms) *exchange_ms = s->xchg_ms;
    if (merge_ms) *merge_ms = s->merge_ms;
    return ACCORD_OK;
}

} // extern "C"
