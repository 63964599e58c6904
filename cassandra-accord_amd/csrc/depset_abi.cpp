// C ABI of the deps-set operations (include/accord_deps.h: accord_deps_union / _slice / _invert;
// SURVEY.md §8a a9, a10).  Host orchestration only: every pass runs in depset.hip on the store's
// stream, with one host read of the sizes between count and fill passes.
#include "store_impl.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

namespace {

enum Tmp { T_VLEN, T_KLEN, T_BLEN, T_VEOFF, T_KEOFF, T_BEOFF, T_VOWN, T_VLST, T_KOWN, T_KLST, T_CNTV, T_CNTK,
           T_VRANK, T_KRANK, T_RB, T_BOWN, T_BTOT, T_BSZ, T_BSCAN, T_PTRS, T_SCAN, T_TOT, T_SEL0, T_SEL1 };

struct SideView {   // one side of one host-described device view
    const uint32_t *key_off, *lo, *hi, *val_off, *vals, *x_off;
    const int32_t *x;
    const uint32_t *val_cnt;          // gapped txnIds (KeyDeps of a compute result), else nullptr
};

SideView side_of(const accord_deps &d, bool range)
{
    if (!range) return SideView{d.kd_key_off, d.kd_keys, nullptr, d.kd_val_off, d.kd_vals, d.kd_k2v_off, d.kd_k2v,
                                d.kd_val_cnt};
    return SideView{d.rd_rng_off, d.rd_rng_start, d.rd_rng_end, d.rd_val_off, d.rd_vals, d.rd_r2v_off, d.rd_r2v, nullptr};
}

// device pointer table of G views' side -> DsSide
int32_t make_side(accord_store *s, const std::vector<SideView> &v, bool range, DevBuf &buf, accord::DsSide &S)
{
    const size_t G = v.size();
    std::vector<const void *> tbl(8 * G);
    for (size_t g = 0; g < G; ++g) {
        if (!v[g].key_off || !v[g].val_off || !v[g].x_off)
            return fail(s, ACCORD_ERR_ARG, "deps view %zu has no %s offsets", g, range ? "RangeDeps" : "KeyDeps");
        tbl[0 * G + g] = v[g].key_off; tbl[1 * G + g] = v[g].lo; tbl[2 * G + g] = v[g].hi;
        tbl[3 * G + g] = v[g].val_off; tbl[4 * G + g] = v[g].vals; tbl[5 * G + g] = v[g].x_off;
        tbl[6 * G + g] = v[g].x;
        tbl[7 * G + g] = v[g].val_cnt;
    }
    HIPCHECK(s, buf.ensure(tbl.size() * sizeof(void *)));
    HIPCHECK(s, hipMemcpyAsync(buf.p, tbl.data(), tbl.size() * sizeof(void *), hipMemcpyHostToDevice, s->stream));
    const void *const *p = (const void *const *)buf.p;
    S.key_off = (const uint32_t *const *)(p + 0 * G); S.lo = (const uint32_t *const *)(p + 1 * G);
    S.hi = (const uint32_t *const *)(p + 2 * G); S.val_off = (const uint32_t *const *)(p + 3 * G);
    S.vals = (const uint32_t *const *)(p + 4 * G); S.x_off = (const uint32_t *const *)(p + 5 * G);
    S.x = (const int32_t *const *)(p + 6 * G);
    S.val_cnt = (const uint32_t *const *)(p + 7 * G);
    S.G = (uint32_t)G;
    S.range = range;
    return ACCORD_OK;
}

// exclusive scans with their totals read back in one sync
struct Scans {
    accord_store *s;
    int k = 0;
    unsigned long long *dev;
    int32_t add(const uint32_t *in, uint32_t *out, uint32_t n)
    {
        HIPCHECK(s, s->op_tmp[T_SCAN].ensure_zeroed(accord::scan_temp_bytes(n), s->stream));
        accord::exclusive_scan_u32(in, out, n, dev + k++, s->op_tmp[T_SCAN].p, s->stream);
        return ACCORD_OK;
    }
    int32_t read(unsigned long long *h)
    {
        HIPCHECK(s, hipMemcpyAsync(s->pinned->totals, dev, (size_t)k * 8, hipMemcpyDeviceToHost, s->stream));
        HIPCHECK(s, hipStreamSynchronize(s->stream));
        for (int i = 0; i < k; ++i) h[i] = s->pinned->totals[i];
        k = 0;
        return ACCORD_OK;
    }
};

int32_t scans_init(accord_store *s, Scans &sc)
{
    sc.s = s;
    HIPCHECK(s, s->op_tmp[T_TOT].ensure(8 * 8));
    sc.dev = s->op_tmp[T_TOT].as<unsigned long long>();
    return ACCORD_OK;
}

#define RC(expr) do { int32_t rc_ = (expr); if (rc_) return rc_; } while (0)

int32_t check_views(accord_store *s, uint32_t np, const accord_deps *parts)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (!parts || np == 0) return fail(s, ACCORD_ERR_ARG, "no deps sets");
    for (uint32_t g = 1; g < np; ++g)
        if (parts[g].n != parts[0].n) return fail(s, ACCORD_ERR_ARG, "deps sets cover different txn counts");
    if ((uint64_t)parts[0].n + 1 >= (1ull << 31)) return fail(s, ACCORD_ERR_CAPACITY, "too many txns");
    return ACCORD_OK;
}

// Union of one side of G parts into the given output buffers of `o`.
// totals_known: the parts' *_total fields are exact (the store's own views), so the input sizes
// need no device read
int32_t union_side(accord_store *s, const accord_deps *parts, uint32_t G, bool range, DepSet &o, bool totals_known = false)
{
    const uint32_t n = parts[0].n;
    const size_t nG = (size_t)n * G, n1 = (size_t)n + 1;
    if (nG >= (1ull << 32)) return fail(s, ACCORD_ERR_CAPACITY, "union of %u x %u lists", n, G);
    std::vector<SideView> v(G);
    for (uint32_t g = 0; g < G; ++g) v[g] = side_of(parts[g], range);
    accord::DsUnionParams p{};
    p.n = n;
    RC(make_side(s, v, range, s->op_tmp[T_PTRS], p.S));
    DevBuf *T = s->op_tmp;
    for (int b : {T_VLEN, T_KLEN, T_BLEN, T_VLST, T_KLST, T_BTOT}) HIPCHECK(s, T[b].ensure(nG * 4 + 4));
    for (int b : {T_VEOFF, T_KEOFF, T_BEOFF}) HIPCHECK(s, T[b].ensure(nG * 4 + 4));
    HIPCHECK(s, T[T_CNTV].ensure(n1 * 4)); HIPCHECK(s, T[T_CNTK].ensure(n1 * 4));
    p.vlen = T[T_VLEN].as<uint32_t>(); p.klen = T[T_KLEN].as<uint32_t>(); p.blen = T[T_BLEN].as<uint32_t>();
    p.veoff = T[T_VEOFF].as<uint32_t>(); p.keoff = T[T_KEOFF].as<uint32_t>(); p.beoff = T[T_BEOFF].as<uint32_t>();
    Scans sc;
    RC(scans_init(s, sc));
    accord::launch_union_lens(p, s->stream);
    RC(sc.add(p.vlen, T[T_VEOFF].as<uint32_t>(), (uint32_t)nG));
    RC(sc.add(p.klen, T[T_KEOFF].as<uint32_t>(), (uint32_t)nG));
    RC(sc.add(p.blen, T[T_BEOFF].as<uint32_t>(), (uint32_t)nG));
    unsigned long long tot[3] = {0, 0, 0};
    if (totals_known) {
        for (uint32_t g = 0; g < G; ++g) {
            const uint64_t nk = range ? parts[g].rd_rngs_total : parts[g].kd_keys_total;
            tot[0] += range ? parts[g].rd_vals_total : parts[g].kd_vals_total;
            tot[1] += nk;
            tot[2] += (range ? parts[g].rd_r2v_total : parts[g].kd_k2v_total) - nk;
        }
        sc.k = 0;
    } else {
        RC(sc.read(tot));
    }
    const uint64_t V = tot[0], K = tot[1], B = tot[2];
    if (V >= (1ull << 32) || K >= (1ull << 32) || B >= (1ull << 32)) return fail(s, ACCORD_ERR_CAPACITY, "union input over 2^32 elements");
    HIPCHECK(s, T[T_VOWN].ensure(V * 4 + 4)); HIPCHECK(s, T[T_VRANK].ensure(V * 4 + 4));
    HIPCHECK(s, T[T_KOWN].ensure(K * 4 + 4)); HIPCHECK(s, T[T_KRANK].ensure(K * 4 + 4));
    HIPCHECK(s, T[T_RB].ensure(B * 4 + 4)); HIPCHECK(s, T[T_BOWN].ensure(B * 4 + 4));
    p.vown = T[T_VOWN].as<uint32_t>(); p.vlst = T[T_VLST].as<uint32_t>();
    p.kown = T[T_KOWN].as<uint32_t>(); p.klst = T[T_KLST].as<uint32_t>();
    p.cnt_vals = T[T_CNTV].as<uint32_t>(); p.cnt_keys = T[T_CNTK].as<uint32_t>();
    accord::launch_union_owners(p, s->stream);
    DevBuf &key_off = range ? o.rng_off : o.key_off, &val_off = range ? o.rval_off : o.val_off, &x_off = range ? o.r_off : o.x_off;
    HIPCHECK(s, key_off.ensure(n1 * 4)); HIPCHECK(s, val_off.ensure(n1 * 4)); HIPCHECK(s, x_off.ensure(n1 * 4));
    RC(sc.add(p.cnt_vals, val_off.as<uint32_t>(), n));
    RC(sc.add(p.cnt_keys, key_off.as<uint32_t>(), n));
    // with the input sizes known the outputs are sized at their bounds (a union holds at most its
    // inputs' elements; the body scan runs over K positions, zero past the union's) and the three
    // totals are read once, at the end; otherwise each size is read before its buffers
    uint64_t UV = V, UK = K;
    if (!totals_known) {
        RC(sc.read(tot));
        UV = tot[0]; UK = tot[1];
    }
    DevBuf &lo = range ? o.rng_start : o.keys, &vals = range ? o.rvals : o.vals, &x = range ? o.r : o.x;
    HIPCHECK(s, lo.ensure(UK * 4 + 4)); HIPCHECK(s, vals.ensure(UV * 4 + 4));
    if (range) HIPCHECK(s, o.rng_end.ensure(UK * 4 + 4));
    HIPCHECK(s, T[T_BSZ].ensure(UK * 4 + 4)); HIPCHECK(s, T[T_BSCAN].ensure(UK * 4 + 8));
    HIPCHECK(s, hipMemsetAsync(T[T_BSZ].p, 0, UK * 4 + 4, s->stream));
    p.out_val_off = val_off.as<uint32_t>(); p.out_key_off = key_off.as<uint32_t>();
    p.vrank = T[T_VRANK].as<uint32_t>(); p.krank = T[T_KRANK].as<uint32_t>(); p.rb = T[T_RB].as<uint32_t>();
    p.bown = T[T_BOWN].as<uint32_t>(); p.btot = T[T_BTOT].as<uint32_t>(); p.bsz = T[T_BSZ].as<uint32_t>();
    p.out_vals = vals.as<uint32_t>(); p.out_lo = lo.as<uint32_t>(); p.out_hi = range ? o.rng_end.as<uint32_t>() : nullptr;
    accord::launch_union_ranks(p, s->stream);
    RC(sc.add(p.bsz, T[T_BSCAN].as<uint32_t>(), (uint32_t)UK));
    uint64_t UB = B;
    if (!totals_known) {
        RC(sc.read(tot));
        UB = tot[0];
    }
    HIPCHECK(s, x.ensure((UK + UB) * 4 + 4));
    p.bscan = T[T_BSCAN].as<uint32_t>();
    p.out_x_off = x_off.as<uint32_t>(); p.out_x = x.as<int32_t>();
    if (n == 0) HIPCHECK(s, hipMemsetAsync(x_off.p, 0, 4, s->stream));
    accord::launch_union_write(p, s->stream);
    HIPCHECK(s, hipGetLastError());
    if (totals_known) {
        RC(sc.read(tot));
        UV = tot[0]; UK = tot[1]; UB = tot[2];
    }
    if (range) { o.tot_rngs = UK; o.tot_rvals = UV; o.tot_r = UK + UB; }
    else { o.tot_keys = UK; o.tot_vals = UV; o.tot_x = UK + UB; }
    return ACCORD_OK;
}

// linearUnion with an empty side is the other side verbatim (both are in canonical form): its
// arrays copied into o in one launch instead of the union's passes and host reads
int32_t copy_side(accord_store *s, const accord_deps &src, bool range, DepSet &o)
{
    if (!range && src.kd_val_cnt) {        // gapped txnIds (a compute result): the dense form, then copy it
        if (src.kd_val_off != s->vub_off.as<uint32_t>())
            return fail(s, ACCORD_ERR_ARG, "copy of a gapped deps view of another store");
        RC(accord_impl::store_dense_keydeps(s));
        HIPCHECK(s, hipMemcpyAsync(s->pinned->totals, &s->status_totals.as<HostTotals>()->totals[7], 8,
                                   hipMemcpyDeviceToHost, s->stream));
        HIPCHECK(s, hipStreamSynchronize(s->stream));
        accord_deps d = src;
        d.kd_val_off = s->kd_val_off.as<uint32_t>(); d.kd_vals = s->kd_vals.as<uint32_t>();
        d.kd_val_cnt = nullptr;
        d.kd_vals_total = s->pinned->totals[0];
        return copy_side(s, d, range, o);
    }
    const size_t n1 = (size_t)src.n + 1;
    const uint64_t K = range ? src.rd_rngs_total : src.kd_keys_total, V = range ? src.rd_vals_total : src.kd_vals_total;
    const uint64_t X = range ? src.rd_r2v_total : src.kd_k2v_total;
    DevBuf &key_off = range ? o.rng_off : o.key_off, &val_off = range ? o.rval_off : o.val_off, &x_off = range ? o.r_off : o.x_off;
    DevBuf &lo = range ? o.rng_start : o.keys, &vals = range ? o.rvals : o.vals, &x = range ? o.r : o.x;
    HIPCHECK(s, key_off.ensure(n1 * 4)); HIPCHECK(s, val_off.ensure(n1 * 4)); HIPCHECK(s, x_off.ensure(n1 * 4));
    HIPCHECK(s, lo.ensure(K * 4 + 4)); HIPCHECK(s, vals.ensure(V * 4 + 4)); HIPCHECK(s, x.ensure(X * 4 + 4));
    if (range) HIPCHECK(s, o.rng_end.ensure(K * 4 + 4));
    accord::CopyList cl;
    cl.add(range ? src.rd_rng_off : src.kd_key_off, key_off.p, n1 * 4);
    cl.add(range ? src.rd_val_off : src.kd_val_off, val_off.p, n1 * 4);
    cl.add(range ? src.rd_r2v_off : src.kd_k2v_off, x_off.p, n1 * 4);
    cl.add(range ? src.rd_rng_start : src.kd_keys, lo.p, K * 4);
    cl.add(range ? src.rd_vals : src.kd_vals, vals.p, V * 4);
    cl.add(range ? (const void *)src.rd_r2v : (const void *)src.kd_k2v, x.p, X * 4);
    if (range) cl.add(src.rd_rng_end, o.rng_end.p, K * 4);
    accord::launch_copy_words(cl, s->stream);
    HIPCHECK(s, hipGetLastError());
    if (range) { o.tot_rngs = K; o.tot_rvals = V; o.tot_r = X; }
    else { o.tot_keys = K; o.tot_vals = V; o.tot_x = X; }
    return ACCORD_OK;
}

int32_t slice_side(accord_store *s, const accord_deps &src, bool range, const uint32_t *d_sel_off,
                   const uint32_t *d_ss, const uint32_t *d_se, uint32_t nsel, DepSet &o)
{
    const uint32_t n = src.n;
    const size_t n1 = (size_t)n + 1;
    const uint64_t K = range ? src.rd_rngs_total : src.kd_keys_total, V = range ? src.rd_vals_total : src.kd_vals_total;
    accord::DsSliceParams p{};
    p.n = n;
    std::vector<SideView> v{side_of(src, range)};
    RC(make_side(s, v, range, s->op_tmp[T_PTRS], p.S));
    DevBuf *T = s->op_tmp;
    HIPCHECK(s, T[T_KRANK].ensure(K * 4 + 4));          // ksel
    HIPCHECK(s, T[T_VLST].ensure(n1 * 4));              // mode
    HIPCHECK(s, T[T_CNTK].ensure(n1 * 4)); HIPCHECK(s, T[T_CNTV].ensure(n1 * 4)); HIPCHECK(s, T[T_KLST].ensure(n1 * 4));
    HIPCHECK(s, T[T_VOWN].ensure(V * 4 + 4));           // used
    HIPCHECK(s, T[T_VRANK].ensure(V * 4 + 4));          // remap
    HIPCHECK(s, hipMemsetAsync(T[T_VOWN].p, 0, V * 4 + 4, s->stream));
    p.sel_off = d_sel_off; p.sel_start = d_ss; p.sel_end = d_se; p.nsel = nsel;
    p.ksel = T[T_KRANK].as<uint32_t>(); p.mode = T[T_VLST].as<uint32_t>();
    p.cnt_keys = T[T_CNTK].as<uint32_t>(); p.cnt_vals = T[T_CNTV].as<uint32_t>(); p.cnt_x = T[T_KLST].as<uint32_t>();
    p.used = T[T_VOWN].as<uint32_t>(); p.remap = T[T_VRANK].as<uint32_t>();
    accord::launch_slice_select(p, s->stream);
    DevBuf &key_off = range ? o.rng_off : o.key_off, &val_off = range ? o.rval_off : o.val_off, &x_off = range ? o.r_off : o.x_off;
    HIPCHECK(s, key_off.ensure(n1 * 4)); HIPCHECK(s, val_off.ensure(n1 * 4)); HIPCHECK(s, x_off.ensure(n1 * 4));
    Scans sc;
    RC(scans_init(s, sc));
    RC(sc.add(p.cnt_keys, key_off.as<uint32_t>(), n));
    RC(sc.add(p.cnt_vals, val_off.as<uint32_t>(), n));
    RC(sc.add(p.cnt_x, x_off.as<uint32_t>(), n));
    unsigned long long tot[3];
    RC(sc.read(tot));
    DevBuf &lo = range ? o.rng_start : o.keys, &vals = range ? o.rvals : o.vals, &x = range ? o.r : o.x;
    HIPCHECK(s, lo.ensure(tot[0] * 4 + 4)); HIPCHECK(s, vals.ensure(tot[1] * 4 + 4)); HIPCHECK(s, x.ensure(tot[2] * 4 + 4));
    if (range) HIPCHECK(s, o.rng_end.ensure(tot[0] * 4 + 4));
    p.out_key_off = key_off.as<uint32_t>(); p.out_val_off = val_off.as<uint32_t>(); p.out_x_off = x_off.as<uint32_t>();
    p.out_lo = lo.as<uint32_t>(); p.out_hi = range ? o.rng_end.as<uint32_t>() : nullptr;
    p.out_vals = vals.as<uint32_t>(); p.out_x = x.as<int32_t>();
    accord::launch_slice_write(p, s->stream);
    HIPCHECK(s, hipGetLastError());
    if (range) { o.tot_rngs = tot[0]; o.tot_rvals = tot[1]; o.tot_r = tot[2]; }
    else { o.tot_keys = tot[0]; o.tot_vals = tot[1]; o.tot_x = tot[2]; }
    return ACCORD_OK;
}

void op_begin(accord_store *s)
{
    if (s->events) (void)hipEventRecord(s->ev[EV_OP_START], s->stream);
}
int32_t op_end(accord_store *s)
{
    if (s->events) {
        (void)hipEventRecord(s->ev[EV_OP_END], s->stream);
        (void)hipEventSynchronize(s->ev[EV_OP_END]);
        (void)hipEventElapsedTime(&s->ops_ms, s->ev[EV_OP_START], s->ev[EV_OP_END]);
    }
    HIPCHECK(s, hipStreamSynchronize(s->stream));
    return ACCORD_OK;
}

DepSet &next_set(accord_store *s)
{
    return s->ds[s->ds_cur == 0 ? 1 : 0];
}

void publish(accord_store *s, DepSet &o, uint32_t n)
{
    o.n = n;
    s->ds_cur = (&o == &s->ds[0]) ? 0 : 1;
    s->ds_rb = false;
    s->computed = true;
    s->wo_done = false;
}

struct InverseOwner {
    std::vector<uint32_t> koff, roff;
    std::vector<int32_t> k, r;
};

} // namespace

namespace accord_impl {

// The redundant RangeDeps of every txn of the computed batch (RedundantBefore.collectDeps,
// redundant.hip), then PartialDeps.with of the computed deps and it (linearUnion on both sides,
// as accord_deps_union): messages/PreAccept.java:262-263.
static accord::RbParams rb_params(accord_store *s)
{
    const uint32_t n = s->n;
    const size_t n1 = (size_t)n + 1;
    HostTotals *dev = s->status_totals.as<HostTotals>();
    accord::RbParams p{};
    p.n = n;
    p.msb = s->msb.as<uint64_t>();
    p.exec_msb = s->has_exec ? s->exec_msb.as<uint64_t>() : nullptr;
    p.key_off = s->key_off.as<uint32_t>(); p.key_ord = s->key_ord.as<uint32_t>();
    p.rng_off = s->R ? s->rng_off.as<uint32_t>() : nullptr;
    p.rng_start = s->R ? s->rng_start.as<uint32_t>() : nullptr;
    p.rng_end = s->R ? s->rng_end.as<uint32_t>() : nullptr;
    p.m = s->rb_m;
    p.e_start = s->rb_start.as<uint32_t>(); p.e_end = s->rb_end.as<uint32_t>(); p.e_bound = s->rb_bound.as<uint32_t>();
    p.e_start_epoch = s->rb_sep.as<uint64_t>(); p.e_end_epoch = s->rb_eep.as<uint64_t>();
    p.min_epoch = s->rb_min_epoch;
    uint32_t *cnt = s->rb_cnt.as<uint32_t>();
    p.cnt_rngs = cnt; p.cnt_vals = cnt + n1; p.cnt_r2v = cnt + 2 * n1;
    p.status = &dev->rb_status;
    return p;
}

int32_t redundant_count(accord_store *s)
{
    const uint32_t n = s->n;
    const size_t n1 = (size_t)n + 1;
    hipStream_t st = s->stream;
    DepSet &r = s->rb_set;
    HIPCHECK(s, s->rb_cnt.ensure(3 * n1 * 4));
    HIPCHECK(s, r.rng_off.ensure(n1 * 4)); HIPCHECK(s, r.rval_off.ensure(n1 * 4)); HIPCHECK(s, r.r_off.ensure(n1 * 4));
    HostTotals *dev = s->status_totals.as<HostTotals>();
    if (!s->rb_status_zeroed) {   // (the compute's init launch zeroes them when it runs first)
        accord::FillList fl;
        fl.add(&dev->rb_status.first, sizeof(dev->rb_status.first), 0xFFFFFFFFu);
        fl.add(&dev->rb_status.overflow, 4, 0u);
        fl.add(&dev->rb_status.overflow_first, 4, 0xFFFFFFFFu);
        accord::launch_fill_words(fl, st);
    }
    s->rb_status_zeroed = false;
    const accord::RbParams p = rb_params(s);
    accord::launch_rb_count(p, st);
    HIPCHECK(s, s->op_tmp[T_SCAN].ensure_zeroed(accord::scan_temp_bytes(n), st));
    void *tmp = s->op_tmp[T_SCAN].p;
    {   // the three offsets in one launch
        const uint32_t *in[3] = {p.cnt_rngs, p.cnt_vals, p.cnt_r2v};
        uint32_t *out[3] = {r.rng_off.as<uint32_t>(), r.rval_off.as<uint32_t>(), r.r_off.as<uint32_t>()};
        unsigned long long *tot[3] = {&dev->rb_tot[0], &dev->rb_tot[1], &dev->rb_tot[2]};
        accord::exclusive_scan_multi(3, in, out, tot, n, tmp, st);
    }
    HIPCHECK(s, hipGetLastError());
    return ACCORD_OK;
}

int32_t redundant_apply(accord_store *s)
{
    const uint32_t n = s->n;
    const size_t n1 = (size_t)n + 1;
    hipStream_t st = s->stream;
    DepSet &r = s->rb_set;
    if (s->pinned->rb_status.overflow)
        return fail(s, ACCORD_ERR_CAPACITY, "%u txns touch more than %u RedundantBefore entries (first: txn %u)",
                    s->pinned->rb_status.overflow, accord::RB_MAX, s->pinned->rb_status.overflow_first);
    const unsigned long long tot[3] = {s->pinned->rb_tot[0], s->pinned->rb_tot[1], s->pinned->rb_tot[2]};
    HIPCHECK(s, s->rb_zero.ensure(n1 * 4));
    HIPCHECK(s, hipMemsetAsync(s->rb_zero.p, 0, n1 * 4, st));
    accord::RbParams p = rb_params(s);
    HIPCHECK(s, r.rng_start.ensure(tot[0] * 4 + 4)); HIPCHECK(s, r.rng_end.ensure(tot[0] * 4 + 4));
    HIPCHECK(s, r.rvals.ensure(tot[1] * 4 + 4)); HIPCHECK(s, r.r.ensure(tot[2] * 4 + 4));
    p.rng_off_out = r.rng_off.as<uint32_t>(); p.val_off_out = r.rval_off.as<uint32_t>(); p.r2v_off_out = r.r_off.as<uint32_t>();
    p.out_start = r.rng_start.as<uint32_t>(); p.out_end = r.rng_end.as<uint32_t>();
    p.out_vals = r.rvals.as<uint32_t>(); p.out_r2v = r.r.as<int32_t>();
    accord::launch_rb_fill(p, st);
    HIPCHECK(s, hipGetLastError());
    accord_deps parts[2];
    RC(accord_deps_device_view(s, &parts[0]));
    std::memset(&parts[1], 0, sizeof(parts[1]));
    parts[1].n = n;
    parts[1].kd_key_off = parts[1].kd_val_off = parts[1].kd_k2v_off = s->rb_zero.as<uint32_t>();
    parts[1].rd_rngs_total = tot[0]; parts[1].rd_vals_total = tot[1]; parts[1].rd_r2v_total = tot[2];
    parts[1].rd_rng_off = r.rng_off.as<uint32_t>(); parts[1].rd_rng_start = r.rng_start.as<uint32_t>();
    parts[1].rd_rng_end = r.rng_end.as<uint32_t>(); parts[1].rd_val_off = r.rval_off.as<uint32_t>();
    parts[1].rd_vals = r.rvals.as<uint32_t>(); parts[1].rd_r2v_off = r.r_off.as<uint32_t>();
    parts[1].rd_r2v = r.r.as<int32_t>();
    DepSet &o = next_set(s);
    // the redundant deps are RangeDeps only: the KeyDeps side is the computed one verbatim, and a
    // RangeDeps side with an empty part is the other part
    RC(copy_side(s, parts[0], false, o));
    if (parts[0].rd_rngs_total == 0) RC(copy_side(s, parts[1], true, o));
    else if (tot[0] == 0) RC(copy_side(s, parts[0], true, o));
    else RC(union_side(s, parts, 2, true, o, true));
    HIPCHECK(s, hipStreamSynchronize(st));
    publish(s, o, n);
    s->ds_rb = true;
    return ACCORD_OK;
}

CurDeps cur_deps(const accord_store *s)
{
    CurDeps c{};
    if (s->ds_cur >= 0) {
        const DepSet &x = s->ds[s->ds_cur];
        c.kd_key_off = x.key_off.as<uint32_t>(); c.kd_keys = x.keys.as<uint32_t>();
        c.kd_val_off = x.val_off.as<uint32_t>(); c.kd_vals = x.vals.as<uint32_t>();
        c.kd_k2v_off = x.x_off.as<uint32_t>(); c.kd_k2v = x.x.as<uint32_t>();
        c.rd_val_off = x.rval_off.as<uint32_t>(); c.rd_vals = x.rvals.as<uint32_t>();
        c.rd_rng_off = x.rng_off.as<uint32_t>(); c.rd_rng_start = x.rng_start.as<uint32_t>();
        c.rd_rng_end = x.rng_end.as<uint32_t>(); c.rd_r2v_off = x.r_off.as<uint32_t>(); c.rd_r2v = x.r.as<uint32_t>();
        c.tot_keys = x.tot_keys; c.tot_vals = x.tot_vals; c.tot_k2v = x.tot_x; c.tot_rvals = x.tot_rvals;
        c.tot_rngs = x.tot_rngs; c.tot_r2v = x.tot_r;
    } else {
        c.kd_key_off = s->kd_key_off.as<uint32_t>(); c.kd_keys = s->kd_keys.as<uint32_t>();
        c.kd_val_off = s->vub_off.as<uint32_t>(); c.kd_vals = s->vgap.as<uint32_t>();   // gapped
        c.kd_val_cnt = s->cnt_vals.as<uint32_t>();
        c.kd_k2v_off = s->kd_k2v_off.as<uint32_t>(); c.kd_k2v = s->kd_k2v.as<uint32_t>();
        c.rd_val_off = s->rd_val_off.as<uint32_t>(); c.rd_vals = s->rd_vals.as<uint32_t>();
        c.rd_rng_off = s->rd_rng_off.as<uint32_t>(); c.rd_rng_start = s->rd_rng_start.as<uint32_t>();
        c.rd_rng_end = s->rd_rng_end.as<uint32_t>(); c.rd_r2v_off = s->rd_r2v_off.as<uint32_t>();
        c.rd_r2v = s->rd_r2v.as<uint32_t>();
        c.tot_keys = s->tot_keys; c.tot_vals = s->tot_vals; c.tot_k2v = s->tot_k2v; c.tot_rvals = s->tot_rvals;
        c.tot_rngs = s->tot_rngs; c.tot_r2v = s->tot_r2v;
    }
    return c;
}

} // namespace accord_impl

extern "C" {

int32_t accord_redundant_before_set(accord_store *s, uint32_t m, const uint32_t *start, const uint32_t *end,
                                    const uint64_t *start_epoch, const uint64_t *end_epoch, const uint32_t *bound,
                                    uint64_t min_epoch)
{
    return accord_redundant_before_set_ex(s, m, start, end, start_epoch, end_epoch, bound, nullptr, nullptr, nullptr,
                                          min_epoch);
}

int32_t accord_redundant_before_set_ex(accord_store *s, uint32_t m, const uint32_t *start, const uint32_t *end,
                                       const uint64_t *start_epoch, const uint64_t *end_epoch, const uint32_t *bound,
                                       const uint32_t *local, const uint32_t *boot, const uint8_t *stale,
                                       uint64_t min_epoch)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (m && (!start || !end || !start_epoch || !end_epoch || !bound)) return fail(s, ACCORD_ERR_ARG, "null argument");
    for (uint32_t i = 0; i < m; ++i) {
        if (!(start[i] < end[i])) return fail(s, ACCORD_ERR_RANGES, "RedundantBefore entry %u is empty", i);
        if (i && end[i - 1] > start[i])
            return fail(s, ACCORD_ERR_RANGES, "RedundantBefore entries %u, %u not ascending and disjoint", i - 1, i);
    }
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    // the rest of each entry (removeRedundantDependencies); absent arrays: NONE, NONE, not stale
    bool ext = false;
    for (uint32_t i = 0; i < m && !ext; ++i)
        ext = (local && local[i] != ACCORD_NO_TXN) || (boot && boot[i] != ACCORD_NO_TXN) || (stale && stale[i]);
    if (m) {   // every array staged in page-locked memory, one host-to-device copy, one scatter launch
        const size_t w4 = ((size_t)m + 3) / 4;              // stale bytes, in words
        const size_t words = (size_t)m * (3 + 2 + 2) + (ext ? (size_t)m * 2 + w4 : 0);
        if (s->rb_host_cap < words * 4) {
            if (s->rb_host) (void)hipHostFree(s->rb_host);
            s->rb_host = nullptr; s->rb_host_cap = 0;
            HIPCHECK(s, hipHostMalloc(&s->rb_host, words * 8, hipHostMallocDefault));
            s->rb_host_cap = words * 8;
        }
        HIPCHECK(s, s->rb_pack.ensure(words * 4));
        HIPCHECK(s, s->rb_start.ensure((size_t)m * 4)); HIPCHECK(s, s->rb_end.ensure((size_t)m * 4));
        HIPCHECK(s, s->rb_bound.ensure((size_t)m * 4));
        HIPCHECK(s, s->rb_sep.ensure((size_t)m * 8)); HIPCHECK(s, s->rb_eep.ensure((size_t)m * 8));
        uint32_t *h = (uint32_t *)s->rb_host;
        const uint32_t *dp = s->rb_pack.as<uint32_t>();
        accord::CopyList cl;
        size_t o = 0;
        auto put = [&](const void *src, size_t nw, void *dst) {
            std::memcpy(h + o, src, nw * 4);
            cl.add(dp + o, dst, nw * 4);
            o += nw;
        };
        put(start, m, s->rb_start.p); put(end, m, s->rb_end.p); put(bound, m, s->rb_bound.p);
        put(start_epoch, (size_t)m * 2, s->rb_sep.p); put(end_epoch, (size_t)m * 2, s->rb_eep.p);
        if (ext) {
            HIPCHECK(s, s->rb_local.ensure((size_t)m * 4)); HIPCHECK(s, s->rb_boot.ensure((size_t)m * 4));
            HIPCHECK(s, s->rb_stale.ensure(w4 * 4 + 8));
            uint32_t *lo = h + o;
            for (uint32_t i = 0; i < m; ++i) lo[i] = local ? local[i] : ACCORD_NO_TXN;
            cl.add(dp + o, s->rb_local.p, (size_t)m * 4); o += m;
            uint32_t *bo = h + o;
            for (uint32_t i = 0; i < m; ++i) bo[i] = boot ? boot[i] : ACCORD_NO_TXN;
            cl.add(dp + o, s->rb_boot.p, (size_t)m * 4); o += m;
            uint8_t *st = (uint8_t *)(h + o);
            std::memset(st, 0, w4 * 4);
            for (uint32_t i = 0; i < m; ++i) st[i] = stale && stale[i] ? 1 : 0;
            cl.add(dp + o, s->rb_stale.p, w4 * 4); o += w4;
        }
        HIPCHECK(s, hipMemcpyAsync(s->rb_pack.p, s->rb_host, o * 4, hipMemcpyHostToDevice, s->stream));
        accord::launch_copy_words(cl, s->stream);
        HIPCHECK(s, hipStreamSynchronize(s->stream));     // the staging is reused by the next call
    }
    if (ext != s->rb_ext || ext) s->rdy_force_full = true;   // readiness re-evaluates everything
    s->rb_ext = ext;
    s->rb_m = m;
    s->rb_min_epoch = min_epoch;
    if (accord_impl::registered_mode(s)) RC(accord_impl::status_truncate_carry(s, m, start, end, bound));
    return ACCORD_OK;
}

int32_t accord_deps_union(accord_store *s, uint32_t nparts, const accord_deps *parts)
{
    RC(check_views(s, nparts, parts));
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    op_begin(s);
    // up to 64 parts per pass; more fold into the running result (linearUnion is associative).  A
    // later pass writes the buffer the store's current deps sat in, so those must come first.
    for (uint32_t g = 64; g < nparts; ++g)
        for (const DepSet &d : s->ds)
            if (d.key_off.p && parts[g].kd_key_off == d.key_off.as<uint32_t>())
                return fail(s, ACCORD_ERR_ARG, "union part %u is this store's own deps set: pass it among the first 64", g);
    const uint32_t n = parts[0].n;
    uint32_t done = 0;
    std::vector<accord_deps> grp;
    while (done < nparts) {
        grp.clear();
        if (done) {
            grp.emplace_back();
            RC(accord_deps_device_view(s, &grp.back()));   // the union so far
        }
        const uint32_t take = std::min<uint32_t>(nparts - done, 64u - (uint32_t)grp.size());
        grp.insert(grp.end(), parts + done, parts + done + take);
        done += take;
        DepSet &o = next_set(s);
        RC(union_side(s, grp.data(), (uint32_t)grp.size(), false, o));
        RC(union_side(s, grp.data(), (uint32_t)grp.size(), true, o));
        HIPCHECK(s, hipStreamSynchronize(s->stream));
        publish(s, o, n);
    }
    RC(op_end(s));
    return ACCORD_OK;
}

int32_t accord_deps_slice(accord_store *s, const accord_deps *src, const uint32_t *sel_off, const uint32_t *sel_start,
                          const uint32_t *sel_end, uint32_t nsel)
{
    RC(check_views(s, 1, src));
    const uint32_t n = src->n;
    const uint64_t total = sel_off ? sel_off[n] : nsel;
    if (total && (!sel_start || !sel_end)) return fail(s, ACCORD_ERR_ARG, "select ranges without bounds");
    if (sel_off && sel_off[0] != 0) return fail(s, ACCORD_ERR_ARG, "select CSR must start at 0");
    // Ranges invariants (AbstractRanges.sortAndDeoverlap): non-empty, sorted, de-overlapped
    for (uint32_t t = 0; t < (sel_off ? n : 1); ++t) {
        const uint64_t a = sel_off ? sel_off[t] : 0, b = sel_off ? sel_off[t + 1] : nsel;
        if (b < a) return fail(s, ACCORD_ERR_ARG, "select CSR offsets decrease at txn %u", t);
        for (uint64_t q = a; q < b; ++q) {
            if (sel_start[q] >= sel_end[q]) return fail(s, ACCORD_ERR_RANGES, "empty select range (%u,%u]", sel_start[q], sel_end[q]);
            if (q > a && sel_start[q] < sel_end[q - 1]) return fail(s, ACCORD_ERR_RANGES, "select ranges not sorted/de-overlapped");
        }
    }
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    op_begin(s);
    DevBuf *T = s->op_tmp;
    HIPCHECK(s, T[T_SEL0].ensure(((size_t)n + 1) * 4));
    HIPCHECK(s, T[T_SEL1].ensure(total * 8 + 8));
    uint32_t *d_off = sel_off ? T[T_SEL0].as<uint32_t>() : nullptr;
    uint32_t *d_ss = T[T_SEL1].as<uint32_t>(), *d_se = d_ss + total;
    if (sel_off) HIPCHECK(s, hipMemcpyAsync(d_off, sel_off, ((size_t)n + 1) * 4, hipMemcpyHostToDevice, s->stream));
    if (total) {
        HIPCHECK(s, hipMemcpyAsync(d_ss, sel_start, total * 4, hipMemcpyHostToDevice, s->stream));
        HIPCHECK(s, hipMemcpyAsync(d_se, sel_end, total * 4, hipMemcpyHostToDevice, s->stream));
    }
    DepSet &o = next_set(s);
    RC(slice_side(s, *src, false, d_off, d_ss, d_se, nsel, o));
    RC(slice_side(s, *src, true, d_off, d_ss, d_se, nsel, o));
    RC(op_end(s));
    publish(s, o, n);
    return ACCORD_OK;
}

int32_t accord_deps_invert(accord_store *s, const accord_deps *src, accord_deps_inverse *out)
{
    RC(check_views(s, 1, src));
    if (!out) return fail(s, ACCORD_ERR_ARG, "null output");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    const uint32_t n = src->n;
    InverseOwner *own = new (std::nothrow) InverseOwner();
    if (!own) return fail(s, ACCORD_ERR_OOM, "out of host memory");
    op_begin(s);
    int32_t rc = ACCORD_OK;
    for (int side = 0; side < 2 && rc == ACCORD_OK; ++side) {
        const bool range = side == 1;
        const uint64_t V = range ? src->rd_vals_total : src->kd_vals_total;   // (gapped: the array length)
        accord::DsInvertParams p{};
        p.n = n;
        std::vector<SideView> v{side_of(*src, range)};
        if ((rc = make_side(s, v, range, s->op_tmp[T_PTRS], p.S))) break;
        DevBuf *T = s->op_tmp;
        hipError_t e = T[T_VLEN].ensure(((size_t)n + 1) * 4);
        if (e == hipSuccess) e = T[T_KLEN].ensure(((size_t)n + 1) * 4);
        if (e != hipSuccess) { rc = fail(s, ACCORD_ERR_HIP, "invert: %s", hipGetErrorString(e)); break; }
        // per txn |txnIds| + body, scanned: the inverse's offsets and its exact size
        p.sizes = T[T_KLEN].as<uint32_t>(); p.out_off = T[T_VLEN].as<uint32_t>();
        accord::launch_invert_sizes(p, s->stream);
        Scans sc;
        unsigned long long tot[1] = {0};
        if ((rc = scans_init(s, sc)) || (rc = sc.add(p.sizes, p.out_off, n)) || (rc = sc.read(tot))) break;
        const uint64_t total = tot[0];
        e = T[T_RB].ensure(total * 4 + 4);
        if (e == hipSuccess) e = T[T_VRANK].ensure(V * 4 + 4);
        if (e == hipSuccess) e = hipMemsetAsync(T[T_RB].p, 0, total * 4 + 4, s->stream);
        if (e != hipSuccess) { rc = fail(s, ACCORD_ERR_HIP, "invert: %s", hipGetErrorString(e)); break; }
        p.out = T[T_RB].as<int32_t>(); p.cursor = T[T_VRANK].as<uint32_t>();
        accord::launch_invert(p, s->stream);
        std::vector<uint32_t> &ho = range ? own->roff : own->koff;
        std::vector<int32_t> &hv = range ? own->r : own->k;
        try { ho.resize((size_t)n + 1); hv.resize(total + 1); } catch (...) { rc = fail(s, ACCORD_ERR_OOM, "out of host memory"); break; }
        e = hipMemcpyAsync(ho.data(), p.out_off, ((size_t)n + 1) * 4, hipMemcpyDeviceToHost, s->stream);
        if (e == hipSuccess && total) e = hipMemcpyAsync(hv.data(), p.out, total * 4, hipMemcpyDeviceToHost, s->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
        if (e == hipSuccess) e = hipGetLastError();
        if (e != hipSuccess) rc = fail(s, ACCORD_ERR_HIP, "invert: %s", hipGetErrorString(e));
        if (range) out->rd_total = total; else out->kd_total = total;
    }
    if (rc == ACCORD_OK) rc = op_end(s);
    if (rc != ACCORD_OK) { delete own; return rc; }
    out->n = n;
    out->kd_t2k_off = own->koff.data(); out->kd_t2k = own->k.data();
    out->rd_t2r_off = own->roff.data(); out->rd_t2r = own->r.data();
    out->owner = own;
    return ACCORD_OK;
}

int32_t accord_deps_upload(accord_store *s, const accord_deps *h)
{
    RC(check_views(s, 1, h));
    const uint32_t n = h->n;
    const size_t n1 = (size_t)n + 1;
    if (!h->kd_key_off || !h->kd_val_off || !h->kd_k2v_off || !h->rd_rng_off || !h->rd_val_off || !h->rd_r2v_off)
        return fail(s, ACCORD_ERR_ARG, "accord_deps_upload: missing offsets");
    const uint32_t *offs[6] = {h->kd_key_off, h->kd_val_off, h->kd_k2v_off, h->rd_rng_off, h->rd_val_off, h->rd_r2v_off};
    const uint64_t tots[6] = {h->kd_keys_total, h->kd_vals_total, h->kd_k2v_total, h->rd_rngs_total, h->rd_vals_total, h->rd_r2v_total};
    for (int a = 0; a < 6; ++a) {
        if (offs[a][0] != 0 || offs[a][n] != tots[a]) return fail(s, ACCORD_ERR_ARG, "accord_deps_upload: offsets/totals mismatch");
        for (uint32_t t = 0; t < n; ++t)
            if (offs[a][t + 1] < offs[a][t]) return fail(s, ACCORD_ERR_ARG, "accord_deps_upload: offsets decrease at txn %u", t);
    }
    // gapped txnIds (a downloaded compute result): made dense on the host, then uploaded
    std::vector<uint32_t> dv_off, dv;
    accord_deps hd = *h;
    if (h->kd_val_cnt) {
        dv_off.assign(n1, 0);
        for (uint32_t t = 0; t < n; ++t) {
            if ((uint64_t)h->kd_val_off[t] + h->kd_val_cnt[t] > h->kd_val_off[t + 1])
                return fail(s, ACCORD_ERR_ARG, "accord_deps_upload: txnIds count past the next offset at txn %u", t);
            dv_off[t + 1] = dv_off[t] + h->kd_val_cnt[t];
        }
        dv.resize(dv_off[n]);
        for (uint32_t t = 0; t < n; ++t)
            std::memcpy(dv.data() + dv_off[t], h->kd_vals + h->kd_val_off[t], (size_t)h->kd_val_cnt[t] * 4);
        hd.kd_val_off = dv_off.data(); hd.kd_vals = dv.data(); hd.kd_vals_total = dv_off[n]; hd.kd_val_cnt = nullptr;
        h = &hd;
    }
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    DepSet &o = next_set(s);
    struct { DevBuf *d; const void *src; size_t bytes; } cp[] = {
        {&o.key_off, h->kd_key_off, n1 * 4}, {&o.keys, h->kd_keys, h->kd_keys_total * 4},
        {&o.val_off, h->kd_val_off, n1 * 4}, {&o.vals, h->kd_vals, h->kd_vals_total * 4},
        {&o.x_off, h->kd_k2v_off, n1 * 4}, {&o.x, h->kd_k2v, h->kd_k2v_total * 4},
        {&o.rng_off, h->rd_rng_off, n1 * 4}, {&o.rng_start, h->rd_rng_start, h->rd_rngs_total * 4},
        {&o.rng_end, h->rd_rng_end, h->rd_rngs_total * 4}, {&o.rval_off, h->rd_val_off, n1 * 4},
        {&o.rvals, h->rd_vals, h->rd_vals_total * 4}, {&o.r_off, h->rd_r2v_off, n1 * 4},
        {&o.r, h->rd_r2v, h->rd_r2v_total * 4}};
    for (auto &c : cp) {
        HIPCHECK(s, c.d->ensure(c.bytes + 4));
        if (c.bytes) {
            if (!c.src) return fail(s, ACCORD_ERR_ARG, "accord_deps_upload: null data array");
            HIPCHECK(s, hipMemcpyAsync(c.d->p, c.src, c.bytes, hipMemcpyHostToDevice, s->stream));
        }
    }
    HIPCHECK(s, hipStreamSynchronize(s->stream));
    o.tot_keys = h->kd_keys_total; o.tot_vals = h->kd_vals_total; o.tot_x = h->kd_k2v_total;
    o.tot_rngs = h->rd_rngs_total; o.tot_rvals = h->rd_vals_total; o.tot_r = h->rd_r2v_total;
    publish(s, o, n);
    return ACCORD_OK;
}

struct StabOwner {
    std::vector<uint32_t> off, v;
};

int32_t accord_deps_range_stab(accord_store *s, const accord_deps *src, const uint32_t *q_off, const uint32_t *q_start,
                               const uint32_t *q_end, accord_range_stab *out)
{
    RC(check_views(s, 1, src));
    if (!out || !q_off) return fail(s, ACCORD_ERR_ARG, "accord_deps_range_stab: null argument");
    if (!src->rd_rng_off || !src->rd_val_off || !src->rd_r2v_off)
        return fail(s, ACCORD_ERR_ARG, "accord_deps_range_stab: deps view without RangeDeps offsets");
    const uint32_t n = src->n;
    if (q_off[0] != 0) return fail(s, ACCORD_ERR_ARG, "query offsets must start at 0");
    for (uint32_t i = 0; i < n; ++i)
        if (q_off[i + 1] < q_off[i]) return fail(s, ACCORD_ERR_ARG, "query offsets decrease at txn %u", i);
    const uint32_t nq = q_off[n];
    if (nq && (!q_start || !q_end)) return fail(s, ACCORD_ERR_ARG, "queries without bounds");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    StabOwner *own = new (std::nothrow) StabOwner();
    if (!own) return fail(s, ACCORD_ERR_OOM, "out of host memory");
    struct Guard { StabOwner *&o; ~Guard() { delete o; } } guard{own};
    op_begin(s);
    hipStream_t st = s->stream;
    DevBuf *T = s->op_tmp;
    const size_t n1 = (size_t)n + 1, q1 = (size_t)nq + 1;
    HIPCHECK(s, T[T_VLEN].ensure(n1 * 4)); HIPCHECK(s, T[T_KLEN].ensure(q1 * 4)); HIPCHECK(s, T[T_BLEN].ensure(q1 * 4));
    HIPCHECK(s, T[T_VEOFF].ensure(q1 * 4)); HIPCHECK(s, T[T_KEOFF].ensure(n1 * 4)); HIPCHECK(s, T[T_BEOFF].ensure(n1 * 4));
    HIPCHECK(s, T[T_KLST].ensure(q1 * 4)); HIPCHECK(s, T[T_CNTV].ensure(q1 * 4));
    HIPCHECK(s, s->status_totals.ensure(sizeof(HostTotals)));
    HostTotals *dev = s->status_totals.as<HostTotals>();
    HIPCHECK(s, hipMemsetAsync(dev, 0xFF, sizeof(HostTotals), st));
    HIPCHECK(s, hipMemsetAsync(&dev->status.overflow, 0, sizeof(uint32_t), st));
    HIPCHECK(s, hipMemcpyAsync(T[T_VLEN].p, q_off, n1 * 4, hipMemcpyHostToDevice, st));
    if (nq) {
        HIPCHECK(s, hipMemcpyAsync(T[T_KLEN].p, q_start, (size_t)nq * 4, hipMemcpyHostToDevice, st));
        HIPCHECK(s, hipMemcpyAsync(T[T_BLEN].p, q_end, (size_t)nq * 4, hipMemcpyHostToDevice, st));
    }
    accord::RangeIndexParams p{};
    p.n = n;
    p.rng_off = src->rd_rng_off; p.rs = src->rd_rng_start; p.re = src->rd_rng_end;
    p.val_off = src->rd_val_off; p.vals = src->rd_vals; p.r2v_off = src->rd_r2v_off; p.r2v = src->rd_r2v;
    p.status = &dev->status;
    // 1. checkpoints per txn, their offsets
    HIPCHECK(s, hipMemsetAsync(T[T_KEOFF].p, 0, n1 * 4, st));
    p.chk_cnt = T[T_KEOFF].as<uint32_t>();
    accord::launch_ri_chk_count(p, st);
    Scans sc;
    RC(scans_init(s, sc));
    RC(sc.add(p.chk_cnt, T[T_BEOFF].as<uint32_t>(), n + 1));
    unsigned long long tot[1];
    RC(sc.read(tot));
    const uint64_t nchk = tot[0];
    if (nchk >= (1ull << 31)) return fail(s, ACCORD_ERR_CAPACITY, "range index: %llu checkpoints", (unsigned long long)nchk);
    p.chk_off = T[T_BEOFF].as<uint32_t>();
    // 2. checkpoint lists: sizes, offsets, contents
    HIPCHECK(s, T[T_VOWN].ensure((nchk + 1) * 4)); HIPCHECK(s, T[T_VLST].ensure((nchk + 1) * 4));
    HIPCHECK(s, hipMemsetAsync(T[T_VOWN].p, 0, (nchk + 1) * 4, st));
    p.list_cnt = T[T_VOWN].as<uint32_t>();
    accord::launch_ri_lists(p, (uint32_t)nchk, false, st);
    RC(sc.add(p.list_cnt, T[T_VLST].as<uint32_t>(), (uint32_t)nchk + 1));
    RC(sc.read(tot));
    const uint64_t L = tot[0];
    if (L >= (1ull << 32)) return fail(s, ACCORD_ERR_CAPACITY, "range index: %llu checkpoint entries", (unsigned long long)L);
    HIPCHECK(s, T[T_KOWN].ensure(L * 4 + 4));
    p.list_off = T[T_VLST].as<uint32_t>(); p.lists = T[T_KOWN].as<uint32_t>();
    accord::launch_ri_lists(p, (uint32_t)nchk, true, st);
    // 3. stab: per query |txnIds|, offsets, the txnIds
    accord::launch_ri_qtxn(n, T[T_VLEN].as<uint32_t>(), T[T_VEOFF].as<uint32_t>(), st);
    HIPCHECK(s, hipMemsetAsync(T[T_KLST].p, 0, q1 * 4, st));
    p.nq = nq; p.q_txn = T[T_VEOFF].as<uint32_t>(); p.q_s = T[T_KLEN].as<uint32_t>(); p.q_e = T[T_BLEN].as<uint32_t>();
    p.out_cnt = T[T_KLST].as<uint32_t>();
    accord::launch_ri_stab(p, false, st);
    RC(sc.add(p.out_cnt, T[T_CNTV].as<uint32_t>(), nq + 1));
    RC(sc.read(tot));
    const uint64_t total = tot[0];
    HIPCHECK(s, hipMemcpyAsync(s->pinned, dev, sizeof(HostTotals), hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    if (s->pinned->status.overflow)
        return fail(s, ACCORD_ERR_CAPACITY, "range stab: txn %u has more than %u RangeDeps ranges or %u txnIds",
                    s->pinned->status.overflow_first, accord::RI_MAX_RANGES, accord::RI_UMAX);
    HIPCHECK(s, T[T_CNTK].ensure(total * 4 + 4));
    p.out_off = T[T_CNTV].as<uint32_t>(); p.out = T[T_CNTK].as<uint32_t>();
    accord::launch_ri_stab(p, true, st);
    HIPCHECK(s, hipGetLastError());
    try { own->off.resize(q1); own->v.resize(total + 1); } catch (...) { return fail(s, ACCORD_ERR_OOM, "out of host memory"); }
    HIPCHECK(s, hipMemcpyAsync(own->off.data(), p.out_off, q1 * 4, hipMemcpyDeviceToHost, st));
    if (total) HIPCHECK(s, hipMemcpyAsync(own->v.data(), p.out, total * 4, hipMemcpyDeviceToHost, st));
    RC(op_end(s));
    out->nq = nq;
    out->total = total;
    out->off = own->off.data();
    out->txn = own->v.data();
    out->owner = own;
    own = nullptr;          // released by accord_range_stab_release
    return ACCORD_OK;
}

void accord_range_stab_release(accord_range_stab *r)
{
    if (!r) return;
    delete (StabOwner *)r->owner;
    std::memset(r, 0, sizeof(*r));
}

void accord_deps_inverse_release(accord_deps_inverse *inv)
{
    if (!inv) return;
    delete (InverseOwner *)inv->owner;
    std::memset(inv, 0, sizeof(*inv));
}

int32_t accord_ops_timing(accord_store *s, float *ms)
{
    if (!s || !ms) return fail(s, ACCORD_ERR_ARG, "null argument");
    *ms = s->ops_ms;
    return ACCORD_OK;
}

} // extern "C"
