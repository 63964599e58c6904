// C ABI implementation (include/accord_deps.h): one accord_store == one CommandStore == one
// HIP stream, with a grow-only HBM arena for the batch, the per-key histories and the outputs.
#include "store_impl.h"

#include <algorithm>

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace accord_impl {

thread_local std::string g_last_error;

int32_t fail(accord_store *s, int32_t code, const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (s) s->err = buf;
    g_last_error = buf;
    return code;
}

} // namespace accord_impl

namespace {

int bits_for(uint32_t maxval)
{
    int b = 0;
    while (b < 32 && (maxval >> b) != 0) ++b;
    return b < 1 ? 1 : b;
}

void record(accord_store *s, int stage)
{
    if (s->events) (void)hipEventRecord(s->ev[stage], s->stream);
}

const char *code_name(int32_t c)
{
    switch (c) {
    case ACCORD_ERR_UNSORTED: return "batch TxnIds are not strictly ascending (Timestamp.compareTo)";
    case ACCORD_ERR_KIND: return "txn kind has no witnesses() (LocalOnly or invalid ordinal)";
    case ACCORD_ERR_KEYS: return "keys not sorted unique or outside the store's key range";
    case ACCORD_ERR_DOMAIN: return "TxnId domain bit inconsistent with its keys/ranges";
    case ACCORD_ERR_RANGES: return "ranges not sorted, de-overlapped and non-empty";
    case ACCORD_ERR_ARG: return "malformed CSR offsets";
    default: return "error";
    }
}

} // namespace

extern "C" {

uint32_t accord_abi_version(void) { return ACCORD_ABI_VERSION; }

int32_t accord_store_create(const accord_store_cfg *cfg, accord_store **out)
{
    if (!cfg || !out) return fail(nullptr, ACCORD_ERR_ARG, "accord_store_create: null argument");
    *out = nullptr;
    if (cfg->key_hi <= cfg->key_lo) return fail(nullptr, ACCORD_ERR_ARG, "empty key range [%u,%u)", cfg->key_lo, cfg->key_hi);
    if (cfg->nstores) {
        const uint32_t *b = cfg->store_bounds;
        if (!b) return fail(nullptr, ACCORD_ERR_ARG, "nstores = %u without store_bounds", cfg->nstores);
        for (uint32_t j = 0; j < cfg->nstores; ++j)
            if (b[j] >= b[j + 1]) return fail(nullptr, ACCORD_ERR_ARG, "store bounds not ascending at %u", j);
        if (cfg->key_lo < b[0] || (b[cfg->nstores] != ACCORD_KEY_END && cfg->key_hi > b[cfg->nstores]))
            return fail(nullptr, ACCORD_ERR_ARG, "key range [%u,%u) outside the stores [%u,%u)", cfg->key_lo,
                        cfg->key_hi, b[0], b[cfg->nstores]);
    }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0)
        return fail(nullptr, ACCORD_ERR_HIP, "no HIP device available (%s)", hipGetErrorString(e));
    if (cfg->device < 0 || cfg->device >= ndev) return fail(nullptr, ACCORD_ERR_ARG, "bad device %d", cfg->device);
    accord_store *s = new (std::nothrow) accord_store();
    if (!s) return fail(nullptr, ACCORD_ERR_OOM, "out of host memory");
    s->cfg = *cfg;
    if (cfg->nstores) s->st_bounds.assign(cfg->store_bounds, cfg->store_bounds + cfg->nstores + 1);
    s->cfg.store_bounds = nullptr;   // borrowed for the call only
    if ((e = hipSetDevice(cfg->device)) != hipSuccess || (e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking)) != hipSuccess) {
        delete s;
        return fail(nullptr, ACCORD_ERR_HIP, "stream create: %s", hipGetErrorString(e));
    }
    if ((e = hipHostMalloc((void **)&s->pinned, sizeof(HostTotals), hipHostMallocDefault)) != hipSuccess) {
        (void)hipStreamDestroy(s->stream);
        delete s;
        return fail(nullptr, ACCORD_ERR_HIP, "pinned alloc: %s", hipGetErrorString(e));
    }
    s->events = (cfg->flags & ACCORD_STORE_PROFILE) != 0;
    s->resident = (cfg->flags & ACCORD_STORE_RESIDENT) != 0;
    if (s->events)
        for (auto &ev : s->ev) (void)hipEventCreate(&ev);
    s->ev_created = s->events;
    const uint64_t span_need = (uint64_t)cfg->window + 2048;
    s->wpl = span_need <= 4096 ? 1 : span_need <= 8192 ? 2 : 4;
    *out = s;
    return ACCORD_OK;
}

int32_t accord_store_destroy(accord_store *s)
{
    if (!s) return ACCORD_OK;
    (void)hipSetDevice(s->cfg.device);
    (void)hipStreamSynchronize(s->stream);
    DevBuf *bufs[] = {&s->msb, &s->lsb, &s->node, &s->key_off, &s->key_ord, &s->rng_off, &s->rng_start, &s->rng_end,
                      &s->pair_key, &s->pair_ent, &s->sort_key, &s->sort_pair, &s->tmp_key, &s->tmp_val, &s->tmp_ent, &s->hist, &s->slice, &s->hist_tmp, &s->cnt_vub, &s->vub_off, &s->vgap, &s->fk_recs, &s->fk_list, &s->cv_tmp, &s->fk_ubits, &s->fk_umode,
                      &s->seg_start, &s->seg_end, &s->mc_state, &s->mc_state2, &s->mc_out, &s->mc_cnt, &s->mc_po, &s->radix_tmp, &s->cnt_keys, &s->cnt_vals, &s->cnt_k2v,
                      &s->kd_key_off, &s->kd_val_off, &s->kd_k2v_off, &s->scan_tmp, &s->status_totals,
                      &s->kd_keys, &s->kd_vals, &s->kd_k2v, &s->rd_zero_off,
                      &s->rng_owner, &s->is_range, &s->rt_excl, &s->range_txns, &s->cnt_rngs, &s->cnt_rvals,
                      &s->cnt_r2v, &s->rd_rng_off, &s->rd_val_off, &s->rd_r2v_off, &s->rd_rng_start, &s->rd_rng_end,
                      &s->rd_vals, &s->rd_r2v, &s->rd_big, &s->rt_hits, &s->rk_cp, &s->rk_cnt, &s->rk_off, &s->rk_slices, &s->rk_cls, &s->txn_index, &s->m_key_off, &s->m_val_off, &s->m_k2v_off,
                      &s->m_keys, &s->m_vals, &s->m_k2v, &s->m_cnt_keys, &s->m_cnt_vals, &s->m_cnt_k2v, &s->m_ptrs,
                      &s->m_zero, &s->wo_cnt, &s->wo_off, &s->wo_words, &s->wo_aoi, &s->pred_cnt, &s->pred_off, &s->preds,
                      &s->level, &s->wo_info, &s->lv_tmp, &s->pred_own, &s->cy_key, &s->cy_ent, &s->cy_key2, &s->cy_ent2,
                      &s->carry_tmp, &s->rg_tmsb, &s->rg_tlsb, &s->rg_tnode, &s->rg_tg, &s->rg_status, &s->rg_emsb,
                      &s->rg_elsb, &s->rg_enode, &s->rg_flag, &s->rg_gcnt, &s->rg_goff, &s->rg_hist2, &s->rg_kbound, &s->rg_cwflag, &s->rg_cwoff, &s->rg_cwpos, &s->rg_cwpm, &s->rg_cwchunk, &s->rg_hxchunk, &s->rg_hx, &s->rg_hu,
                      &s->rc_owner, &s->rc_start, &s->rc_end, &s->rc_kind, &s->rc_owner2, &s->rc_start2,
                      &s->rc_end2, &s->rc_kind2, &s->rc_first, &s->rc_flag, &s->rc_offs, &s->rdy_kseg0, &s->rdy_kseg1, &s->rdy_dirty, &s->rdy_dirty2, &s->rg_cchg, &s->rdy_dlist, &s->rdy_work, &s->rdy_wcnt, &s->rg_chg, &s->rdy_part, &s->rdy_sum, &s->rdy_out, &s->rdy_kb, &s->rdy_launch,
                      &s->bk_list, &s->bk_wex, &s->rb_start, &s->rb_end, &s->rb_bound, &s->rb_sep, &s->rb_eep, &s->rb_cnt, &s->rb_zero,
                      &s->rb_local, &s->rb_boot, &s->rb_stale, &s->wo_eal, &s->wo_err, &s->rr_ovf, &s->rr_spill, &s->rdy_spill, &s->rdy_spill_mem, &s->up_stage};
    accord_impl::shard_comm_destroy(s);
    accord_impl::segment_destroy(s);
    accord_impl::ready_destroy(s);
    accord_impl::pinned_arena_destroy(s);
    for (DevBuf *b : bufs) b->release();
    for (DepSet &d : s->ds) d.release();
    s->rb_set.release();
    for (DevBuf &b : s->op_tmp) b.release();
    if (s->ev_created)
        for (auto &ev : s->ev) (void)hipEventDestroy(ev);
    if (s->pinned) (void)hipHostFree(s->pinned);
    if (s->reg_host) (void)hipHostFree(s->reg_host);
    if (s->rb_host) (void)hipHostFree(s->rb_host);
    s->rb_pack.release();
    if (s->up_host) (void)hipHostFree(s->up_host);
    for (hipEvent_t &e : s->up_ev)
        if (e) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(s->stream);
    delete s;
    return ACCORD_OK;
}

const char *accord_last_error(const accord_store *s)
{
    return s ? s->err.c_str() : accord_impl::g_last_error.c_str();
}

void *accord_store_stream(accord_store *s) { return s ? (void *)s->stream : nullptr; }

int32_t accord_batch_upload(accord_store *s, const accord_batch *b)
{
    if (!s || !b || !b->msb || !b->lsb || !b->node || !b->key_off || (!b->key_ord && b->n))
        return fail(s, ACCORD_ERR_ARG, "accord_batch_upload: null argument");
    if (b->n >= (1u << 29)) return fail(s, ACCORD_ERR_CAPACITY, "batch of %u txns exceeds 2^29", b->n);
    if (b->key_off[b->n] >= (1u << 28)) return fail(s, ACCORD_ERR_CAPACITY, "batch of %u (txn, key) pairs exceeds 2^28", b->key_off[b->n]);
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    const uint32_t n = b->n;
    for (uint32_t i = 0; i < n; ++i)   // CSR sanity before anything indexes with it
        if (b->key_off[i + 1] < b->key_off[i] || (b->rng_off && b->rng_off[i + 1] < b->rng_off[i]))
            return fail(s, ACCORD_ERR_ARG, "CSR offsets decrease at txn %u", i);
    if (b->key_off[0] != 0 || (b->rng_off && b->rng_off[0] != 0))
        return fail(s, ACCORD_ERR_ARG, "CSR offsets must start at 0");
    const uint32_t P = b->key_off[n];
    const uint32_t *ro = b->rng_off, *rs = b->rng_start, *re = b->rng_end;
    uint32_t R = ro ? ro[n] : 0;
    if (R && (!rs || !re)) return fail(s, ACCORD_ERR_ARG, "range CSR without range bounds");
    if (R && !s->st_bounds.empty()) {
        // slice every range Minimal to the handle's CommandStores (include/accord_deps.h
        // accord_store_cfg.store_bounds; AbstractRanges.sliceMinimal, primitives/AbstractRanges.java:
        // 339-377): the ranges are checked first, so a slice never hides a bad payload
        for (uint32_t i = 0; i < n; ++i)
            for (uint32_t r = ro[i]; r < ro[i + 1]; ++r)
                if (rs[r] >= re[r] || (r > ro[i] && re[r - 1] > rs[r]))
                    return fail(s, ACCORD_ERR_RANGES, "txn %u: %s", i, code_name(ACCORD_ERR_RANGES));
        const std::vector<uint32_t> &B = s->st_bounds;
        const uint32_t S = (uint32_t)B.size() - 1;
        s->sl_off.resize((size_t)n + 1);
        s->sl_start.clear(); s->sl_end.clear();
        s->sl_off[0] = 0;
        for (uint32_t i = 0; i < n; ++i) {
            for (uint32_t r = ro[i]; r < ro[i + 1]; ++r) {
                const int64_t a = rs[r], z = re[r];
                // first store whose upper end (B[j+1] - 1, open at ACCORD_KEY_END) lies above a
                uint32_t j = (uint32_t)(std::upper_bound(B.begin() + 1, B.end() - 1, (uint32_t)std::min<int64_t>(a + 1, UINT32_MAX)) - B.begin()) - 1;
                for (; j < S; ++j) {
                    const int64_t lo = (int64_t)B[j] - 1;
                    const int64_t hi = B[j + 1] == ACCORD_KEY_END ? INT64_MAX : (int64_t)B[j + 1] - 1;
                    if (lo >= z) break;
                    if (!(a < hi && lo < z)) continue;
                    s->sl_start.push_back((uint32_t)std::max(a, lo));
                    s->sl_end.push_back((uint32_t)std::min(z, hi));
                }
            }
            s->sl_off[i + 1] = (uint32_t)s->sl_start.size();
        }
        ro = s->sl_off.data(); rs = s->sl_start.data(); re = s->sl_end.data();
        R = ro[n];
    }
    uint32_t nrt = 0, kinds = 0;
    for (uint32_t i = 0; i < n; ++i) {
        nrt += (uint32_t)(b->lsb[i] & 1);
        if (b->key_off[i + 1] > b->key_off[i]) kinds |= 1u << ((b->lsb[i] >> 1) & 7);   // history entry kinds
    }
    if (b->txn_index && nrt)
        return fail(s, ACCORD_ERR_ARG, "txn_index (store subset of a stream) is supported for key txns only");
    s->n = n; s->P = P; s->R = R; s->n_range_txns = nrt; s->b_kinds = kinds;
    s->rk_keys_total = 0;                // sizes the range txns' stored key slices
    if (nrt && ro)
        for (uint32_t i = 0; i < n; ++i)
            if (b->lsb[i] & 1)
                for (uint32_t r = ro[i]; r < ro[i + 1]; ++r) {
                    const uint64_t ks = std::max<uint64_t>((uint64_t)rs[r] + 1, s->cfg.key_lo);
                    const uint64_t ke = std::min<uint64_t>(re[r], (uint64_t)s->cfg.key_hi - 1);
                    if (ks <= ke) s->rk_keys_total += ke - ks + 1;
                }
    if (s->rk_keys_total >= (1ull << 32))
        return fail(s, ACCORD_ERR_CAPACITY, "range txns cover %llu (txn, key) pairs, over 2^32",
                    (unsigned long long)s->rk_keys_total);
    s->has_batch = false; s->computed = false; s->merged = false; s->m_pending = false; s->ds_cur = -1; s->mc_next = 0;
    s->b_registered = false;
    s->rdy_batch_gen = nullptr;
    HIPCHECK(s, s->msb.ensure((size_t)n * 8));
    HIPCHECK(s, s->lsb.ensure((size_t)n * 8));
    HIPCHECK(s, s->node.ensure((size_t)n * 4));
    HIPCHECK(s, s->key_off.ensure(((size_t)n + 1) * 4));
    HIPCHECK(s, s->key_ord.ensure((size_t)P * 4));
    HIPCHECK(s, s->rng_off.ensure(((size_t)n + 1) * 4));
    HIPCHECK(s, s->rng_start.ensure((size_t)R * 4));
    HIPCHECK(s, s->rng_end.ensure((size_t)R * 4));
    if ((b->exec_msb != nullptr) != (b->exec_lsb != nullptr) || (b->exec_msb != nullptr) != (b->exec_node != nullptr))
        return fail(s, ACCORD_ERR_ARG, "executeAt needs all of exec_msb, exec_lsb, exec_node");
    // the batch's arrays: a small batch (a resident / registered store's) packed into pinned staging,
    // one host-to-device copy and one device scatter; a large one copied array by array
    struct Part { void *dst; const void *src; size_t bytes; };
    std::vector<Part> parts;
    parts.push_back({s->msb.p, b->msb, (size_t)n * 8});
    parts.push_back({s->lsb.p, b->lsb, (size_t)n * 8});
    parts.push_back({s->node.p, b->node, (size_t)n * 4});
    parts.push_back({s->key_off.p, b->key_off, ((size_t)n + 1) * 4});
    parts.push_back({s->key_ord.p, b->key_ord, (size_t)P * 4});
    if (ro) parts.push_back({s->rng_off.p, ro, ((size_t)n + 1) * 4});
    parts.push_back({s->rng_start.p, rs, (size_t)R * 4});
    parts.push_back({s->rng_end.p, re, (size_t)R * 4});
    if (b->txn_index || s->resident) HIPCHECK(s, s->txn_index.ensure((size_t)n * 4 + 4));
    if (b->txn_index) parts.push_back({s->txn_index.p, b->txn_index, (size_t)n * 4});
    if (b->exec_msb) {
        HIPCHECK(s, s->exec_msb.ensure((size_t)n * 8));
        HIPCHECK(s, s->exec_lsb.ensure((size_t)n * 8));
        HIPCHECK(s, s->exec_node.ensure((size_t)n * 4));
        parts.push_back({s->exec_msb.p, b->exec_msb, (size_t)n * 8});
        parts.push_back({s->exec_lsb.p, b->exec_lsb, (size_t)n * 8});
        parts.push_back({s->exec_node.p, b->exec_node, (size_t)n * 4});
    }
    s->user_txn_index = b->txn_index != nullptr;
    s->has_txn_index = s->user_txn_index || s->resident;
    const bool gen_index = s->has_txn_index && !s->user_txn_index;     // resident: next_global + t
    size_t packed = 0;
    for (const Part &q : parts) packed += (q.bytes + 15) & ~(size_t)15;
    // zero range offsets and a resident store's stream positions ride in the pack (src nullptr: zeros)
    const size_t extra = (!ro ? ((((size_t)n + 1) * 4 + 15) & ~(size_t)15) : 0) + (gen_index ? (((size_t)n * 4 + 15) & ~(size_t)15) : 0);
    bool synced_copy = true;
    if (packed + extra <= (8u << 20)) {
        if (!ro) parts.push_back({s->rng_off.p, nullptr, ((size_t)n + 1) * 4});
        if (gen_index) parts.push_back({s->txn_index.p, nullptr, (size_t)n * 4});
        packed += extra;
        // two halves of pinned staging used in turn: an upload waits only for the copy two uploads
        // back (an event), not for its own (the compute is ordered after it on the stream)
        const size_t half = std::max<size_t>(packed, 1u << 16);
        if (s->up_host_cap < 2 * half) {
            HIPCHECK(s, hipStreamSynchronize(s->stream));       // no copy still reads the old staging
            if (s->up_host) (void)hipHostFree(s->up_host);
            s->up_host = nullptr; s->up_host_cap = 0;
            HIPCHECK(s, hipHostMalloc(&s->up_host, 4 * half, hipHostMallocDefault));
            s->up_host_cap = 4 * half;
            s->up_ev_live[0] = s->up_ev_live[1] = false;
        }
        const uint32_t hb = s->up_half;
        s->up_half ^= 1u;
        if (s->up_ev_live[hb]) HIPCHECK(s, hipEventSynchronize(s->up_ev[hb]));
        s->up_ev_live[hb] = false;
        char *hp = (char *)s->up_host + hb * (s->up_host_cap / 2);
        HIPCHECK(s, s->up_stage.ensure(packed + 16));
        accord::CopyList cl;
        size_t off = 0;
        for (const Part &q : parts) {
            if (q.bytes) {
                if (q.src) std::memcpy(hp + off, q.src, q.bytes);
                else if (q.dst == s->txn_index.p && gen_index) {
                    uint32_t *ti = (uint32_t *)(hp + off);
                    for (uint32_t t = 0; t < n; ++t) ti[t] = s->next_global + t;
                } else std::memset(hp + off, 0, q.bytes);
                cl.add((const char *)s->up_stage.p + off, q.dst, q.bytes);
            }
            off += (q.bytes + 15) & ~(size_t)15;
        }
        if (packed) {
            HIPCHECK(s, hipMemcpyAsync(s->up_stage.p, hp, packed, hipMemcpyHostToDevice, s->stream));
            if (!s->up_ev[hb]) HIPCHECK(s, hipEventCreateWithFlags(&s->up_ev[hb], hipEventDisableTiming));
            HIPCHECK(s, hipEventRecord(s->up_ev[hb], s->stream));
            s->up_ev_live[hb] = true;
            synced_copy = false;
        }
        accord::launch_copy_words(cl, s->stream);
    } else {
        if (!ro) HIPCHECK(s, hipMemsetAsync(s->rng_off.p, 0, ((size_t)n + 1) * 4, s->stream));
        for (const Part &q : parts)
            if (q.bytes) HIPCHECK(s, hipMemcpyAsync(q.dst, q.src, q.bytes, hipMemcpyHostToDevice, s->stream));
        if (gen_index) accord::launch_gen_index(n, s->next_global, s->txn_index.as<uint32_t>(), s->stream);
    }
    // where the batch ends in the stream (committed to the store when its compute succeeds)
    s->b_end = !s->resident ? n : (n == 0 ? s->next_global : (s->user_txn_index ? b->txn_index[n - 1] + 1u : s->next_global + n));
    if (s->resident && n && (uint64_t)s->next_global + n > (1ull << 29))
        return fail(s, ACCORD_ERR_CAPACITY, "resident store stream exceeds 2^29 txns");
    if (n) { s->b_last_msb = b->msb[n - 1]; s->b_last_lsb = b->lsb[n - 1]; s->b_last_node = b->node[n - 1]; }
    s->has_exec = b->exec_msb != nullptr;
    // the large path copied from the caller's pageable arrays: wait for it; the packed path's host
    // inputs were consumed into the staging above
    if (synced_copy) HIPCHECK(s, hipStreamSynchronize(s->stream));
    else HIPCHECK(s, hipGetLastError());
    s->has_batch = true;
    return ACCORD_OK;
}

int32_t accord_deps_compute(accord_store *s)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (!s->has_batch) return fail(s, ACCORD_ERR_STATE, "accord_deps_compute before accord_batch_upload");
    if (s->b_registered) return fail(s, ACCORD_ERR_STATE, "the uploaded batch is already part of the resident store's stream");
    if (s->seg_active && !s->seg_carry_ok)
        return fail(s, ACCORD_ERR_STATE, "a stream segment computes after accord_segment_carry (its CommandsForKey state)");
    // a stream segment's store ends with its segment: no carry is kept for a next batch (the later
    // segments build theirs from its summary, segment.hip)
    const bool keep_carry = s->resident && !s->seg_active;
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    const uint32_t n = s->n, P = s->P, R = s->R, nrt = s->n_range_txns;
    const uint32_t nkeys = s->cfg.key_hi - s->cfg.key_lo;
    const size_t n1 = (size_t)n + 1;
    hipStream_t st = s->stream;
    s->computed = false;
    s->kd_dense = false;
    s->merged = false;
    s->m_pending = false;
    s->ds_cur = -1;
    s->wo_done = false;
    s->rdy_batch_gen = nullptr;

    // history = [entries a resident store carried over | this batch's pairs], key-major after the sort
    const uint32_t C = s->resident ? s->carry_n : 0u;
    const uint32_t PH = C + P;
    if ((uint64_t)C + P >= (1ull << 28)) return fail(s, ACCORD_ERR_CAPACITY, "history of %u + %u entries exceeds 2^28", C, P);
    HIPCHECK(s, s->pair_key.ensure((size_t)PH * 4));
    HIPCHECK(s, s->pair_ent.ensure((size_t)PH * 4));
    HIPCHECK(s, s->sort_key.ensure((size_t)PH * 4));
    HIPCHECK(s, s->sort_pair.ensure((size_t)PH * 4));
    HIPCHECK(s, s->tmp_key.ensure((size_t)PH * 4));
    HIPCHECK(s, s->tmp_val.ensure((size_t)PH * 4));
    HIPCHECK(s, s->tmp_ent.ensure((size_t)PH * 4));
    HIPCHECK(s, s->hist.ensure((size_t)PH * 4));
    HIPCHECK(s, s->slice.ensure((size_t)P * sizeof(accord::PairSlice)));
    HIPCHECK(s, s->cnt_vub.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->vub_off.ensure(n1 * 4));
    HIPCHECK(s, s->hist_tmp.ensure(accord::history_temp_bytes(PH)));
    HIPCHECK(s, s->seg_start.ensure((size_t)nkeys * 4));
    HIPCHECK(s, s->seg_end.ensure((size_t)nkeys * 4));
    HIPCHECK(s, s->radix_tmp.ensure(accord::radix_sort_temp_bytes(PH)));
    if (keep_carry) {
        HIPCHECK(s, s->cy_key2.ensure((size_t)PH * 4 + 4));
        HIPCHECK(s, s->cy_ent2.ensure((size_t)PH * 4 + 4));
        HIPCHECK(s, s->carry_tmp.ensure(accord::carry_temp_bytes(PH, nkeys)));
    }
    HIPCHECK(s, s->cnt_keys.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->cnt_vals.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->cnt_k2v.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->cnt_rngs.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->cnt_rvals.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->cnt_r2v.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->kd_key_off.ensure(n1 * 4));
    HIPCHECK(s, s->kd_k2v_off.ensure(n1 * 4));
    HIPCHECK(s, s->rd_rng_off.ensure(n1 * 4));
    HIPCHECK(s, s->rd_val_off.ensure(n1 * 4));
    HIPCHECK(s, s->rd_r2v_off.ensure(n1 * 4));
    // the store's scan state, shared by every scan of the pipeline (radix digit offsets, CSR offsets,
    // carry compaction): sized for the longest
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(
                    accord::scan_temp_bytes(std::max({n, PH, accord::radix_sort_scan_len(PH), (s->resident ? s->rc_n : 0u) + R})),
                    s->stream));
    // the scan state's 30-bit epochs advance once per scan (a few dozen per compute): re-zeroed long
    // before they could wrap onto a status word still in the buffer
    if (++s->computes_since_zero >= (1u << 22)) {
        HIPCHECK(s, hipMemsetAsync(s->scan_tmp.p, 0, s->scan_tmp.cap, st));
        s->computes_since_zero = 0;
    }
    HIPCHECK(s, s->status_totals.ensure(sizeof(HostTotals)));
    HIPCHECK(s, s->rng_owner.ensure((size_t)R * 4));
    HIPCHECK(s, s->is_range.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->rt_excl.ensure(n1 * 4));
    HIPCHECK(s, s->range_txns.ensure((size_t)nrt * 4 + 4));
    if (nrt) HIPCHECK(s, s->rk_cls.ensure(accord::rangekeys_class_bytes(nrt)));

    HIPCHECK(s, s->fk_list.ensure((size_t)n * 4 + 64));
    HIPCHECK(s, s->bk_list.ensure((size_t)n * 4 + 64));
    HIPCHECK(s, s->bk_wex.ensure((size_t)P * 4 + 4));
    // RangeDeps for the batch: its own range commands and, in a resident store, the carried ones
    const uint32_t ncr = s->resident ? s->rc_n : 0u;
    const bool rdeps = R || ncr;
    if (rdeps) HIPCHECK(s, s->rd_big.ensure(((size_t)2 * n + 64) * 4));   // big list | tile fallback list
    if (rdeps) HIPCHECK(s, s->rt_hits.ensure((size_t)n * (1 + accord::RT_HIT_WORDS) * 4 + 64));

    HostTotals *dev = s->status_totals.as<HostTotals>();
    // a resident store's batch of up to 16 Ki pairs is sorted alone (one workgroup) and merged into
    // its key-major carry (accord::merge_join_batch) instead of re-sorting [carry | batch]
    const int kbits = bits_for(nkeys - 1);
    // (a stream segment's carry is in stream order, not key-major: it always takes the sort)
    const bool merge = C && !s->seg_active && accord::merge_join_fits(P, kbits);
    record(s, EV_START);
    {   // every small initialisation of the pipeline in one launch
        accord::FillList fl;
        fl.add(&dev->status.first, sizeof(dev->status.first), 0xFFFFFFFFu);
        fl.add(&dev->status.overflow, 4, 0u);
        fl.add(&dev->status.overflow_first, 4, 0xFFFFFFFFu);
        fl.add(s->seg_start.p, (size_t)nkeys * 4, 0u);
        fl.add(s->seg_end.p, (size_t)nkeys * 4, 0u);
        fl.add(s->fk_list.p, 4, 0u);                                   // fallback list count
        fl.add(s->bk_list.p, 4, 0u);                                   // big-txn list count
        if (nrt) fl.add(s->rk_cls.p, 8 * 4, 0u);                        // union class list counts
        if (rdeps) {
            fl.add(s->rd_big.p, 4, 0u);                                 // big range-hit list count
            fl.add(s->rd_big.as<uint32_t>() + 32 + n, 4, 0u);           // tile fallback list count
        } else {
            fl.add(s->rd_rng_off.p, n1 * 4, 0u);
            fl.add(s->rd_val_off.p, n1 * 4, 0u);
            fl.add(s->rd_r2v_off.p, n1 * 4, 0u);
            fl.add(&dev->totals[3], 3 * sizeof(unsigned long long), 0u);
        }
        // the registered store's key flags and the RedundantBefore status, zeroed here rather than by
        // launches of their own (status_general_count, redundant_count)
        s->rg_flag_zeroed = s->rb_status_zeroed = false;
        if (accord_impl::registered_mode(s) && C && s->next_global) {
            HIPCHECK(s, s->rg_flag.ensure((size_t)nkeys * 4 + 4));
            fl.add(s->rg_flag.p, (size_t)nkeys * 4, 0u);
            s->rg_flag_zeroed = true;
        }
        if (s->rb_m) {
            fl.add(&dev->rb_status.first, sizeof(dev->rb_status.first), 0xFFFFFFFFu);
            fl.add(&dev->rb_status.overflow, 4, 0u);
            fl.add(&dev->rb_status.overflow_first, 4, 0xFFFFFFFFu);
            s->rb_status_zeroed = true;
        }
        accord::CopyList cl;          // a resident store's carried history heads the pairs
        if (C && !merge) {
            cl.add(s->cy_key.p, s->pair_key.p, (size_t)C * 4);
            cl.add(s->cy_ent.p, s->pair_ent.p, (size_t)C * 4);
        }
        accord::launch_init_words(fl, cl, st);
    }
    accord::StreamPos sp{};
    sp.min_gi = s->resident ? s->next_global : 0u;
    sp.has_prev = (s->resident && s->has_prev) ? 1u : 0u;
    sp.prev_msb = s->prev_msb; sp.prev_lsb = s->prev_lsb; sp.prev_node = s->prev_node;
    accord::launch_validate_pack(n, s->msb.as<uint64_t>(), s->lsb.as<uint64_t>(), s->node.as<int32_t>(),
                                 s->key_off.as<uint32_t>(), s->key_ord.as<uint32_t>(), s->rng_off.as<uint32_t>(),
                                 R ? s->rng_start.as<uint32_t>() : nullptr, R ? s->rng_end.as<uint32_t>() : nullptr,
                                 s->cfg.key_lo, s->cfg.key_hi, s->pair_key.as<uint32_t>() + C, s->pair_ent.as<uint32_t>() + C,
                                 R ? s->rng_owner.as<uint32_t>() : nullptr, s->is_range.as<uint32_t>(),
                                 s->has_txn_index ? s->txn_index.as<uint32_t>() : nullptr, sp, &dev->status, st);
    if (nrt) {
        accord::exclusive_scan_u32(s->is_range.as<uint32_t>(), s->rt_excl.as<uint32_t>(), n, &dev->totals[6],
                                   s->scan_tmp.p, st);
        accord::launch_compact_flags(n, s->is_range.as<uint32_t>(), s->rt_excl.as<uint32_t>(),
                                     s->range_txns.as<uint32_t>(), st);
    }
    const uint32_t *bound_l = nullptr, *bound_g = nullptr, *pair_bound = nullptr;
    if (s->has_exec) {
        HIPCHECK(s, s->bound_l.ensure((size_t)n * 4 + 4));
        HIPCHECK(s, s->bound_g.ensure((size_t)n * 4 + 4));
        HIPCHECK(s, s->pair_bound.ensure((size_t)P * 4 + 4));
        accord::launch_accept_bounds(n, s->msb.as<uint64_t>(), s->lsb.as<uint64_t>(), s->node.as<int32_t>(),
                                     s->exec_msb.as<uint64_t>(), s->exec_lsb.as<uint64_t>(), s->exec_node.as<int32_t>(),
                                     s->key_off.as<uint32_t>(), s->has_txn_index ? s->txn_index.as<uint32_t>() : nullptr,
                                     s->bound_l.as<uint32_t>(), s->bound_g.as<uint32_t>(), s->pair_bound.as<uint32_t>(),
                                     &dev->status, st);
        bound_l = s->bound_l.as<uint32_t>(); bound_g = s->bound_g.as<uint32_t>(); pair_bound = s->pair_bound.as<uint32_t>();
    }
    record(s, EV_VALIDATE);
    if (merge)
        accord::merge_join_batch(s->cy_key.as<uint32_t>(), s->cy_ent.as<uint32_t>(), C, s->pair_key.as<uint32_t>() + C,
                                 s->pair_ent.as<uint32_t>() + C, P, kbits, s->tmp_key.as<uint32_t>(),
                                 s->tmp_val.as<uint32_t>(), s->sort_key.as<uint32_t>(), s->sort_pair.as<uint32_t>(), s->hist.as<uint32_t>(), st);
    else
        accord::radix_sort_pairs(s->pair_key.as<uint32_t>(), nullptr, s->sort_key.as<uint32_t>(),
                                 s->sort_pair.as<uint32_t>(), s->tmp_key.as<uint32_t>(), s->tmp_val.as<uint32_t>(),
                                 s->pair_ent.as<uint32_t>(), s->hist.as<uint32_t>(), s->tmp_ent.as<uint32_t>(), PH,
                                 kbits, s->radix_tmp.p, s->scan_tmp.p, st);
    record(s, EV_SORT);
    accord::launch_history(PH, nkeys, s->cfg.window, s->sort_key.as<uint32_t>(), s->sort_pair.as<uint32_t>(),
                           s->hist.as<uint32_t>(), s->seg_start.as<uint32_t>(),
                           s->seg_end.as<uint32_t>(), s->slice.as<accord::PairSlice>(),
                           s->hist_tmp.p, pair_bound, C, st);
    record(s, EV_SEGMENT);

    accord::KeyDepsParams kp{};
    kp.n = n; kp.P = P;
    kp.msb = s->msb.as<uint64_t>(); kp.lsb = s->lsb.as<uint64_t>(); kp.node = s->node.as<int32_t>();
    kp.key_off = s->key_off.as<uint32_t>(); kp.key_ord = s->key_ord.as<uint32_t>();
    kp.txn_index = s->has_txn_index ? s->txn_index.as<uint32_t>() : nullptr;
    kp.key_lo = s->cfg.key_lo; kp.key_hi = s->cfg.key_hi; kp.window = s->cfg.window;
    kp.hist = s->hist.as<uint32_t>();
    bool general = false;                    // pairs on keys with registered statuses: general filter
    if (accord_impl::registered_mode(s)) {   // (its emitted entries are sized with the outputs below)
        int32_t rc = accord_impl::status_general_count(s, C, PH, &general);
        if (rc) return rc;
    }
    kp.slice = s->slice.as<accord::PairSlice>();
    kp.cnt_vub = s->cnt_vub.as<uint32_t>();
    kp.cnt_vals = s->cnt_vals.as<uint32_t>();
    kp.status = &dev->status;
    kp.bound_g = bound_g;

    accord::RangeDepsParams rp{};
    rp.bound_l = bound_l;
    rp.n = n; rp.lsb = kp.lsb; rp.key_off = kp.key_off; rp.key_ord = kp.key_ord;
    rp.rng_off = s->rng_off.as<uint32_t>(); rp.rng_start = s->rng_start.as<uint32_t>();
    rp.rng_end = s->rng_end.as<uint32_t>(); rp.rng_owner = s->rng_owner.as<uint32_t>();
    rp.window = s->cfg.window; rp.key_lo = s->cfg.key_lo; rp.key_hi = s->cfg.key_hi;
    rp.hist = kp.hist; rp.seg_start = s->seg_start.as<uint32_t>(); rp.seg_end = s->seg_end.as<uint32_t>();
    {
        const accord::HistoryViews hv = accord::history_views(s->hist_tmp.p, PH);
        rp.pw_local = hv.pw_local; rp.pw_carry = hv.pw_carry; rp.pw_tile = accord::HISTORY_TILE;
        rp.c_local = hv.c_local; rp.ccarry = hv.ccarry;
    }
    rp.nkeys = nkeys;
    rp.kinds_present = (s->resident ? s->hist_kinds : 0u) | s->b_kinds;
    // resident stores: txn i is stream position g0 + i; the checkpoint blocks span every window
    rp.g0 = s->resident ? s->next_global : 0u;
    rp.ncr = ncr;
    rp.rc_owner = s->rc_owner.as<uint32_t>(); rp.rc_start = s->rc_start.as<uint32_t>();
    rp.rc_end = s->rc_end.as<uint32_t>(); rp.rc_kind = s->rc_kind.as<uint32_t>();
    rp.cp_base = (rp.g0 > s->cfg.window ? rp.g0 - s->cfg.window : 0u) >> accord::RK_CP_SHIFT;
    rp.ncp = n ? ((rp.g0 + n - 1) >> accord::RK_CP_SHIFT) - rp.cp_base + 1 : 1;
    rp.cnt_vals_exact = s->cnt_vals.as<uint32_t>();
    const bool reg_ranges = nrt && accord_impl::registered_mode(s);   // no window: the general range-key pass
    if (nrt && !reg_ranges) {
        HIPCHECK(s, s->rk_cp.ensure(accord::rangekeys_cp_bytes(rp.ncp, nkeys)));
        HIPCHECK(s, s->rk_cnt.ensure((size_t)nrt * 4 + 4));
        HIPCHECK(s, s->rk_off.ensure(((size_t)nrt + 1) * 4));
        HIPCHECK(s, s->rk_slices.ensure(s->rk_keys_total * 8 + 8));
        rp.cp = s->rk_cp.as<uint2>();
        rp.rk_off = s->rk_off.as<uint32_t>();
        rp.rk_slices = s->rk_slices.as<uint2>();
    }
    rp.n_range_txns = nrt; rp.range_txns = s->range_txns.as<uint32_t>();
    rp.rk_cls = s->rk_cls.as<uint32_t>();
    rp.rk_bitmap = 1u;          // span-bitmap union where a body spans < 4096 txns (else the sort)
    rp.cnt_rngs = s->cnt_rngs.as<uint32_t>(); rp.cnt_vals = s->cnt_rvals.as<uint32_t>(); rp.cnt_r2v = s->cnt_r2v.as<uint32_t>();
    // range txns' KeyDeps: exact txnIds count into the upper-bound array (their bound is exact)
    rp.cnt_keys = s->cnt_keys.as<uint32_t>(); rp.cnt_vals_k = s->cnt_vub.as<uint32_t>(); rp.cnt_k2v = s->cnt_k2v.as<uint32_t>();
    rp.status = &dev->status;

    // sizes: key txns from the per-pair witnessed counts, range txns by their own count pass
    if (nrt && !reg_ranges) accord::launch_rangekeys_checkpoints(PH, s->sort_key.as<uint32_t>(), rp, st);
    record(s, EV_C_RKCP);
    if (nrt && !reg_ranges) {
        accord::launch_rangekeys_nkeys(rp, s->rk_cnt.as<uint32_t>(), st);
        accord::exclusive_scan_u32(s->rk_cnt.as<uint32_t>(), s->rk_off.as<uint32_t>(), nrt, &dev->totals[6],
                                   s->scan_tmp.p, st);
    }
    record(s, EV_C_RKN);
    accord::launch_keydeps_sizes(n, kp.key_off, kp.slice, rp.cnt_keys, s->cnt_vub.as<uint32_t>(),
                                 rp.cnt_k2v, &dev->status, st);
    record(s, EV_C_KDS);
    if (reg_ranges) {
        int32_t rc = accord_impl::status_range_keys(s, rp, false);
        if (rc) return rc;
    } else if (nrt) {
        accord::launch_rangekeys_count(rp, st);
    }
    record(s, EV_C_RK);
    if (rdeps) {
        rp.rd_big_count = s->rd_big.as<uint32_t>();
        rp.rd_big_list = rp.rd_big_count + 16;
        rp.rd_fb_count = rp.rd_big_count + 32 + n;
        // the fill pass reuses the count pass's hits (config 3 8.06 -> 7.77 ms, profiles/r04_b/
        // rangedeps_hits_ab.txt); ACCORD_RT_REUSE=0: it rescans
        const char *ru = getenv("ACCORD_RT_REUSE");
        rp.rt_h = ru && ru[0] == '0' ? nullptr : s->rt_hits.as<uint32_t>();
        rp.rt_hits = s->rt_hits.as<uint32_t>() + n;
        rp.rd_fb_list = rp.rd_fb_count + 16;
        accord::launch_rangedeps_count(rp, st);
    }
    record(s, EV_COUNT);
    // Speculative fill (key-only batches): the output arrays -- and a registered store's extended
    // history -- keep the capacity earlier batches gave them, and the fill is queued behind the sizes
    // without the host reading them first; the scan of the KeyDeps sizes checks the totals against the
    // capacities as it writes them (kernels.h SpecCheck) and sets an abort word every fill kernel
    // reads first -- only then does the host grow the arrays and fill again, after the final sync.  A
    // stream of like-sized batches never waits on the host mid-pipeline.
    const bool spec = n && !nrt && !rdeps && s->kd_keys.p && s->vgap.p && s->kd_k2v.p;
    accord::SpecCheck sc{};
    if (spec) {
        // the kernels address every output array with 32-bit byte offsets: totals past 2^30 never fit
        const uint64_t lim = (1ull << 30) - 1;
        sc.abort = &dev->spec_abort;
        sc.status = &dev->status;
        sc.cap[0] = std::min<uint64_t>(s->kd_keys.cap / 4, lim);
        sc.cap[1] = std::min<uint64_t>(s->vgap.cap / 4 - 1, lim);
        sc.cap[2] = std::min<uint64_t>(s->kd_k2v.cap / 4, lim);
        if (general) {
            HIPCHECK(s, s->rg_hist2.ensure(((size_t)PH + 1) * 4));
            sc.xtot = &dev->totals[9];
            sc.cap_x = s->rg_hist2.cap / 4 - PH;
        }
    }
    {   // KeyDeps offsets (and RangeDeps offsets) in one launch each
        const uint32_t *in[3] = {rp.cnt_keys, kp.cnt_vub, rp.cnt_k2v};
        uint32_t *out[3] = {s->kd_key_off.as<uint32_t>(), s->vub_off.as<uint32_t>(), s->kd_k2v_off.as<uint32_t>()};
        unsigned long long *tot[3] = {&dev->totals[0], &dev->totals[1], &dev->totals[2]};
        accord::exclusive_scan_multi(3, in, out, tot, n, s->scan_tmp.p, st, spec ? &sc : nullptr);
    }
    if (rdeps) {
        const uint32_t *in[3] = {rp.cnt_rngs, rp.cnt_vals, rp.cnt_r2v};
        uint32_t *out[3] = {s->rd_rng_off.as<uint32_t>(), s->rd_val_off.as<uint32_t>(), s->rd_r2v_off.as<uint32_t>()};
        unsigned long long *tot[3] = {&dev->totals[3], &dev->totals[4], &dev->totals[5]};
        accord::exclusive_scan_multi(3, in, out, tot, n, s->scan_tmp.p, st);
    }
    record(s, EV_SCAN);
    // the fast fill's per-txn records need only the offsets: built while the host reads the sizes
    HIPCHECK(s, s->fk_recs.ensure(accord::keydeps_fast_temp_bytes(n)));
    kp.kd_key_off = s->kd_key_off.as<uint32_t>(); kp.vub_off = s->vub_off.as<uint32_t>();
    kp.kd_k2v_off = s->kd_k2v_off.as<uint32_t>();
    accord::launch_keydeps_recs(kp, s->fk_recs.p, st);
    if (!spec) {
        HIPCHECK(s, hipMemcpyAsync(s->pinned, dev, sizeof(HostTotals), hipMemcpyDeviceToHost, st));
        HIPCHECK(s, hipStreamSynchronize(st));
    }

    auto check_status = [&](const HostTotals &h) -> int32_t {
        if (h.status.first != ~0ull) {
            const uint32_t where = (uint32_t)(h.status.first >> 32);
            const int32_t code = -(int32_t)(uint32_t)(h.status.first & 0xFFFFFFFFu);
            return fail(s, code, "%s (txn %u)", code_name(code), where);
        }
        if (h.status.overflow)
            return fail(s, ACCORD_ERR_CAPACITY, "%u txns exceed a per-txn capacity of this build (first: txn %u)",
                        h.status.overflow, h.status.overflow_first);
        return ACCORD_OK;
    };
    // the sizes are on the host: check them, take them, size the outputs
    auto take_sizes = [&]() -> int32_t {
        const HostTotals &h = *s->pinned;
        int32_t rc = check_status(h);
        if (rc) return rc;
        // the device kernels address every output array with 32-bit byte offsets
        for (int t = 0; t < 6; ++t)
            if (h.totals[t] >= (1ull << 30)) return fail(s, ACCORD_ERR_CAPACITY, "deps output exceeds 2^30 entries");
        s->tot_keys = h.totals[0]; s->tot_k2v = h.totals[2];
        s->tot_rngs = h.totals[3]; s->tot_rvals = h.totals[4]; s->tot_r2v = h.totals[5];
        return ACCORD_OK;
    };
    auto size_outputs = [&]() -> int32_t {
        HIPCHECK(s, s->kd_keys.ensure(s->tot_keys * 4));
        HIPCHECK(s, s->vgap.ensure(s->pinned->totals[1] * 4 + 4));   // KeyDeps txnIds, gapped (accord_deps.kd_val_cnt)
        HIPCHECK(s, s->kd_k2v.ensure(s->tot_k2v * 4));
        HIPCHECK(s, s->rd_rng_start.ensure(s->tot_rngs * 4));
        HIPCHECK(s, s->rd_rng_end.ensure(s->tot_rngs * 4));
        HIPCHECK(s, s->rd_vals.ensure(s->tot_rvals * 4));
        HIPCHECK(s, s->rd_r2v.ensure(s->tot_r2v * 4));
        kp.kd_keys = s->kd_keys.as<uint32_t>(); kp.vgap = s->vgap.as<uint32_t>(); kp.kd_k2v = s->kd_k2v.as<int32_t>();
        return ACCORD_OK;
    };
    if (!spec) {
        int32_t rc = take_sizes();
        if (rc) return rc;
    }
    if (general) {                                      // the fill reads the extended history
        const uint32_t *h = nullptr;
        int32_t rc = accord_impl::status_general_emit(s, PH, spec ? 0 : s->pinned->totals[9],
                                                      spec ? &dev->spec_abort : nullptr, &h);
        if (rc) return rc;
        kp.hist = h;
        rp.hist = h;
    }
    if (spec) {     // the arrays as they are: the check aborts the fill if they are too small
        kp.kd_keys = s->kd_keys.as<uint32_t>(); kp.vgap = s->vgap.as<uint32_t>(); kp.kd_k2v = s->kd_k2v.as<int32_t>();
        kp.abort = &dev->spec_abort;
    } else {
        int32_t rc = size_outputs();
        if (rc) return rc;
    }
    kp.kd_key_off = s->kd_key_off.as<uint32_t>(); kp.vub_off = s->vub_off.as<uint32_t>();
    kp.kd_k2v_off = s->kd_k2v_off.as<uint32_t>();
    rp.kd_key_off = kp.kd_key_off; rp.kd_val_off = kp.vub_off; rp.kd_k2v_off = kp.kd_k2v_off;
    rp.kd_keys = kp.kd_keys; rp.kd_vals = kp.vgap; rp.kd_k2v = kp.kd_k2v;
    rp.rd_rng_off = s->rd_rng_off.as<uint32_t>(); rp.rd_val_off = s->rd_val_off.as<uint32_t>();
    rp.rd_r2v_off = s->rd_r2v_off.as<uint32_t>();
    rp.rd_rng_start = s->rd_rng_start.as<uint32_t>(); rp.rd_rng_end = s->rd_rng_end.as<uint32_t>();
    rp.rd_vals = s->rd_vals.as<uint32_t>(); rp.rd_r2v = s->rd_r2v.as<int32_t>();
    kp.fb_count = s->fk_list.as<uint32_t>();
    kp.fb_list = kp.fb_count + 16;
    kp.big_count = s->bk_list.as<uint32_t>();
    kp.big_list = kp.big_count + 16;
    kp.big_wex = s->bk_wex.as<uint32_t>();
    kp.tiny = (uint64_t)P <= 2ull * n ? 1u : 0u;      // <= 2 keys per txn on average: a store's key block
    accord::launch_keydeps_fill(kp, s->wpl, s->fk_recs.p, st);
    record(s, EV_FILL);
    if (nrt) {
        if (reg_ranges) {
            int32_t rc = accord_impl::status_range_keys(s, rp, true);
            if (rc) return rc;
        } else {
            accord::launch_rangekeys_fill(rp, st);
        }
        accord::launch_rangekeys_union(rp, st);
    }
    if (rdeps) accord::launch_rangedeps_fill(rp, st);
    record(s, EV_RANGE);
    // the txnIds stay where the fill wrote them: each txn's list at its upper-bound offset (vub_off),
    // its length in cnt_vals -- the gapped form of the ABI (include/accord_deps.h, kd_val_cnt)
    if (keep_carry) {
        // what the next batch needs of this history (the stream ends at b_end)
        const uint32_t thr = s->b_end > s->cfg.window ? s->b_end - s->cfg.window : 0u;
        const bool reg = accord_impl::registered_mode(s);
        if (reg) {
            int32_t rc = accord_impl::status_prune_flags(s, PH, accord::carry_flags(s->carry_tmp.p, nkeys));
            if (rc) return rc;
        }
        accord::launch_carry(PH, nkeys, thr, s->sort_key.as<uint32_t>(), s->hist.as<uint32_t>(),
                             s->seg_start.as<uint32_t>(), s->seg_end.as<uint32_t>(),
                             accord::history_views(s->hist_tmp.p, PH), s->carry_tmp.p, s->scan_tmp.p, s->cy_key2.as<uint32_t>(),
                             s->cy_ent2.as<uint32_t>(), &dev->totals[8], reg, st);
        if (rdeps) {    // the range commands the next batch's window can still reach
            const size_t cap = (size_t)ncr + R + 1;
            HIPCHECK(s, s->rc_owner2.ensure(cap * 4)); HIPCHECK(s, s->rc_start2.ensure(cap * 4));
            HIPCHECK(s, s->rc_end2.ensure(cap * 4)); HIPCHECK(s, s->rc_kind2.ensure(cap * 4));
            HIPCHECK(s, s->rc_first.ensure(16));
            uint32_t *flags = nullptr, *offs = nullptr;
            if (reg) {    // registered-status store: erased range commands leave the carry
                HIPCHECK(s, s->rc_flag.ensure(cap * 4));
                HIPCHECK(s, s->rc_offs.ensure(cap * 4));
                flags = s->rc_flag.as<uint32_t>(); offs = s->rc_offs.as<uint32_t>();
            }
            accord::launch_range_carry(rp, R, thr, s->rc_owner2.as<uint32_t>(), s->rc_start2.as<uint32_t>(),
                                       s->rc_end2.as<uint32_t>(), s->rc_kind2.as<uint32_t>(),
                                       s->rc_first.as<uint32_t>(), &dev->totals[9], flags, offs, s->scan_tmp.p, st);
        }
    }
    record(s, EV_COMPACT);
    if (s->rb_m) {      // RedundantBefore.collectDeps' sizes travel with this copy
        int32_t rc = accord_impl::redundant_count(s);
        if (rc) return rc;
    }
    const bool join = s->resident && accord_impl::registered_mode(s);
    if (join) {         // the batch joins the store's TxnId / status tables unless the compute failed
        int32_t rc = accord_impl::status_join_queue(s, &dev->status);
        if (rc) return rc;
    }
    HIPCHECK(s, hipMemcpyAsync(s->pinned, dev, sizeof(HostTotals), hipMemcpyDeviceToHost, st));
    if (s->events)
        HIPCHECK(s, hipMemcpyAsync(&s->pinned->scan, accord::scan_counters(s->scan_tmp.p), sizeof(accord::ScanCounters),
                                   hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    HIPCHECK(s, hipGetLastError());
    if (spec) {
        int32_t rc = take_sizes();
        if (rc) return rc;
        if (s->pinned->spec_abort) {    // the outputs did not fit: grow them and fill again
            if (general) {
                const uint32_t *h = nullptr;
                rc = accord_impl::status_general_emit(s, PH, s->pinned->totals[9], nullptr, &h);
                if (rc) return rc;
                kp.hist = h;
                rp.hist = h;
            }
            rc = size_outputs();
            if (rc) return rc;
            kp.abort = nullptr;
            accord::launch_keydeps_fill(kp, s->wpl, s->fk_recs.p, st);
            record(s, EV_FILL);
            record(s, EV_RANGE);
            record(s, EV_COMPACT);
            HIPCHECK(s, hipMemcpyAsync(&s->pinned->status, &dev->status, sizeof(accord::DevStatus), hipMemcpyDeviceToHost, st));
            HIPCHECK(s, hipStreamSynchronize(st));
            HIPCHECK(s, hipGetLastError());
        }
    }
    {
        int32_t rc = check_status(*s->pinned);
        if (rc) return rc;
        s->tot_vals = s->pinned->totals[1];
    }
    if (s->resident) {      // the batch is part of the store's stream now
        if (join) accord_impl::status_join_commit(s);
        if (keep_carry) {
            std::swap(s->cy_key, s->cy_key2);
            std::swap(s->cy_ent, s->cy_ent2);
            s->carry_n = (uint32_t)s->pinned->totals[8];
        } else {
            s->seg_carry_ok = false;       // the segment's carry was consumed: a rerun takes it again
        }
        ++s->carry_version;
        s->hist_kinds |= s->b_kinds;
        if (rdeps) {
            std::swap(s->rc_owner, s->rc_owner2); std::swap(s->rc_start, s->rc_start2);
            std::swap(s->rc_end, s->rc_end2); std::swap(s->rc_kind, s->rc_kind2);
            s->rc_n = (uint32_t)s->pinned->totals[9];
        }
        s->next_global = s->b_end;
        if (n) {
            s->has_prev = true;
            s->prev_msb = s->b_last_msb; s->prev_lsb = s->b_last_lsb; s->prev_node = s->b_last_node;
        }
        s->b_registered = true;   // computing it again would register it twice
    }

    if (s->events) {
        auto el = [&](int a, int b) { float ms = 0; (void)hipEventElapsedTime(&ms, s->ev[a], s->ev[b]); return ms; };
        s->timing.validate_ms = el(EV_START, EV_VALIDATE);
        s->timing.sort_ms = el(EV_VALIDATE, EV_SORT);
        s->timing.segment_ms = el(EV_SORT, EV_SEGMENT);
        s->timing.count_ms = el(EV_SEGMENT, EV_COUNT);
        s->timing.scan_ms = el(EV_COUNT, EV_SCAN);
        s->timing.fill_ms = el(EV_SCAN, EV_FILL);
        s->timing.range_ms = el(EV_FILL, EV_RANGE);
        s->timing.compact_ms = el(EV_RANGE, EV_COMPACT);
        s->timing.total_ms = el(EV_START, EV_COMPACT);
        s->timing.count_rk_cp_ms = el(EV_SEGMENT, EV_C_RKCP);
        s->timing.count_rk_nkeys_ms = el(EV_C_RKCP, EV_C_RKN);
        s->timing.count_kd_sizes_ms = el(EV_C_RKN, EV_C_KDS);
        s->timing.count_rk_ms = el(EV_C_KDS, EV_C_RK);
        s->timing.count_rd_ms = el(EV_C_RK, EV_COUNT);
        // the store's scan counters are cumulative since the state was (re)zeroed
        const accord::ScanCounters now = s->pinned->scan;
        const bool fresh = now.spins < s->scan_seen.spins || now.fallbacks < s->scan_seen.fallbacks;
        s->timing.scan_spins = fresh ? now.spins : now.spins - s->scan_seen.spins;
        s->timing.scan_fallbacks = fresh ? now.fallbacks : now.fallbacks - s->scan_seen.fallbacks;
        s->scan_seen = now;
    }
    s->timing.pairs = P;
    s->timing.hist_entries = PH;
    s->computed = true;
    if (s->rb_m) return accord_impl::redundant_apply(s);   // builder.build().with(redundant)
    return ACCORD_OK;
}

int32_t accord_store_state(accord_store *s, accord_store_state_info *info)
{
    if (!s || !info) return fail(s, ACCORD_ERR_ARG, "null argument");
    std::memset(info, 0, sizeof(*info));
    info->next_global = s->next_global;
    info->carry_entries = s->carry_n;
    info->txns_registered = s->next_global;
    return ACCORD_OK;
}

int32_t accord_store_reset(accord_store *s)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    s->next_global = 0; s->carry_n = 0; s->rc_n = 0; s->hist_kinds = 0; s->has_prev = false;
    s->seg_active = false; s->seg_sum_ok = false; s->seg_carry_ok = false; s->seg_base = 0; s->seg_sum_n = 0;
    s->rg_tx_n = 0; s->rg_known = 0; s->rg_flag_ok = false;
    s->prev_msb = s->prev_lsb = 0; s->prev_node = 0;
    s->has_batch = false; s->b_registered = false; s->computed = false; s->merged = false; s->m_pending = false;
    s->ds_cur = -1; s->wo_done = false; s->mc_next = 0;
    // RedundantBefore.EMPTY (its bounds are positions of the old stream) and MaxConflicts.EMPTY
    s->rb_m = 0; s->rb_min_epoch = 0; s->rb_ext = false;
    ++s->carry_version;
    accord_impl::ready_destroy(s);
    s->rdy_kb_host.clear(); s->rdy_kb_dirty = false; s->rdy_kb.release();
    if (s->mc_state.p) {
        HIPCHECK(s, hipSetDevice(s->cfg.device));
        HIPCHECK(s, hipMemsetAsync(s->mc_state.p, 0, s->mc_state.cap, s->stream));
        HIPCHECK(s, hipStreamSynchronize(s->stream));
    }
    return ACCORD_OK;
}

int32_t accord_store_set_profile(accord_store *s, uint32_t on)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (on && !s->ev_created) {
        HIPCHECK(s, hipSetDevice(s->cfg.device));
        for (auto &ev : s->ev) HIPCHECK(s, hipEventCreate(&ev));
        s->ev_created = true;
    }
    s->events = on != 0;
    return ACCORD_OK;
}

int32_t accord_store_timing(accord_store *s, accord_timing *t)
{
    if (!s || !t) return fail(s, ACCORD_ERR_ARG, "null argument");
    *t = s->timing;
    return ACCORD_OK;
}

int32_t accord_deps_device_view(accord_store *s, accord_deps *d)
{
    if (!s || !d) return fail(s, ACCORD_ERR_ARG, "null argument");
    if (!s->computed) return fail(s, ACCORD_ERR_STATE, "no computed deps");
    std::memset(d, 0, sizeof(*d));
    if (s->ds_cur >= 0) {
        const DepSet &x = s->ds[s->ds_cur];
        d->n = x.n;
        d->kd_keys_total = x.tot_keys; d->kd_vals_total = x.tot_vals; d->kd_k2v_total = x.tot_x;
        d->rd_rngs_total = x.tot_rngs; d->rd_vals_total = x.tot_rvals; d->rd_r2v_total = x.tot_r;
        d->kd_key_off = x.key_off.as<uint32_t>(); d->kd_keys = x.keys.as<uint32_t>();
        d->kd_val_off = x.val_off.as<uint32_t>(); d->kd_vals = x.vals.as<uint32_t>();
        d->kd_k2v_off = x.x_off.as<uint32_t>(); d->kd_k2v = x.x.as<int32_t>();
        d->rd_rng_off = x.rng_off.as<uint32_t>(); d->rd_rng_start = x.rng_start.as<uint32_t>();
        d->rd_rng_end = x.rng_end.as<uint32_t>(); d->rd_val_off = x.rval_off.as<uint32_t>();
        d->rd_vals = x.rvals.as<uint32_t>(); d->rd_r2v_off = x.r_off.as<uint32_t>(); d->rd_r2v = x.r.as<int32_t>();
        return ACCORD_OK;
    }
    if (s->merged) {
        if (s->m_pending) {
            const int32_t rc = accord_impl::merge_finalize(s);
            if (rc) return rc;
        }
        d->n = s->m_n;
        d->kd_keys_total = s->m_tot_keys; d->kd_vals_total = s->m_tot_vals; d->kd_k2v_total = s->m_tot_k2v;
        d->kd_key_off = s->m_key_off.as<uint32_t>(); d->kd_keys = s->m_keys.as<uint32_t>();
        d->kd_val_off = s->m_val_off.as<uint32_t>(); d->kd_vals = s->m_vals.as<uint32_t>();
        d->kd_k2v_off = s->m_k2v_off.as<uint32_t>(); d->kd_k2v = s->m_k2v.as<int32_t>();
        d->rd_rng_off = d->rd_val_off = d->rd_r2v_off = s->m_zero.as<uint32_t>();
        return ACCORD_OK;
    }
    d->n = s->n;
    d->kd_keys_total = s->tot_keys; d->kd_vals_total = s->tot_vals; d->kd_k2v_total = s->tot_k2v;
    d->kd_key_off = s->kd_key_off.as<uint32_t>(); d->kd_keys = s->kd_keys.as<uint32_t>();
    d->kd_val_off = s->vub_off.as<uint32_t>(); d->kd_vals = s->vgap.as<uint32_t>();
    d->kd_val_cnt = s->cnt_vals.as<uint32_t>();
    d->kd_k2v_off = s->kd_k2v_off.as<uint32_t>(); d->kd_k2v = s->kd_k2v.as<int32_t>();
    d->rd_rngs_total = s->tot_rngs; d->rd_vals_total = s->tot_rvals; d->rd_r2v_total = s->tot_r2v;
    d->rd_rng_off = s->rd_rng_off.as<uint32_t>(); d->rd_val_off = s->rd_val_off.as<uint32_t>();
    d->rd_r2v_off = s->rd_r2v_off.as<uint32_t>(); d->rd_rng_start = s->rd_rng_start.as<uint32_t>();
    d->rd_rng_end = s->rd_rng_end.as<uint32_t>(); d->rd_vals = s->rd_vals.as<uint32_t>();
    d->rd_r2v = s->rd_r2v.as<int32_t>();
    return ACCORD_OK;
}

} // extern "C"

namespace accord_impl {

int32_t store_dense_keydeps(accord_store *s)
{
    if (s->kd_dense) return ACCORD_OK;
    const uint32_t n = s->n;
    const size_t n1 = (size_t)n + 1;
    hipStream_t st = s->stream;
    HostTotals *dev = s->status_totals.as<HostTotals>();
    HIPCHECK(s, s->kd_val_off.ensure(n1 * 4));
    HIPCHECK(s, s->kd_vals.ensure(s->tot_vals * 4 + 4));
    HIPCHECK(s, s->cv_tmp.ensure(accord::compact_temp_bytes(s->tot_vals)));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(n), st));
    accord::exclusive_scan_u32(s->cnt_vals.as<uint32_t>(), s->kd_val_off.as<uint32_t>(), n, &dev->totals[7], s->scan_tmp.p, st);
    accord::launch_compact_vals(n, s->vub_off.as<uint32_t>(), s->kd_val_off.as<uint32_t>(), s->vgap.as<uint32_t>(),
                                s->kd_vals.as<uint32_t>(), s->tot_vals, s->cv_tmp.p, st);
    HIPCHECK(s, hipGetLastError());
    s->kd_dense = true;
    return ACCORD_OK;
}

// Host memory of downloaded deps: one pinned block per result.  A store keeps its last block as a
// reusable arena (page-locked allocation of ~1 GB costs far more than the copy); a result still
// held when the next download starts gets a block of its own.
struct PinnedBlock {
    void *p = nullptr;
    size_t cap = 0;
    bool leased = false;      // a result points into it
    bool orphan = false;      // its store is gone: free it on release
};

void pinned_arena_destroy(accord_store *s)
{
    PinnedBlock *a = s->dl_arena;
    s->dl_arena = nullptr;
    if (!a) return;
    if (a->leased) { a->orphan = true; return; }
    if (a->p) (void)hipHostFree(a->p);
    delete a;
}

} // namespace accord_impl

namespace {

struct HostDepsOwner {
    accord_impl::PinnedBlock *block = nullptr;
    bool arena = false;       // block is its store's arena (returned on release), else owned
};

} // namespace

extern "C" {

int32_t accord_deps_download(accord_store *s, accord_deps *out)
{
    using accord_impl::PinnedBlock;
    if (!s || !out) return fail(s, ACCORD_ERR_ARG, "null argument");
    if (!s->computed) return fail(s, ACCORD_ERR_STATE, "no computed deps");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    accord_deps v;
    int32_t rc = accord_deps_device_view(s, &v);
    if (rc) return rc;
    const size_t n1 = (size_t)v.n + 1;
    // layout: 14 arrays (the last: kd_val_cnt of a gapped result), each 64-byte aligned
    const size_t cnt[14] = {n1, v.kd_keys_total, n1, v.kd_vals_total, n1, v.kd_k2v_total,
                            n1, v.rd_rngs_total, v.rd_rngs_total, n1, v.rd_vals_total, n1, v.rd_r2v_total,
                            v.kd_val_cnt ? (size_t)v.n : 0};
    const void *src[14] = {v.kd_key_off, v.kd_keys, v.kd_val_off, v.kd_vals, v.kd_k2v_off, v.kd_k2v,
                           v.rd_rng_off, v.rd_rng_start, v.rd_rng_end, v.rd_val_off, v.rd_vals, v.rd_r2v_off, v.rd_r2v,
                           v.kd_val_cnt};
    size_t off[14], total = 0;
    for (int a = 0; a < 14; ++a) { off[a] = total; total += (cnt[a] * 4 + 63) & ~(size_t)63; }
    total += 64;
    HostDepsOwner *o = new (std::nothrow) HostDepsOwner();
    if (!o) return fail(s, ACCORD_ERR_OOM, "out of host memory");
    PinnedBlock *blk = s->dl_arena;
    if (blk && !blk->leased && blk->cap < total) {       // grow the arena (page-locked, no zero fill)
        (void)hipHostFree(blk->p);
        blk->p = nullptr; blk->cap = 0;
    }
    if (!blk || blk->leased) {
        blk = new (std::nothrow) PinnedBlock();
        if (!blk) { delete o; return fail(s, ACCORD_ERR_OOM, "out of host memory"); }
        if (!s->dl_arena) s->dl_arena = blk; else o->arena = false;
    }
    o->arena = blk == s->dl_arena;
    if (!blk->p) {
        const size_t want = total + total / 8;           // headroom for the next, slightly larger batch
        if (hipHostMalloc(&blk->p, want, hipHostMallocDefault) != hipSuccess) {
            blk->p = nullptr;
            if (!o->arena) delete blk;
            delete o;
            return fail(s, ACCORD_ERR_OOM, "page-locked host allocation of %zu bytes failed", want);
        }
        blk->cap = want;
    }
    char *base = (char *)blk->p;
    hipError_t e = hipSuccess;
    for (int a = 0; a < 14 && e == hipSuccess; ++a)
        if (cnt[a]) e = hipMemcpyAsync(base + off[a], src[a], cnt[a] * 4, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e != hipSuccess) {
        if (!o->arena) { (void)hipHostFree(blk->p); delete blk; }
        delete o;
        return fail(s, ACCORD_ERR_HIP, "download: %s", hipGetErrorString(e));
    }
    blk->leased = true;
    o->block = blk;
    std::memset(out, 0, sizeof(*out));
    out->n = v.n;
    out->kd_keys_total = v.kd_keys_total; out->kd_vals_total = v.kd_vals_total; out->kd_k2v_total = v.kd_k2v_total;
    out->rd_rngs_total = v.rd_rngs_total; out->rd_vals_total = v.rd_vals_total; out->rd_r2v_total = v.rd_r2v_total;
    uint32_t *ptr[14];
    for (int a = 0; a < 14; ++a) ptr[a] = (uint32_t *)(base + off[a]);
    out->kd_key_off = ptr[0]; out->kd_keys = ptr[1]; out->kd_val_off = ptr[2]; out->kd_vals = ptr[3];
    out->kd_k2v_off = ptr[4]; out->kd_k2v = (int32_t *)ptr[5];
    out->rd_rng_off = ptr[6]; out->rd_rng_start = ptr[7]; out->rd_rng_end = ptr[8]; out->rd_val_off = ptr[9];
    out->rd_vals = ptr[10]; out->rd_r2v_off = ptr[11]; out->rd_r2v = (int32_t *)ptr[12];
    out->kd_val_cnt = v.kd_val_cnt ? ptr[13] : nullptr;
    out->owner = o;
    return ACCORD_OK;
}

void accord_deps_release(accord_deps *d)
{
    if (!d) return;
    HostDepsOwner *o = (HostDepsOwner *)d->owner;
    if (o) {
        accord_impl::PinnedBlock *blk = o->block;
        if (blk) {
            blk->leased = false;
            if (!o->arena || blk->orphan) {
                if (blk->p) (void)hipHostFree(blk->p);
                delete blk;
            }
        }
        delete o;
    }
    std::memset(d, 0, sizeof(*d));
}

int32_t accord_deps_visit(const accord_deps *d, uint32_t txn, accord_visit_fn fn, void *ctx)
{
    if (!d || !fn) return fail(nullptr, ACCORD_ERR_ARG, "accord_deps_visit: null argument");
    if (txn >= d->n) return fail(nullptr, ACCORD_ERR_ARG, "accord_deps_visit: txn %u of %u", txn, d->n);
    // keys ascending, each key's txnIds ascending (KeyDeps: header = end offsets from keyCount)
    const uint32_t k0 = d->kd_key_off[txn], nk = d->kd_key_off[txn + 1] - k0;
    const uint32_t *vals = d->kd_vals + d->kd_val_off[txn];
    const int32_t *x = d->kd_k2v + d->kd_k2v_off[txn];
    for (uint32_t k = 0; k < nk; ++k) {
        const uint32_t from = k == 0 ? nk : (uint32_t)x[k - 1], to = (uint32_t)x[k];
        for (uint32_t b = from; b < to; ++b) {
            const int32_t rc = fn(ctx, 0u, d->kd_keys[k0 + k], 0u, vals[x[b]]);
            if (rc) return rc;
        }
    }
    // then ranges in Range.compare order, each range's txnIds ascending
    if (!d->rd_rng_off) return ACCORD_OK;
    const uint32_t r0 = d->rd_rng_off[txn], nr = d->rd_rng_off[txn + 1] - r0;
    const uint32_t *rvals = d->rd_vals + d->rd_val_off[txn];
    const int32_t *y = d->rd_r2v + d->rd_r2v_off[txn];
    for (uint32_t r = 0; r < nr; ++r) {
        const uint32_t from = r == 0 ? nr : (uint32_t)y[r - 1], to = (uint32_t)y[r];
        for (uint32_t b = from; b < to; ++b) {
            const int32_t rc = fn(ctx, 1u, d->rd_rng_start[r0 + r], d->rd_rng_end[r0 + r], rvals[y[b]]);
            if (rc) return rc;
        }
    }
    return ACCORD_OK;
}

int32_t accord_deps_batch(accord_store *s, const accord_batch *b, accord_deps *out)
{
    int32_t rc = accord_batch_upload(s, b);
    if (rc) return rc;
    rc = accord_deps_compute(s);
    if (rc) return rc;
    return accord_deps_download(s, out);
}

} // extern "C"
