// C ABI of WaitingOn bitsets + execution levelling (include/accord_deps.h; config 5).
// Runs over the store's computed deps and the key histories the deps pipeline left in HBM.
#include "store_impl.h"

#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <new>
#include <vector>

namespace {

void record(accord_store *s, int stage)
{
    if (s->events) (void)hipEventRecord(s->ev[stage], s->stream);
}

struct HostWaitingOnOwner {
    std::vector<uint32_t> level, wo_off;
    std::vector<uint64_t> words, aoi;
};

} // namespace

extern "C" {

int32_t accord_waiting_on_compute(accord_store *s)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (!s->computed) return fail(s, ACCORD_ERR_STATE, "accord_waiting_on_compute before accord_deps_compute");
    if (s->merged || s->has_txn_index)
        return fail(s, ACCORD_ERR_STATE, "WaitingOn levelling runs on a full stream's deps (gather to one store first)");
    if (s->ds_cur >= 0)   // a union / slice / RedundantBefore result: the model's deps are the pipeline's own
        return fail(s, ACCORD_ERR_STATE, "WaitingOn levelling runs on the computed deps, not a deps-set result");
    if (s->has_exec)   // the levelling model is defined on PreAccept deps
        return fail(s, ACCORD_ERR_STATE, "WaitingOn levelling runs on a PreAccept batch's deps, not an Accept batch");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    const uint32_t n = s->n;
    const size_t n1 = (size_t)n + 1;
    hipStream_t st = s->stream;
    s->wo_done = false;
    s->wo_has_aoi = false;
    HIPCHECK(s, s->wo_cnt.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->wo_off.ensure(n1 * 4));
    HIPCHECK(s, s->pred_cnt.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->pred_off.ensure(n1 * 4));
    HIPCHECK(s, s->level.ensure((size_t)n * 4 + 4));
    // levelling: by stripes (levels.hip) unless ACCORD_LV_MODE=serial; ACCORD_LV_STRIPE / ACCORD_LV_RELAX
    // override the stripe length and the sweep bound (tests force the serial fallback with them)
    const char *lv_mode = getenv("ACCORD_LV_MODE");
    const bool striped = !(lv_mode && !strcmp(lv_mode, "serial"));
    const char *lv_z = getenv("ACCORD_LV_STRIPE"), *lv_r = getenv("ACCORD_LV_RELAX");
    const uint32_t stripe = lv_z ? (uint32_t)atoi(lv_z) : accord::levels_stripe_default(n);
    // sweeps: 8 queued with the levelling (config 5 reaches the fixpoint in 6), then up to `relax`
    // in a second round after the host has seen the first round's flag
    const uint32_t relax = lv_r ? (uint32_t)atoi(lv_r) : 32u, relax1 = std::min(relax, 8u);
    HIPCHECK(s, s->lv_tmp.ensure(std::max(accord::levels_temp_bytes(n), accord::levels_striped_temp_bytes(n, stripe))));
    HIPCHECK(s, s->wo_info.ensure(64));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(n), s->stream));
    HostTotals *dev = s->status_totals.as<HostTotals>();

    accord::WaitingOnParams p{};
    p.n = n;
    p.lsb = s->lsb.as<uint64_t>();
    p.key_off = s->key_off.as<uint32_t>();
    p.slice = s->slice.as<accord::PairSlice>();
    p.hist = s->hist.as<uint32_t>();
    p.pw_local = s->hist_tmp.as<uint32_t>();
    p.pw_carry = p.pw_local + s->P;
    p.pw_tile = accord::HISTORY_TILE;
    p.kd_val_off = s->vub_off.as<uint32_t>(); p.kd_vals = s->vgap.as<uint32_t>();   // gapped: counts in cnt_vals
    p.kd_val_cnt = s->cnt_vals.as<uint32_t>();
    p.rd_val_off = s->rd_val_off.as<uint32_t>(); p.rd_vals = s->rd_vals.as<uint32_t>();
    p.pred_cnt = s->pred_cnt.as<uint32_t>();
    p.rw_only = (((s->resident ? s->hist_kinds : 0u) | s->b_kinds) & ~3u) == 0u ? 1u : 0u;

    record(s, EV_WO_START);
    accord::launch_wo_words_count(n, s->kd_key_off.as<uint32_t>(), p.rd_val_off, s->wo_cnt.as<uint32_t>(), st);
    accord::exclusive_scan_u32(s->wo_cnt.as<uint32_t>(), s->wo_off.as<uint32_t>(), n, &dev->totals[0], s->scan_tmp.p, st);
    accord::launch_wo_preds_count(p, st);
    accord::exclusive_scan_u32(p.pred_cnt, s->pred_off.as<uint32_t>(), n, &dev->totals[1], s->scan_tmp.p, st);
    HIPCHECK(s, hipMemcpyAsync(s->pinned->totals, dev->totals, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    s->wo_words_total = s->pinned->totals[0];
    s->preds_total = s->pinned->totals[1];
    if (s->preds_total >= (1ull << 32)) return fail(s, ACCORD_ERR_CAPACITY, "reduced DAG exceeds 2^32 edges");
    HIPCHECK(s, s->wo_words.ensure(s->wo_words_total * 8));
    HIPCHECK(s, s->preds.ensure(s->preds_total * 4));
    if (striped) HIPCHECK(s, s->pred_own.ensure(s->preds_total + 16));
    accord::launch_wo_bits(n, s->kd_key_off.as<uint32_t>(), p.rd_val_off, s->wo_off.as<uint32_t>(),
                           s->wo_words.as<unsigned long long>(), st);
    record(s, EV_WO_BITS);
    p.pred_off = s->pred_off.as<uint32_t>();
    p.preds = s->preds.as<uint32_t>();
    p.pred_own = striped ? s->pred_own.as<uint8_t>() : nullptr;
    accord::launch_wo_preds_fill(p, st);
    record(s, EV_WO_PREDS);
    HIPCHECK(s, hipMemsetAsync(s->wo_info.p, 0, 64, st));
    if (striped)
        accord::launch_levels_striped(n, p.pred_off, p.preds, p.pred_own, s->level.as<uint32_t>(), s->wo_info.as<uint32_t>(),
                                      s->lv_tmp.p, stripe, relax1, st);
    else
        accord::launch_levels(n, p.pred_off, p.preds, s->level.as<uint32_t>(), s->wo_info.as<uint32_t>(),
                              s->lv_tmp.p, st);
    record(s, EV_WO_LEVEL);
    uint32_t info[4] = {0, 0, 0, 0};
    HIPCHECK(s, hipMemcpyAsync(info, s->wo_info.p, sizeof(info), hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    HIPCHECK(s, hipGetLastError());
    if (info[2]) return fail(s, ACCORD_ERR_STATE, "a dependency does not precede its txn");
    s->lv_fallback = false;
    s->lv_stripe = striped ? stripe : 0u;
    if (striped && info[3] && relax > relax1) {   // a second round of sweeps
        accord::launch_levels_sweeps(n, p.pred_off, p.preds, s->level.as<uint32_t>(), s->wo_info.as<uint32_t>(),
                                     s->lv_tmp.p, stripe, relax1, relax, st);
        record(s, EV_WO_LEVEL);
        HIPCHECK(s, hipMemcpyAsync(info, s->wo_info.p, sizeof(info), hipMemcpyDeviceToHost, st));
        HIPCHECK(s, hipStreamSynchronize(st));
        HIPCHECK(s, hipGetLastError());
        if (info[2]) return fail(s, ACCORD_ERR_STATE, "a dependency does not precede its txn");
    }
    if (striped && info[3]) {   // the sweeps did not reach the fixpoint: the serial resolver, exact
        s->lv_fallback = true;
        HIPCHECK(s, hipMemsetAsync(s->wo_info.p, 0, 64, st));
        accord::launch_levels(n, p.pred_off, p.preds, s->level.as<uint32_t>(), s->wo_info.as<uint32_t>(),
                              s->lv_tmp.p, st);
        record(s, EV_WO_LEVEL);
        HIPCHECK(s, hipMemcpyAsync(info, s->wo_info.p, sizeof(info), hipMemcpyDeviceToHost, st));
        HIPCHECK(s, hipStreamSynchronize(st));
        HIPCHECK(s, hipGetLastError());
        if (info[2]) return fail(s, ACCORD_ERR_STATE, "a dependency does not precede its txn");
    }
    if (info[0]) return fail(s, ACCORD_ERR_CAPACITY, "levelling did not drain (%u chunks resolved)", info[0] - 1);
    s->max_level = info[1];
    if (s->events) {
        auto el = [&](int a, int b) { float ms = 0; (void)hipEventElapsedTime(&ms, s->ev[a], s->ev[b]); return ms; };
        // the count + scans before the bitset fill are attributed to the bitset stage
        s->wo_ms[0] = el(EV_WO_START, EV_WO_BITS);
        s->wo_ms[1] = el(EV_WO_BITS, EV_WO_PREDS);
        s->wo_ms[2] = el(EV_WO_PREDS, EV_WO_LEVEL);
    }
    s->wo_done = true;
    return ACCORD_OK;
}

int32_t accord_waiting_on_levelling(accord_store *s, uint32_t *stripe, uint32_t *fallback)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (!s->wo_done) return fail(s, ACCORD_ERR_STATE, "no accord_waiting_on_compute result");
    if (stripe) *stripe = s->lv_stripe;
    if (fallback) *fallback = s->lv_fallback ? 1u : 0u;
    return ACCORD_OK;
}

int32_t accord_waiting_on_initialise(accord_store *s)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (!accord_impl::registered_mode(s))
        return fail(s, ACCORD_ERR_STATE, "accord_waiting_on_initialise needs a registered-status store "
                                         "(resident, window ACCORD_WINDOW_NONE)");
    if (!s->computed) return fail(s, ACCORD_ERR_STATE, "accord_waiting_on_initialise before accord_deps_compute");
    if (s->merged || (s->ds_cur >= 0 && !s->ds_rb))
        return fail(s, ACCORD_ERR_STATE, "accord_waiting_on_initialise runs on the batch's computed deps "
                                         "(or their RedundantBefore union), not a union / slice result");
    {
        const int32_t rc = accord_impl::ready_batch_check(s);   // at most one evaluated generation per batch
        if (rc != ACCORD_OK) return rc;
    }
    const accord_impl::CurDeps cd = accord_impl::cur_deps(s);
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    const uint32_t n = s->n;
    hipStream_t st = s->stream;
    s->wo_done = false;
    HIPCHECK(s, s->wo_cnt.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->wo_off.ensure(((size_t)n + 1) * 4));
    HIPCHECK(s, s->level.ensure((size_t)n * 4 + 4));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(n), s->stream));
    HIPCHECK(s, s->status_totals.ensure(sizeof(HostTotals)));
    HostTotals *dev = s->status_totals.as<HostTotals>();
    accord::launch_wo_words_count(n, cd.kd_key_off, cd.rd_val_off, s->wo_cnt.as<uint32_t>(), st);
    accord::exclusive_scan_u32(s->wo_cnt.as<uint32_t>(), s->wo_off.as<uint32_t>(), n, &dev->totals[0], s->scan_tmp.p, st);
    HIPCHECK(s, hipMemcpyAsync(s->pinned->totals, dev->totals, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    s->wo_words_total = s->pinned->totals[0];
    HIPCHECK(s, s->wo_words.ensure(s->wo_words_total * 8 + 8));
    HIPCHECK(s, s->wo_aoi.ensure(s->wo_words_total * 8 + 8));
    int32_t rc = accord_impl::status_waiting_on_init(s, s->wo_off.as<uint32_t>(), s->wo_words.as<unsigned long long>(),
                                                     s->wo_aoi.as<unsigned long long>());
    if (rc != ACCORD_OK) return rc;
    if (n) HIPCHECK(s, hipMemsetAsync(s->level.p, 0, (size_t)n * 4, st));   // no levelling here
    HIPCHECK(s, hipStreamSynchronize(st));
    HIPCHECK(s, hipGetLastError());
    s->preds_total = 0;
    s->max_level = 0;
    s->wo_has_aoi = true;
    s->wo_done = true;
    rc = accord_impl::ready_track_batch(s);        // the batch joins the waiting set (ready.hip)
    if (rc == ACCORD_OK && s->rdy_event_mode) rc = accord_impl::ready_init_events(s);
    return rc;
}

int32_t accord_waiting_on_download(accord_store *s, accord_waiting_on *out)
{
    if (!s || !out) return fail(s, ACCORD_ERR_ARG, "null argument");
    if (!s->wo_done) return fail(s, ACCORD_ERR_STATE, "no computed WaitingOn");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    HostWaitingOnOwner *o = new (std::nothrow) HostWaitingOnOwner();
    if (!o) return fail(s, ACCORD_ERR_OOM, "out of host memory");
    const size_t n = s->n;
    try {
        o->level.resize(n + 1);
        o->wo_off.resize(n + 1);
        o->words.resize(s->wo_words_total + 1);
        if (s->wo_has_aoi) o->aoi.resize(s->wo_words_total + 1);
    } catch (...) {
        delete o;
        return fail(s, ACCORD_ERR_OOM, "out of host memory");
    }
    hipError_t e = hipSuccess;
    if (n) e = hipMemcpyAsync(o->level.data(), s->level.p, n * 4, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(o->wo_off.data(), s->wo_off.p, (n + 1) * 4, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess && s->wo_words_total)
        e = hipMemcpyAsync(o->words.data(), s->wo_words.p, s->wo_words_total * 8, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess && s->wo_has_aoi && s->wo_words_total)
        e = hipMemcpyAsync(o->aoi.data(), s->wo_aoi.p, s->wo_words_total * 8, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e != hipSuccess) {
        delete o;
        return fail(s, ACCORD_ERR_HIP, "download: %s", hipGetErrorString(e));
    }
    std::memset(out, 0, sizeof(*out));
    out->n = s->n;
    out->max_level = s->max_level;
    out->words_total = s->wo_words_total;
    out->preds_total = s->preds_total;
    out->level = o->level.data();
    out->wo_off = o->wo_off.data();
    out->words = o->words.data();
    out->applied_or_invalidated = s->wo_has_aoi ? o->aoi.data() : nullptr;
    out->owner = o;
    return ACCORD_OK;
}

void accord_waiting_on_release(accord_waiting_on *w)
{
    if (!w) return;
    delete (HostWaitingOnOwner *)w->owner;
    std::memset(w, 0, sizeof(*w));
}

int32_t accord_waiting_on_timing(accord_store *s, float *bits_ms, float *preds_ms, float *level_ms)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (bits_ms) *bits_ms = s->wo_ms[0];
    if (preds_ms) *preds_ms = s->wo_ms[1];
    if (level_ms) *level_ms = s->wo_ms[2];
    return ACCORD_OK;
}

} // extern "C"
