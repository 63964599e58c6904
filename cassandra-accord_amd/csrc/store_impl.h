// Private definition of accord_store shared by the C ABI translation units.
#pragma once
#include "../../include/accord_deps.h"
#include "kernels.h"

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>
#include <algorithm>
#include <vector>

namespace accord_impl {

extern thread_local std::string g_last_error;

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    // a regrowth takes 1.5x: a resident store's history grows a little with every batch, and an
    // exact-size buffer would be freed (a device-wide wait) and allocated again each time
    hipError_t ensure(size_t bytes)
    {
        if (bytes <= cap && p) return hipSuccess;
        size_t want = bytes < 256 ? 256 : bytes;
        if (p) {
            want = std::max(want, cap + cap / 2);
            (void)hipFree(p); p = nullptr; cap = 0;
        }
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    // the same, and every (re)allocation starts zeroed, in `stream` order (scan-state buffers rely
    // on it; the store's streams are non-blocking, so a null-stream memset would not be ordered)
    hipError_t ensure_zeroed(size_t bytes, hipStream_t stream)
    {
        if (bytes <= cap && p) return hipSuccess;
        hipError_t e = ensure(bytes);
        if (e == hipSuccess) e = hipMemsetAsync(p, 0, cap, stream);
        return e;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
    template <typename T> T *as() const { return (T *)p; }
};

struct HostTotals {
    accord::DevStatus status;
    unsigned long long totals[10];  // kd keys, kd vals bound, kd k2v, rd ranges, rd vals, rd r2v, range txns,
                                    // kd vals, resident carry entries, spare
    unsigned long long rb_tot[3];   // RedundantBefore deps: ranges, vals, r2v (counted during compute)
    accord::DevStatus rb_status;    // its capacity status, apart from the compute's
    accord::ScanCounters scan;      // the store's scan-state counters (profiled stores read them)
    uint32_t spec_abort, spec_pad;  // speculative fill: the outputs did not fit (accord_deps_compute)
    accord::DevStatus reg_status;   // accord_txn_register's check, read back (host side only)
};

// A device-resident PartialDeps set (result of accord_deps_union / accord_deps_slice).
struct DepSet {
    uint32_t n = 0;
    DevBuf key_off, keys, val_off, vals, x_off, x;                      // KeyDeps
    DevBuf rng_off, rng_start, rng_end, rval_off, rvals, r_off, r;      // RangeDeps
    uint64_t tot_keys = 0, tot_vals = 0, tot_x = 0, tot_rngs = 0, tot_rvals = 0, tot_r = 0;
    void release()
    {
        DevBuf *b[] = {&key_off, &keys, &val_off, &vals, &x_off, &x, &rng_off, &rng_start, &rng_end, &rval_off, &rvals, &r_off, &r};
        for (DevBuf *p : b) p->release();
    }
};

} // namespace accord_impl
using accord_impl::DevBuf;
using accord_impl::DepSet;
using accord_impl::HostTotals;

enum Stage { EV_START, EV_VALIDATE, EV_SORT, EV_SEGMENT, EV_COUNT, EV_SCAN, EV_FILL, EV_RANGE, EV_COMPACT,
             EV_XCHG_START, EV_XCHG_END, EV_MERGE_END, EV_WO_START, EV_WO_BITS, EV_WO_PREDS, EV_WO_LEVEL,
             EV_OP_START, EV_OP_END, EV_C_RKCP, EV_C_RKN, EV_C_KDS, EV_C_RK, EV_COUNT_ALL };

struct ShardComm;   // RCCL communicator + exchange buffers (shard.cpp)
namespace accord_impl { struct PinnedBlock; void pinned_arena_destroy(accord_store *s); struct ReadyGen; }

struct accord_store {
    accord_store_cfg cfg{};
    hipStream_t stream = nullptr;
    std::string err;
    // the CommandStores this handle hosts (cfg.store_bounds, copied; empty = one unbounded store) and
    // the uploaded batch's ranges sliced Minimal to them (host staging of accord_batch_upload)
    std::vector<uint32_t> st_bounds, sl_off, sl_start, sl_end;
    // batch (device)
    uint32_t n = 0, P = 0, R = 0;
    bool has_batch = false, computed = false;
    bool kd_dense = false;         // kd_val_off / kd_vals hold the compute's txnIds densely (store_dense_keydeps)
    DevBuf msb, lsb, node, key_off, key_ord, rng_off, rng_start, rng_end;
    // work
    DevBuf pair_key, pair_ent, sort_key, sort_pair, tmp_key, tmp_val, tmp_ent, seg_start, seg_end, radix_tmp;
    DevBuf hist, slice, hist_tmp, cnt_vub, vub_off, vgap, fk_recs, fk_list, cv_tmp, fk_ubits, fk_umode;
    DevBuf bk_list, bk_wex;        // big txns (keydeps_big_kernel): count | list, per-pair scratch
    DevBuf rng_owner, is_range, rt_excl, range_txns, cnt_rngs, cnt_rvals, cnt_r2v, rd_rng_off, rd_val_off, rd_r2v_off;
    DevBuf rd_rng_start, rd_rng_end, rd_vals, rd_r2v, rd_big, rk_cp, rk_cnt, rk_off, rk_slices, rk_cls;
    DevBuf rt_hits;                      // RangeDeps tile pass: each txn's hit count and hits, count -> fill
    uint64_t rk_keys_total = 0;      // keys of all range txns' ranges clipped to the store (upload)
    uint32_t n_range_txns = 0;
    uint64_t tot_rngs = 0, tot_rvals = 0, tot_r2v = 0;
    DevBuf cnt_keys, cnt_vals, cnt_k2v, kd_key_off, kd_val_off, kd_k2v_off, scan_tmp, status_totals;
    // outputs
    DevBuf kd_keys, kd_vals, kd_k2v, rd_zero_off;  // rd_zero_off: unused, kept for ABI-compatible views
    uint64_t tot_keys = 0, tot_vals = 0, tot_k2v = 0;
    DevBuf txn_index;              // global stream positions (nullptr = identity)
    bool has_txn_index = false;    // device txn_index valid (given by the caller, or generated)
    bool user_txn_index = false;   // given by the caller (a store subset of a stream)
    // resident CommandsForKey state (ACCORD_STORE_RESIDENT, resident.hip): the stream continues
    // across batches at global position next_global after TxnId prev_*; cy_* = the carried
    // key-major history entries (cy_key relative key ordinal, cy_ent kind<<29 | global txn)
    bool resident = false, has_prev = false;
    uint32_t next_global = 0, carry_n = 0;
    uint32_t hist_kinds = 0, b_kinds = 0;   // entry kinds (bit per kind) carried / of the uploaded batch
    uint64_t prev_msb = 0, prev_lsb = 0;
    int32_t prev_node = 0;
    DevBuf cy_key, cy_ent, cy_key2, cy_ent2, carry_tmp;
    // range commands a later batch may still see (owner global position >= next_global - W,
    // ascending; rc_n of them), double-buffered like the key history carry
    DevBuf rc_owner, rc_start, rc_end, rc_kind, rc_owner2, rc_start2, rc_end2, rc_kind2, rc_first, rc_flag, rc_offs;
    uint32_t rc_n = 0;
    // registered statuses (status.hip; resident + ACCORD_WINDOW_NONE): TxnId table sorted
    // (rg_t*, rg_tx_n entries, rg_tg = global position), InternalStatus + executeAt by global
    // position (rg_known positions), per-batch work
    DevBuf rg_tmsb, rg_tlsb, rg_tnode, rg_tg, rg_status, rg_emsb, rg_elsb, rg_enode;
    DevBuf rg_flag, rg_gcnt, rg_goff, rg_hist2, rg_kbound, rg_cwflag, rg_cwoff, rg_cwpos, rg_cwpm, rg_cwchunk, rg_hxchunk, rg_hx, rg_hu;
    DevBuf rg_chg;                 // per global position: the registration epoch of its last status change
    DevBuf rg_cchg;                // ... of its last change from uncommitted to committed / invalid
    uint32_t rg_epoch = 1;
    uint32_t rg_tx_n = 0, rg_known = 0;
    bool rg_flag_ok = false;       // rg_flag holds this batch's keys-with-registered-status flags
    // the uploaded batch: its carried-entry prefix, where it ends (global) and its last TxnId
    uint32_t b_end = 0;
    bool b_registered = false;     // the uploaded batch was computed into the resident stream
    uint64_t b_last_msb = 0, b_last_lsb = 0;
    int32_t b_last_node = 0;
    // Accept batch: executeAt per txn; bound_l / bound_g = txns started before it (local index,
    // global position), pair_bound = bound_g per (txn, key) pair
    DevBuf exec_msb, exec_lsb, exec_node, bound_l, bound_g, pair_bound;
    bool has_exec = false;
    // merged (K6) result: replaces the computed partial as the store's current deps
    bool merged = false;
    uint32_t m_n = 0, m_txn_lo = 0;
    DevBuf m_key_off, m_val_off, m_k2v_off, m_keys, m_vals, m_k2v, m_cnt_keys, m_cnt_vals, m_cnt_k2v, m_ptrs, m_zero;
    uint64_t m_tot_keys = 0, m_tot_vals = 0, m_tot_k2v = 0;
    bool m_pending = false;        // merged totals / error word in flight to `pinned` (merge_finalize)
    float xchg_ms = 0, merge_ms = 0;
    // WaitingOn + levelling (waiting_on_abi.cpp)
    bool wo_done = false;
    DevBuf wo_cnt, wo_off, wo_words, wo_aoi, pred_cnt, pred_off, preds, pred_own, level, wo_info, lv_tmp;
    bool lv_fallback = false;          // the last levelling fell back to the serial resolver
    uint32_t lv_stripe = 0;            // its stripe length (0: serial resolver alone)
    bool wo_has_aoi = false;       // accord_waiting_on_initialise: appliedOrInvalidated words in wo_aoi
    uint64_t wo_words_total = 0, preds_total = 0;
    uint32_t max_level = 0;
    float wo_ms[3] = {0, 0, 0};
    // deps-set operations (depset_abi.cpp): results double-buffered so an op may read the current
    // set; ds_cur >= 0 makes ds[ds_cur] the store's current deps
    DepSet ds[2];
    int ds_cur = -1;
    bool ds_rb = false;            // ds[ds_cur] is this batch's deps united with RedundantBefore.collectDeps
    DevBuf op_tmp[24];
    // MaxConflicts (maxconflicts.hip): per-key map (double-buffered) and the last fold's outputs
    DevBuf mc_state, mc_state2, mc_out, mc_cnt, mc_po;   // + per-txn pair counts / offsets of a pass
    uint32_t mc_next = 0;          // next txn of the uploaded batch the fold continues at
    float ops_ms = 0;
    // RedundantBefore map (accord_redundant_before_set): rb_m non-null entries, and the redundant
    // RangeDeps of the last computed batch before their union into the result
    uint32_t rb_m = 0;
    uint64_t rb_min_epoch = 0;
    DevBuf rb_start, rb_end, rb_bound, rb_sep, rb_eep, rb_cnt, rb_zero;
    DepSet rb_set;
    // the rest of each Entry (accord_redundant_before_set_ex): locallyAppliedOrInvalidatedBefore,
    // bootstrappedAt (positions, NONE = ACCORD_NO_TXN), stale; rb_ext = some entry can remove a dep
    DevBuf rb_local, rb_boot, rb_stale;
    bool rb_ext = false;
    DevBuf wo_eal;                 // WaitingOn.executeAtLeast per txn of the initialised batch (EalRec)
    DevBuf wo_err;                 // accord_waiting_on_initialise's invariant check (a HostTotals' status word)
    DevBuf rr_ovf;                 // removal kernels: spill header (count, max range deps, max entries) + list
    DevBuf rr_spill;               // removal kernels: HBM scratch of the spill pass
    // execution readiness (ready.hip): the waiting set, one generation per initialised batch
    std::vector<accord_impl::ReadyGen *> rdy_gens;
    accord_impl::ReadyGen *rdy_batch_gen = nullptr;   // the current batch's generation (until the next batch)
    bool rdy_force_full = false;             // an accord_ready_update failed part-way: evaluate everything next
    uint64_t rdy_waiting = 0;
    DevBuf rdy_spill, rdy_spill_mem;   // readiness: txns left to the removal spill pass, its HBM scratch
    // setAppliedAndPropagate: every released Range-domain txn's final appliedOrInvalidated as the
    // positions of its set RangeDeps txnIds (pv_at[g] = 1 + start in the pool, pv_len[g]; 0 = none)
    DevBuf rdy_pv_at, rdy_pv_len, rdy_pv_pool, rdy_pv_cnt;
    // event-exact readiness (accord_ready_set_mode ACCORD_READY_EVENTS, ready.hip): the live
    // generations' parameters, position -> waiting txn, key -> unmanaged slots, position -> carried
    // entries (per carry version), truncated keys
    bool rdy_event_mode = false;
    DevBuf ev_gens, ev_wmap, ev_ukcnt, ev_ukoff, ev_ukw, ev_uks, ev_pkcnt, ev_pkoff, ev_pkent, ev_tk, ev_tot;
    uint64_t ev_pk_version = ~0ull;
    uint32_t ev_pk_n = 0;
    uint32_t rdy_pv_n = 0;                    // pool entries used (read back after every call)
    size_t rdy_pv_pos = 0;                    // positions pv_at / pv_len cover
    DevBuf rdy_sum, rdy_out, rdy_kb, rdy_launch, rdy_part, rdy_kseg0, rdy_kseg1, rdy_dirty, rdy_dirty2, rdy_dlist, rdy_work, rdy_wcnt;
    uint32_t rdy_call = 0;                    // accord_ready_update calls (ids of the dirty marks)
    bool rg_flag_zeroed = false;              // the compute's init launch zeroed rg_flag (status_general_count)
    bool rb_status_zeroed = false;            // ... and the RedundantBefore status words (redundant_count)
    const void *rdy_hdr_zero = nullptr;       // rdy_out whose header the last call left zeroed (rd_host_out_kernel);
                                              // reset whenever rdy_out is reallocated
    uint32_t rdy_seen = 0;                    // rg_epoch the last accord_ready_update saw
    uint64_t rdy_sum_version = ~0ull;         // carry version the key summaries belong to
    uint64_t rdy_kseg_version = ~0ull, carry_version = 0;   // the carry's segment bounds are cached per carry version
    void *rdy_host = nullptr;                 // page-locked: the ready count + list readback
    void *rdy_tab_host = nullptr;             // pinned staging of the evaluation launch tables
    std::vector<uint8_t> rdy_tab_last;        // the tables last sent, and where to
    void *rdy_tab_dev = nullptr;
    void *reg_host = nullptr;                 // pinned staging of accord_txn_register's events (one copy)
    void *rb_host = nullptr;                  // pinned staging of accord_redundant_before_set's entries (one copy)
    size_t rb_host_cap = 0;
    DevBuf rb_pack;                           // ... their device landing, scattered by one launch
    size_t reg_host_cap = 0;
    void *up_host = nullptr;                  // pinned staging of a small batch's upload (one copy)
    size_t up_host_cap = 0;
    hipEvent_t up_ev[2] = {nullptr, nullptr}; // the staging halves' copies (accord_batch_upload)
    bool up_ev_live[2] = {false, false};
    uint32_t up_half = 0;
    DevBuf up_stage;                          // its device side, scattered to the batch arrays
    size_t rdy_tab_cap = 0;
    uint64_t *rdy_stats = nullptr;            // ACCORD_READY_STATS diagnostics
    std::vector<uint32_t> rdy_kb_host;       // per key: shardRedundantBefore as a position (cumulative max)
    bool rdy_kb_dirty = false;
    std::vector<uint32_t> rdy_list;          // the last accord_ready_update's ready txns
    std::vector<uint64_t> rdy_eal_msb, rdy_eal_lsb;   // and their executesAtLeast
    std::vector<int32_t> rdy_eal_node;
    // stream segments (segment.hip): the store owns positions [seg_base, seg_base + n) of every
    // CommandStore; its summary for later segments, and the fold of earlier ones into the carry
    bool seg_active = false, seg_sum_ok = false, seg_carry_ok = false;
    uint32_t seg_base = 0;
    uint64_t seg_sum_n = 0;
    float seg_summary_ms = 0, seg_carry_ms = 0;
    hipEvent_t seg_ev[4] = {};
    bool seg_ev_created = false;
    DevBuf sg_lastw, sg_flag, sg_off, sg_key, sg_ent, sg_cnt, sg_koff, sg_word, sg_lw;
    ShardComm *comm = nullptr;
    HostTotals *pinned = nullptr;
    accord_impl::PinnedBlock *dl_arena = nullptr;   // page-locked host arena of accord_deps_download
    hipEvent_t ev[EV_COUNT_ALL] = {};
    bool events = false;
    bool ev_created = false;                 // the HIP events exist (profiling switched on once)
    accord_timing timing{};
    accord::ScanCounters scan_seen{};   // scan counters at the end of the previous profiled compute
    uint32_t computes_since_zero = 0;   // computes since the scan state was last zeroed
    int wpl = 1;
};


namespace accord_impl {
int32_t fail(accord_store *s, int32_t code, const char *fmt, ...);
void shard_comm_destroy(accord_store *s);
void segment_destroy(accord_store *s);      // stream segments' buffers and events (segment.hip)
int32_t merge_finalize(accord_store *s);   // read a bounded merge's totals (shard.cpp)
// registered statuses (status.hip)
bool registered_mode(const accord_store *s);
int32_t status_general_count(accord_store *s, uint32_t C, uint32_t PH, bool *pending);
int32_t status_general_emit(accord_store *s, uint32_t PH, uint64_t X, const uint32_t *abort,
                            const uint32_t **hist_for_fill);
int32_t status_prune_flags(accord_store *s, uint32_t PH, uint32_t *keep_flag);
int32_t status_truncate_carry(accord_store *s, uint32_t m, const uint32_t *start, const uint32_t *end,
                              const uint32_t *bound);
int32_t status_join_queue(accord_store *s, const accord::DevStatus *guard);
void status_join_commit(accord_store *s);
int32_t status_range_keys(accord_store *s, const accord::RangeDepsParams &rp, bool fill);
int32_t status_waiting_on_init(accord_store *s, const uint32_t *wo_off, unsigned long long *words,
                               unsigned long long *aoi);
// execution readiness (ready.hip)
int32_t ready_track_batch(accord_store *s);
int32_t ready_batch_check(accord_store *s);
void ready_destroy(accord_store *s);
// event-exact readiness: a registration's events replayed in order (instead of the bulk status
// apply), a generation's initialisation, and the keys a truncation took entries from
int32_t ready_register_events(accord_store *s, uint32_t n, const uint32_t *pos, const uint8_t *status,
                              const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode, uint32_t epoch);
int32_t ready_init_events(accord_store *s);
int32_t ready_truncate_keys(accord_store *s, const std::vector<uint32_t> &kb, std::vector<uint32_t> &keys);
int32_t ready_truncate_events(accord_store *s, const std::vector<uint32_t> &keys);
// RedundantBefore.collectDeps of the computed batch, unioned into the store's result (depset_abi.cpp):
// the count and its scans are queued inside the compute (totals arrive with its final copy), the
// fill and the union after it
int32_t redundant_count(accord_store *s);
int32_t redundant_apply(accord_store *s);
// The batch's current deps (device): the pipeline's own output, or its RedundantBefore union.
struct CurDeps {
    const uint32_t *kd_key_off, *kd_keys, *kd_val_off, *kd_vals, *kd_k2v_off, *kd_k2v;
    const uint32_t *kd_val_cnt;       // gapped KeyDeps txnIds (the compute's own output), else nullptr
    const uint32_t *rd_val_off, *rd_vals;
    const uint32_t *rd_rng_off, *rd_rng_start, *rd_rng_end, *rd_r2v_off, *rd_r2v;
    uint64_t tot_keys, tot_vals, tot_k2v, tot_rvals, tot_rngs, tot_r2v;
};
CurDeps cur_deps(const accord_store *s);
// The compute's KeyDeps txnIds in dense form (kd_val_off / kd_vals: the scan of cnt_vals and the
// compaction of vgap), for the operations that ship or copy them; once per compute
int32_t store_dense_keydeps(accord_store *s);
}
using accord_impl::fail;

#define HIPCHECK(s, expr)                                                                             \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) return fail((s), ACCORD_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)
