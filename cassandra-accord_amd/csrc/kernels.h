// Host-side launch wrappers of the deps kernels (implemented in *.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "device_common.h"

namespace accord {

// device error word codes (first error wins; see include/accord_deps.h)
struct DevStatus {
    unsigned long long first;   // (txn << 32) | -code of the lowest-index failure; ~0 = none
    uint32_t overflow;          // txns that exceeded the per-wave capacity
    uint32_t overflow_first;    // lowest such txn (~0 = none)
};

// ---- radix sort (radix_sort.hip) ----
size_t radix_sort_temp_bytes(uint32_t n);
uint32_t radix_sort_scan_len(uint32_t n);   // longest scan the sort runs (size its scan state for it)
// Stable LSD sort of (key, val) by key over `bits` low bits.  Result ends in keys_out/vals_out.
// keys_tmp/vals_tmp are ping-pong buffers of n entries.
// ents_in (optional, may be null) is a second value carried the same way into ents_out.
void radix_sort_pairs(const uint32_t *keys_in, const uint32_t *vals_in, uint32_t *keys_out, uint32_t *vals_out,
                      uint32_t *keys_tmp, uint32_t *vals_tmp, const uint32_t *ents_in, uint32_t *ents_out,
                      uint32_t *ents_tmp, uint32_t n, int bits, void *temp, void *scan_state, hipStream_t s);
// A resident store's batch (P pairs: keys bkey, entries bent, TxnId order) joined to its carried
// key-major history (C entries) without re-sorting the carry: the same sort_key / sort_pair / hist
// as radix_sort_pairs over [carry | batch].  comp_tmp, sorted_tmp: P words each.  merge_join_fits:
// P and the key bits qualify (chunks of 1024 pairs sorted in LDS, up to 16 of them).
bool merge_join_fits(uint32_t P, int bits);
void merge_join_batch(const uint32_t *ckey, const uint32_t *cent, uint32_t C, const uint32_t *bkey,
                      const uint32_t *bent, uint32_t P, int bits, uint32_t *comp_tmp, uint32_t *sorted_tmp,
                      uint32_t *sort_key, uint32_t *sort_pair, uint32_t *hist, hipStream_t s);

// ---- small fills in one launch (scan.hip): descriptor k sets words [0, d[k].words) of d[k].p ----
struct FillDesc {
    uint32_t *p;
    uint32_t words, value;
};
// Capacity: the most descriptors any caller adds is 16 fills (the compute's init launch) and 12
// copies (accord_batch_upload's pack); both lists keep headroom, and an add past the capacity is a
// programming error that stops the process instead of writing past the array.
[[noreturn]] void list_capacity_exceeded(const char *what);
struct FillList {
    static constexpr uint32_t CAP = 24;
    FillDesc d[CAP];
    uint32_t nd = 0;
    void add(void *p, size_t bytes, uint32_t value)
    {
        if (bytes < 4) return;
        if (nd >= CAP) list_capacity_exceeded("FillList");
        d[nd++] = FillDesc{(uint32_t *)p, (uint32_t)(bytes / 4), value};
    }
};
void launch_fill_words(const FillList &L, hipStream_t s);
// small device-to-device copies in one launch: descriptor k copies d[k].words words
struct CopyDesc {
    const uint32_t *src;
    uint32_t *dst;
    uint32_t words;
};
struct CopyList {
    static constexpr uint32_t CAP = 20;
    CopyDesc d[CAP];
    uint32_t nd = 0;
    void add(const void *src, void *dst, size_t bytes)
    {
        if (bytes < 4) return;
        if (nd >= CAP) list_capacity_exceeded("CopyList");
        d[nd++] = CopyDesc{(const uint32_t *)src, (uint32_t *)dst, (uint32_t)(bytes / 4)};
    }
};
void launch_copy_words(const CopyList &L, hipStream_t s);
void launch_init_words(const FillList &F, const CopyList &L, hipStream_t s);   // both in one launch

// ---- scan (scan.hip) ----
// temp: a scan-state buffer of at least scan_temp_bytes(n) bytes, ZERO when allocated
// (DevBuf::ensure_zeroed) and used for nothing else, starting at the same address for every scan
// that shares it (the store's scan_tmp); scans sharing it must run in stream order (it resets itself).
size_t scan_temp_bytes(uint32_t n);
// cumulative counters at the start of a scan-state buffer (since it was allocated): look-back spin
// iterations, and look-backs that stopped waiting and summed the predecessors' inputs
struct ScanCounters {
    unsigned long long spins;
    unsigned long long fallbacks;
};
inline const void *scan_counters(const void *temp) { return (const char *)temp + 16; }
// out[i] = sum(in[0..i)), i in [0, n]; out has n+1 entries; total also written to *total_dev (u64).
void exclusive_scan_u32(const uint32_t *in, uint32_t *out, uint32_t n, unsigned long long *total_dev, void *temp,
                        hipStream_t s);
// The speculative fill's check (store.cpp), done by the scan of the KeyDeps sizes as it writes the
// totals: *abort = 1 when a total exceeds its capacity (keys, txnIds bound, k2v -- the scan's three
// arrays), the registered store's general-pass extension *xtot exceeds cap_x, or *status records a
// failure; else 0.
struct SpecCheck {
    uint32_t *abort;
    const DevStatus *status;
    const unsigned long long *xtot;    // nullptr: no extension
    unsigned long long cap[3], cap_x;
};
// the same for na (1..4) arrays of n counts in one launch (total[k] may be null); spec (na == 3):
// the speculative fill's check on the totals
void exclusive_scan_multi(int na, const uint32_t *const *in, uint32_t *const *out, unsigned long long *const *total,
                          uint32_t n, void *temp, hipStream_t s, const SpecCheck *spec = nullptr);

// ---- key deps pipeline (keydeps.hip) ----
// Per (txn, key) pair, txn-major: the deps slice [lo, pos) of the key's history, the number of
// its entries the txn's kind witnesses, and the pair's store-relative key ordinal.  One 16-byte
// record so the key-major -> txn-major scatter is a single store per pair (and the fill reads the
// key with the slice).
struct alignas(16) PairSlice {
    uint32_t lo, pos, wcnt, key;
};

struct KeyDepsParams {
    uint32_t n;
    uint32_t P;                        // (txn, key) pairs of the batch (key_off[n])
    const uint64_t *msb, *lsb;
    const int32_t *node;
    const uint32_t *key_off, *key_ord;
    const uint32_t *txn_index;         // global stream positions or nullptr
    uint32_t key_lo, key_hi;
    uint32_t window;
    const uint32_t *hist;              // key-major history entries (kind<<29 | global txn)
    const PairSlice *slice;            // txn-major per pair
    const uint32_t *cnt_vub;           // txnIds upper bound per txn (sizes pass / rangekeys count)
    uint32_t *cnt_vals;                // out: exact txnIds count per txn
    const uint32_t *kd_key_off, *vub_off, *kd_k2v_off;
    uint32_t *kd_keys, *vgap;          // txnIds land at vgap[vub_off[i] ..], compacted afterwards
    int32_t *kd_k2v;
    DevStatus *status;
    // fast path / fallback: the txns the fast kernel could not take, processed by the general one
    uint32_t *fb_list, *fb_count;
    // Accept batch: per txn the global position bounding its candidates (txns started before its
    // executeAt); nullptr = PreAccept (bound = own position).  The txn itself is never a dep (p1).
    const uint32_t *bound_g;
    // big txns (more keys than a wave has lanes, or more distinct far deps than the general kernel's
    // far list): listed by the general kernel, built by a workgroup each (big_wex: scratch per pair)
    uint32_t *big_list, *big_count, *big_wex;
    uint32_t tiny;                     // thread-per-txn pass for tiny txns (batches of few keys per txn)
    // speculative fill (store.cpp): a word set by the sizes' scan (SpecCheck) when the outputs would not fit;
    // every fill kernel then returns at once.  nullptr: the fill runs unconditionally
    const uint32_t *abort;
};

// Where a batch sits in the store's stream: global positions start at min_gi, and (has_prev) the
// first TxnId must follow the last one the (resident) store holds.
struct StreamPos {
    uint32_t min_gi, has_prev;
    uint64_t prev_msb, prev_lsb;
    int32_t prev_node, pad;
};
// txn-major validation + (key, entry) pair packing; range CSR owners and range-txn flags
void launch_validate_pack(uint32_t n, const uint64_t *msb, const uint64_t *lsb, const int32_t *node,
                          const uint32_t *key_off, const uint32_t *key_ord, const uint32_t *rng_off,
                          const uint32_t *rng_start, const uint32_t *rng_end, uint32_t key_lo, uint32_t key_hi,
                          uint32_t *pair_key, uint32_t *pair_ent, uint32_t *rng_owner, uint32_t *is_range,
                          const uint32_t *txn_index, const StreamPos &sp, DevStatus *status, hipStream_t s);
// Accept batch: bound_l[t] = #batch txns with txnId < executeAt[t], bound_g[t] = its global
// position, pair_bound[p] = bound_g of p's txn; executeAt < txnId -> ACCORD_ERR_ARG
void launch_accept_bounds(uint32_t n, const uint64_t *msb, const uint64_t *lsb, const int32_t *node,
                          const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode, const uint32_t *key_off,
                          const uint32_t *txn_index, uint32_t *bound_l, uint32_t *bound_g, uint32_t *pair_bound,
                          DevStatus *status, hipStream_t s);
// range_txns[excl[i]] = i for every i with is_range[i]
void launch_compact_flags(uint32_t n, const uint32_t *flags, const uint32_t *excl, uint32_t *out, hipStream_t s);
size_t history_temp_bytes(uint32_t P);
// key-major: history entries, segments, and per pair its deps slice (txn-major PairSlice).  P counts
// the combined history; sorted_pair values < carry are a resident store's carried entries (no slice).
void launch_history(uint32_t P, uint32_t nkeys, uint32_t window, const uint32_t *sorted_key,
                    const uint32_t *sorted_pair, const uint32_t *hist, uint32_t *seg_start,
                    uint32_t *seg_end, PairSlice *slice, void *temp, const uint32_t *pair_bound, uint32_t carry,
                    hipStream_t s);
// history tile size of the Write max-scan carry (pw_local / pw_carry) and class-count carries
constexpr uint32_t HISTORY_TILE = 4096;
// Views into the history temp buffer launch_history leaves behind: (last Write <= x) + 1 =
// max(pw_local[x], pw_carry[x / HISTORY_TILE]); witnessed counts via witnessed_upto(c_local, ccarry).
struct HistoryViews {
    uint32_t *pw_local, *pw_carry;
    uint64_t *c_local;
    ClassCarry *ccarry;
};
HistoryViews history_views(void *temp, uint32_t P);
// per txn: keys, txnIds upper bound and keysToTxnIds sizes from the witnessed counts
void launch_keydeps_sizes(uint32_t n, const uint32_t *key_off, const PairSlice *slice, uint32_t *cnt_keys,
                          uint32_t *cnt_vub, uint32_t *cnt_k2v, DevStatus *status, hipStream_t s);
// fill = fast kernel over every txn (k <= 8, <= 256 candidates, deps in the near span) + the general
// kernel over the txns it hands back (p.fb_list / p.fb_count, count zeroed before the launch)
size_t keydeps_fast_temp_bytes(uint32_t n);
void launch_keydeps_recs(const KeyDepsParams &p, void *recs, hipStream_t s);   // before launch_keydeps_fill
void launch_keydeps_fill(const KeyDepsParams &p, int span_words_per_lane, void *recs, hipStream_t s);
void launch_keydeps_big(const KeyDepsParams &p, hipStream_t s);
// vals[val_off[i] ..] = vgap[vub_off[i] ..] (val_off[i+1] - val_off[i] entries): the dense form of a
// gapped KeyDeps txnIds array, for the operations that ship or copy it (store_dense_keydeps)
size_t compact_temp_bytes(uint64_t max_total);
void launch_compact_vals(uint32_t n, const uint32_t *vub_off, const uint32_t *val_off, const uint32_t *vgap,
                         uint32_t *vals, uint64_t max_total, void *temp, hipStream_t s);

// ---- resident CFK state across batches (resident.hip) ----
void launch_gen_index(uint32_t n, uint32_t base, uint32_t *out, hipStream_t s);
size_t carry_temp_bytes(uint32_t P, uint32_t nkeys);   // scan state separate (scan of P flags)
// the entries of the combined history a later batch can still reach (per key: from the last Write
// with txn < thr, else everything; or, flags_given, the keep flags already in carry_flags(temp))
// -> out_key/out_ent, key-major; their count in *total
uint32_t *carry_flags(void *temp, uint32_t nkeys);   // [P + 1] keep flags inside the carry temp
void launch_carry(uint32_t P, uint32_t nkeys, uint32_t thr, const uint32_t *sorted_key, const uint32_t *hist,
                  const uint32_t *seg_start, const uint32_t *seg_end, const HistoryViews &hv, void *temp,
                  void *scan_state, uint32_t *out_key, uint32_t *out_ent, unsigned long long *total, bool flags_given,
                  hipStream_t s);

// ---- range txns (rangedeps.hip) ----
constexpr uint32_t RT_HIT_WORDS = 8;   // 16 hits per txn (rangedeps_tile_kernel's RT_HL)
struct RangeDepsParams {
    uint32_t n;
    const uint64_t *lsb;
    const uint32_t *key_off, *key_ord;
    const uint32_t *rng_off, *rng_start, *rng_end, *rng_owner;
    uint32_t window, key_lo, key_hi;
    // history (for range txns' KeyDeps)
    const uint32_t *hist, *seg_start, *seg_end, *pw_local, *pw_carry;
    uint32_t pw_tile;
    uint32_t kinds_present;             // entry kinds in the history (bit per kind; SP and XSP together)
    const uint64_t *c_local;            // witnessed counts (HistoryViews)
    const ClassCarry *ccarry;
    uint2 *cp;                          // checkpoints: first history position with txn >= b << RK_CP_SHIFT
                                        //   {position, its txn, (last Write before it) + 1, 0}
    uint32_t nkeys, ncp;                //   per key (cp[b * nkeys + k]), ncp blocks
    uint32_t *cnt_vals_exact;           // exact txnIds count per txn (range txns: written by the union pass)
    uint32_t *rd_big_list, *rd_big_count;   // txns with more range hits than the per-txn pass holds
    uint32_t *rd_fb_list, *rd_fb_count;     // txns the tile pass hands to the per-txn pass
    uint32_t *rt_h, *rt_hits;               // tile pass: per txn its hit count (~0: per-txn pass) and
                                            //   RT_HIT_WORDS words of 16-bit candidate slots, count -> fill
    const uint32_t *rk_off;             // per range txn: first of its stored key slices
    uint2 *rk_slices;                   // (lo, raw | wcnt << 16) per key of every range txn's ranges
    uint32_t n_range_txns;
    const uint32_t *range_txns;
    uint32_t *rk_cls;                   // union size classes: counts [0, 8), then per class n_range_txns
                                        //   records {txn, D, body base, txnIds base} (uint4)
    uint32_t rk_bitmap;                 // union by span bitmap when the body spans < 4096 txns (else sort)
    const uint32_t *bound_l;            // Accept batch: txns started before executeAt (nullptr = i)
    // resident stores: txn i of the batch is stream position g0 + i; the range commands carried
    // from earlier batches (owner positions ascending, all before g0) precede the batch's own in
    // the candidate order; checkpoints cover txn blocks [cp_base, cp_base + ncp)
    uint32_t g0, ncr, cp_base;
    const uint32_t *rc_owner, *rc_start, *rc_end, *rc_kind;
    // RangeDeps counts / outputs
    uint32_t *cnt_rngs, *cnt_vals, *cnt_r2v;
    const uint32_t *rd_rng_off, *rd_val_off, *rd_r2v_off;
    uint32_t *rd_rng_start, *rd_rng_end, *rd_vals;
    int32_t *rd_r2v;
    // KeyDeps of range txns: counts / outputs (shared with the key-txn arrays)
    uint32_t *cnt_keys, *cnt_vals_k, *cnt_k2v;
    const uint32_t *kd_key_off, *kd_val_off, *kd_k2v_off;
    uint32_t *kd_keys, *kd_vals;
    int32_t *kd_k2v;
    DevStatus *status;
};
void launch_rangedeps_count(const RangeDepsParams &p, hipStream_t s);
void launch_rangedeps_fill(const RangeDepsParams &p, hipStream_t s);
// KeyDeps of range txns: checkpoints (needs the history of the batch), per-txn sizes, the body
// filled with dep txn indices, then per txn the sorted unique txnIds (into kd_vals at the txnIds
// upper-bound offsets) and the body rewritten to ranks.
constexpr uint32_t RK_CP_SHIFT = 12;
size_t rangekeys_cp_bytes(uint32_t ncp, uint32_t nkeys);
void launch_rangekeys_checkpoints(uint32_t PH, const uint32_t *sorted_key, const RangeDepsParams &p, hipStream_t s);
// carried range command kind no txn witnesses (witness masks use kinds 0..4): an ACCORD_ST_ERASED one
constexpr uint32_t RC_KIND_ERASED = 7;
// resident stores: the range commands a later batch can still see (owner >= thr), carried and this
// batch's, into the out arrays (a suffix of the candidate order); *kept = their number.  flags /
// offs (ncr + R + 1 words each, registered-status stores): also drop the erased ones (a flag scan).
void launch_range_carry(const RangeDepsParams &p, uint32_t R, uint32_t thr, uint32_t *out_owner, uint32_t *out_start,
                        uint32_t *out_end, uint32_t *out_kind, uint32_t *first_tmp, unsigned long long *kept,
                        uint32_t *flags, uint32_t *offs, void *scan_state, hipStream_t s);
// keys of every range txn's ranges (clipped to the store), for the stored-slice offsets
void launch_rangekeys_nkeys(const RangeDepsParams &p, uint32_t *cnt, hipStream_t s);
void launch_rangekeys_count(const RangeDepsParams &p, hipStream_t s);
void launch_rangekeys_fill(const RangeDepsParams &p, hipStream_t s);
constexpr uint32_t RK_CLASSES = 5;
inline size_t rangekeys_class_bytes(uint32_t nrt) { return ((size_t)RK_CLASSES * nrt * 4 + 8) * 4; }
void launch_rangekeys_union(const RangeDepsParams &p, hipStream_t s);

// ---- K6 merge (merge.hip) ----
struct MergeParams {
    uint32_t n;        // txns (aligned across parts)
    uint32_t G;        // parts
    uint32_t txn_lo;   // global stream position of txn 0
    const uint32_t *const *key_off;
    const uint32_t *const *keys;
    const uint32_t *const *val_off;
    const uint32_t *const *val_cnt;   // per part: gapped txnIds' counts, or nullptr (dense)
    const uint32_t *const *vals;
    const uint32_t *const *k2v_off;
    const int32_t *const *k2v;
    uint32_t *cnt_keys, *cnt_vals, *cnt_k2v;
    const uint32_t *out_key_off, *out_val_off, *out_k2v_off;
    uint32_t *out_keys, *out_vals;
    int32_t *out_k2v;
    DevStatus *status;
};
void launch_merge_count(const MergeParams &p, hipStream_t s);
void launch_merge_fill(const MergeParams &p, hipStream_t s);
// ---- exchange plan (merge.hip): the 6 CSR offset arrays of a partial (KeyDeps keys / txnIds /
// keysToTxnIds, RangeDeps ranges / txnIds / rangesToTxnIds) ----
constexpr int XCHG_NA = 6;
struct XchgOffsets {
    uint32_t *p[XCHG_NA];
};
// c[t] = #subset txns with global position < t (t in [0, n_total]) of a store holding a subset of
// the stream (txn_index); ind is scratch of n_total + 1 words
void launch_expand_index(uint32_t n, uint32_t n_total, const uint32_t *txn_index, uint32_t *ind, uint32_t *c,
                         void *scan_tmp, unsigned long long *total, hipStream_t s);
// out.p[a][t] = in.p[a][c[t]], t in [0, n_total]
void launch_expand_offsets(uint32_t n_total, const uint32_t *c, const XchgOffsets &in, const XchgOffsets &out,
                           hipStream_t s);
// counts[2*XCHG_NA*d + a] / [.. + XCHG_NA + a] = element count / first element of offset array a
// for destination d (txns [d*n_total/G, (d+1)*n_total/G)); counts[2*XCHG_NA*G] = 0 (status)
void launch_xchg_counts(uint32_t G, uint32_t n_total, const XchgOffsets &e, unsigned long long *counts, hipStream_t s);

// ---- SearchableRangeList stabbing of RangeDeps (rangeindex.hip) ----
constexpr uint32_t RI_C = 16;                  // ranges per checkpoint block
constexpr uint32_t RI_UMAX = 32768;            // RangeDeps txnIds of one txn the LDS bitmap holds
constexpr uint32_t RI_MAX_RANGES = 1u << 16;   // RangeDeps ranges of one txn the index covers
struct RangeIndexParams {
    uint32_t n;
    const uint32_t *rng_off, *rs, *re, *val_off, *vals, *r2v_off;
    const int32_t *r2v;
    uint32_t *chk_cnt;                         // [n] checkpoints per txn (scanned into chk_off)
    const uint32_t *chk_off;                   // [n + 1]
    uint32_t *list_cnt;                        // [nchk] list sizes (scanned into list_off)
    const uint32_t *list_off;                  // [nchk + 1]
    uint32_t *lists;
    uint32_t nq;
    const uint32_t *q_txn, *q_s, *q_e;         // queries (qs, qe] of txn q_txn
    uint32_t *out_cnt;
    const uint32_t *out_off;
    uint32_t *out;
    DevStatus *status;
};
void launch_ri_chk_count(const RangeIndexParams &p, hipStream_t s);
void launch_ri_lists(const RangeIndexParams &p, uint32_t nchk, bool fill, hipStream_t s);
void launch_ri_qtxn(uint32_t n, const uint32_t *q_off, uint32_t *q_txn, hipStream_t s);
void launch_ri_stab(const RangeIndexParams &p, bool fill, hipStream_t s);

// ---- deps-set operations: union / slice / invert (depset.hip) ----
// One side (KeyDeps: lo = key ordinals, hi unused; RangeDeps: ranges (lo, hi]) of G device deps
// sets, as device pointer tables indexed by part.  Offsets may start anywhere (element g of a
// data array is at index off[t] - off[0]).
struct DsSide {
    const uint32_t *const *key_off, *const *lo, *const *hi, *const *val_off, *const *vals, *const *x_off;
    const uint32_t *const *val_cnt;   // per part: gapped txnIds' counts, or nullptr (dense)
    const int32_t *const *x;
    uint32_t G;
    bool range;
};
struct DsUnionParams {
    uint32_t n;
    DsSide S;
    uint32_t *vlen, *klen, *blen;                   // per (txn, part)
    const uint32_t *veoff, *keoff, *beoff;          // element scratch offsets per (txn, part)
    uint32_t *vown, *vlst, *kown, *klst;            // owner prefixes / owners per list
    uint32_t *cnt_vals, *cnt_keys;                  // union sizes per txn
    const uint32_t *out_val_off, *out_key_off;
    uint32_t *vrank, *krank, *rb, *bown, *btot, *bsz;
    const uint32_t *bscan;                          // exclusive scan of bsz (union keys + 1)
    uint32_t *out_vals, *out_lo, *out_hi, *out_x_off;
    int32_t *out_x;
};
struct DsSliceParams {
    uint32_t n;
    DsSide S;                                       // G = 1
    const uint32_t *sel_off, *sel_start, *sel_end;  // device; sel_off null = nsel shared ranges
    uint32_t nsel;
    uint32_t *ksel, *mode, *cnt_keys, *cnt_vals, *cnt_x, *used, *remap;
    const uint32_t *out_key_off, *out_val_off, *out_x_off;
    uint32_t *out_lo, *out_hi, *out_vals;
    int32_t *out_x;
};
struct DsInvertParams {
    uint32_t n;
    DsSide S;                                       // G = 1
    uint32_t *sizes;                                // [n] per txn (launch_invert_sizes)
    uint32_t *out_off;                              // [n+1] = exclusive scan of sizes
    int32_t *out;                                   // zeroed before the launch
    uint32_t *cursor;                               // per txnId element
};
// union: lens -> (scan veoff/keoff/beoff) -> owners -> (scan union sizes) -> ranks + body owners +
// body sizes (bsz zeroed) -> (scan bsz) -> write
void launch_union_lens(const DsUnionParams &p, hipStream_t s);
void launch_union_owners(const DsUnionParams &p, hipStream_t s);
void launch_union_ranks(const DsUnionParams &p, hipStream_t s);
void launch_union_write(const DsUnionParams &p, hipStream_t s);
// slice: select + mark (used zeroed) + counts -> (scans) -> write
void launch_slice_select(const DsSliceParams &p, hipStream_t s);
void launch_slice_write(const DsSliceParams &p, hipStream_t s);
void launch_invert_sizes(const DsInvertParams &p, hipStream_t s);
void launch_invert(const DsInvertParams &p, hipStream_t s);

// ---- WaitingOn bitsets + execution levelling (waiting_on.hip) ----
struct WaitingOnParams {
    uint32_t n;
    const uint64_t *lsb;
    const uint32_t *key_off;                       // txn-major pairs (slice index)
    const PairSlice *slice;
    const uint32_t *hist, *pw_local, *pw_carry;
    uint32_t pw_tile;
    const uint32_t *kd_val_off, *kd_vals;          // full KeyDeps (non-reduced txns)
    const uint32_t *kd_val_cnt;                    // gapped txnIds: per-txn count (nullptr: dense)
    const uint32_t *rd_val_off, *rd_vals;          // RangeDeps txnIds
    uint32_t *pred_cnt;
    const uint32_t *pred_off;
    uint32_t *preds;
    uint8_t *pred_own;                             // fill: per predecessor, its txn's index mod 64 (or nullptr)
    uint32_t rw_only;                              // every history entry a Read or a Write (count pass: no entry reads)
};
void launch_wo_words_count(uint32_t n, const uint32_t *kd_key_off, const uint32_t *rd_val_off, uint32_t *cnt,
                           hipStream_t s);
void launch_wo_bits(uint32_t n, const uint32_t *kd_key_off, const uint32_t *rd_val_off, const uint32_t *wo_off,
                    unsigned long long *words, hipStream_t s);
void launch_wo_preds_count(const WaitingOnParams &p, hipStream_t s);
void launch_wo_preds_fill(const WaitingOnParams &p, hipStream_t s);
// level[i] for all i; info[0] = 1 + chunks resolved when a wave hit the defensive spin bound
// (must stay 0), info[1] = max level, info[2] = 1 if a predecessor does not precede its txn.
// info must be zeroed before the launch; temp holds levels_temp_bytes(n).
size_t levels_temp_bytes(uint32_t n);
void launch_levels(uint32_t n, const uint32_t *pred_off, const uint32_t *preds, uint32_t *level, uint32_t *info,
                   void *temp, hipStream_t s);
// The same levels by stripes of `stripe` txns (levels.hip): per-stripe max-plus walks with 63
// symbolic sources, the sources resolved in stripe order, relaxation to the fixpoint (at most
// `relax` sweeps).  info[3] = 1 when the sweeps did not reach the fixpoint: level[] is then a lower
// bound and the caller runs more sweeps (launch_levels_sweeps) or launch_levels.  info[1], info[2] as above; info zeroed by the caller.
uint32_t levels_stripe_default(uint32_t n);
size_t levels_striped_temp_bytes(uint32_t n, uint32_t stripe);
void launch_levels_striped(uint32_t n, const uint32_t *pred_off, const uint32_t *preds, const uint8_t *pred_own,
                           uint32_t *level, uint32_t *info, void *temp, uint32_t stripe, uint32_t relax, hipStream_t s);
// further sweeps [from, to) of the same levelling (the flags of sweeps < from stay), then info[1] / info[3]
void launch_levels_sweeps(uint32_t n, const uint32_t *pred_off, const uint32_t *preds, uint32_t *level,
                          uint32_t *info, void *temp, uint32_t stripe, uint32_t from, uint32_t to, hipStream_t s);

// ---- RedundantBefore.collectDeps (redundant.hip) ----
constexpr uint32_t RB_NONE = 0xFFFFFFFFu;   // shardAppliedOrInvalidatedBefore == Timestamp.NONE
constexpr uint32_t RB_MAX = 64;             // map entries one txn may touch
struct RbParams {
    uint32_t n;
    const uint64_t *msb, *exec_msb;                    // executeAt epoch (exec_msb null: txnId)
    const uint32_t *key_off, *key_ord, *rng_off, *rng_start, *rng_end;
    uint32_t m;                                        // map entries, (e_start, e_end] ascending, disjoint
    const uint32_t *e_start, *e_end, *e_bound;
    const uint64_t *e_start_epoch, *e_end_epoch;
    uint64_t min_epoch;
    uint32_t *cnt_rngs, *cnt_vals, *cnt_r2v;           // count pass
    const uint32_t *rng_off_out, *val_off_out, *r2v_off_out;
    uint32_t *out_start, *out_end, *out_vals;
    int32_t *out_r2v;
    DevStatus *status;
};
void launch_rb_count(const RbParams &p, hipStream_t s);
void launch_rb_fill(const RbParams &p, hipStream_t s);

} // namespace accord
