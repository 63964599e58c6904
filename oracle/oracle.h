/*
 * oracle.h -- CPU restatement of the reference (ifesdjeen/cassandra-accord, accord-core)
 * dependency-calculation hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is linked into, loaded by or called
 * from the product library (libaccord_deps.so) or its host mirror.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and only as the
 * checker / the timed CPU baseline.
 *
 * The reference is 100% Java and there is no JVM in this image, so it can
 * be neither compiled nor imported: oracle/_ref does not exist.  Parity of this restatement
 * is pinned by (1) restated reference property tests (KeyDepsTest canonical model,
 * SearchableRangeListTest brute force, RangeDepsTest) and (2) hand-derived known-answer
 * tests committed under tests/golden/ whose expected outputs cite the reference lines that
 * justify them (SURVEY.md §8c list of required KATs).  CFK mapReduceActive has no reference
 * test of its own (CommandsForKey.java:126 "TODO (required): randomised testing"), so for
 * that row parity rests on the restatement + KATs.
 *
 * Two restatements of the deps calculation are provided:
 *   - "literal": per-key CommandsForKey objects with sorted TxnInfo[] + committed[] rebuilt on
 *     every status change (CommandsForKey.java:422-470, 880-944), the linear mapReduceActive
 *     scan (:614-650), the linear range-command scan (InMemoryCommandStore.java:883-1016) and
 *     the RelationMultiMap.AbstractBuilder (RelationMultiMap.java:88-271).  This is the
 *     reference algorithm and is what bench.py times as the CPU baseline ("port").
 *   - "fast": the same function computed from per-key histories in O(deps) -- used to check
 *     the GPU at the full benchmark sizes; itself checked against "literal" in tests.
 */
#ifndef ACCORD_ORACLE_H
#define ACCORD_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* A seeded transaction stream, SoA, in TxnId order (SURVEY.md §8d "Synthetic stream").
 * Key txns carry sorted unique key ordinals in key_off/key_ord; range txns carry sorted,
 * de-overlapped (start,end] ranges in rng_off/rng_start/rng_end (IntKey semantics,
 * Range.EndInclusive: Range.java:40-88). */
typedef struct {
    uint32_t n;
    const uint64_t *msb;
    const uint64_t *lsb;
    const int32_t  *node;
    const uint32_t *key_off;    /* [n+1] */
    const uint32_t *key_ord;    /* [key_off[n]] */
    const uint32_t *rng_off;    /* [n+1] or NULL */
    const uint32_t *rng_start;  /* [rng_off[n]] */
    const uint32_t *rng_end;
    uint32_t window;            /* W of the status-at-time model */
    /* Accept batches (messages/Accept.java:113-117): per txn the startedBefore = executeAt
     * passed to PreAccept.calculatePartialDeps (p1 = txnId when executeAt != txnId).  NULL =
     * PreAccept (startedBefore = txnId).  executeAt must not precede its txnId. */
    const uint64_t *exec_msb;
    const uint64_t *exec_lsb;
    const int32_t  *exec_node;
    /* a resident store fed the stream batch by batch (include/accord_deps.h ACCORD_STORE_RESIDENT):
     * txn i only sees txns registered when its batch is computed, i.e. positions < batch_end[i].
     * Matters for Accept batches whose executeAt lies past their batch.  NULL = one batch. */
    const uint32_t *batch_end;
    /* fast restatement only: per txn the position below which txns are committed at executeAt =
     * txnId (replaces i - W; NULL = the window model).  A resident registered-status store whose
     * batches are COMMITTED (executeAt = TxnId) right after they are computed -- the schedule of
     * bench.py --registered -- has applied_before[i] = the first position of i's batch (COMMITTED
     * and APPLIED prune alike in mapReduceActive, local/CommandsForKey.java:634-645). */
    const uint32_t *applied_before;
    /* fast restatement only: per txn the shardRedundantBefore in force when its batch is computed,
     * as a position: CommandsForKey.withRedundantBefore (local/CommandsForKey.java:1654-1684) has
     * dropped every key entry below it (one bound for every key but key 0, which lies in no
     * (start, end] entry; range commands are not affected).
     * NULL = no truncation. */
    const uint32_t *floor;
} or_stream;

/* Per-txn PartialDeps in the exact reference layout (KeyDeps.java:150-187,
 * RangeDeps.java:81-99): for txn i,
 *   keys      = kd_keys[kd_key_off[i] .. kd_key_off[i+1])           (sorted unique ordinals)
 *   txnIds    = kd_vals[kd_val_off[i] .. kd_val_off[i+1])           (indices into the stream)
 *   keysToTxnIds = kd_k2v[kd_k2v_off[i] .. kd_k2v_off[i+1])         (exact int[] contents)
 * and likewise for RangeDeps with ranges (rd_rng_start/rd_rng_end). */
typedef struct {
    uint32_t n;
    uint32_t *kd_key_off, *kd_keys, *kd_val_off, *kd_vals, *kd_k2v_off;
    int32_t  *kd_k2v;
    uint32_t *rd_rng_off, *rd_rng_start, *rd_rng_end, *rd_val_off, *rd_vals, *rd_r2v_off;
    int32_t  *rd_r2v;
} or_deps;

int  or_stream_deps_literal(const or_stream *s, or_deps *out);
int  or_stream_deps_fast(const or_stream *s, or_deps *out);
/* literal model restricted to the first `limit` txns (CPU-baseline sample) */
int  or_stream_deps_literal_prefix(const or_stream *s, uint32_t limit, or_deps *out);
void or_deps_free(or_deps *d);

/* ---- stateful literal CommandStore (resident store + status events, key txns only) ---- */
typedef struct or_lstore or_lstore;
or_lstore *or_lstore_create(uint32_t nkeys);
void       or_lstore_free(or_lstore *s);
/* one batch in TxnId order after everything the store holds; values are global positions */
int        or_lstore_batch(or_lstore *s, const or_stream *b, or_deps *out);
/* InternalStatus events (0 TRANSITIVELY_KNOWN .. 7 INVALID_OR_TRUNCATED) for known txns */
int        or_lstore_register(or_lstore *s, uint32_t n, const uint64_t *msb, const uint64_t *lsb, const int32_t *node,
                              const uint8_t *status, const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode);
uint32_t   or_lstore_size(const or_lstore *s);
/* CommandsForKey.withRedundantBefore (local/CommandsForKey.java:1654-1684) on every key: the map's
 * m entries (start, end] ascending and disjoint, bound = shardRedundantBefore as a position
 * (0xFFFFFFFF = NONE); each key's txns below its entry's bound leave its CommandsForKey.  Later
 * status events for a dropped txn no longer reach that key. */
int        or_lstore_truncate(or_lstore *s, uint32_t m, const uint32_t *start, const uint32_t *end,
                              const uint32_t *bound);
/* Execution readiness (see oracle.c): the n txns at positions base.. join the
 * waiting set with their deps d (values = positions, as or_lstore_batch returns them) and every
 * WaitingOn bit set; or_lstore_ready re-evaluates every waiting txn against the current state and
 * returns (ascending) the txns that became ReadyToExecute -- no bit left, status STABLE -- which
 * leave the set. */
int        or_lstore_waiting_add(or_lstore *s, uint32_t base, const or_deps *d, uint32_t n);
int        or_lstore_ready(or_lstore *s, uint32_t *ready_out, uint32_t *nready);
/* as or_lstore_ready, plus each ready txn's Command.executesAtLeast (executeAtLeast for awaitsOnlyDeps
 * kinds when set, else executeAt) */
int        or_lstore_ready_ex(or_lstore *s, uint32_t *ready_out, uint32_t *nready, uint64_t *eal_msb, uint64_t *eal_lsb,
                              int32_t *eal_node);
/* event mode (default off): key bits are cleared only when CommandsForKey.notifyAndUpdatePending
 * (local/CommandsForKey.java:1163-1215) would evaluate them -- notify over committed[] between next /
 * nextWrite per the event's status (COMMITTED before nextWrite notifies nobody), notifyUnmanaged COMMIT
 * on a txn committing, APPLY while minUncommitted is null or next is not; events are the register calls
 * (one txn at a time, array order), a waiter's own STABLE transition (replayed at waiting_add when it is
 * Stable already) and truncations (APPLY only).  Range-dep bits follow their deps' statuses as before. */
void       or_lstore_event_mode(or_lstore *s, int on);
/* the RedundantBefore map readiness reads (removeRedundantDependencies, local/CommandStore.java:601-678):
 * m entries (start, end] ascending and disjoint, [sep, eep), locallyAppliedOrInvalidatedBefore and
 * bootstrappedAt as positions (0xFFFFFFFF = TxnId.NONE), stale = staleUntilAtLeast != null; m = 0 clears */
int        or_lstore_redundant(or_lstore *s, uint32_t m, const uint32_t *start, const uint32_t *end, const uint64_t *sep,
                               const uint64_t *eep, const uint32_t *local, const uint32_t *boot, const uint8_t *stale);
uint32_t   or_lstore_waiting(const or_lstore *s);

/* ---- primitives restated for the reference's own property tests ---- */

/* Timestamp.compareTo (Timestamp.java:208-217) */
int or_ts_compare(uint64_t amsb, uint64_t alsb, int32_t anode, uint64_t bmsb, uint64_t blsb, int32_t bnode);
/* Timestamp.equals (Timestamp.java:244-249) */
int or_ts_equals(uint64_t amsb, uint64_t alsb, int32_t anode, uint64_t bmsb, uint64_t blsb, int32_t bnode);

/* KeyDeps.Builder (RelationMultiMap.AbstractBuilder) fed with `nadds` (key, value) adds in
 * the given order; values are indices into a TxnId table (tbl_*).  Output is one KeyDeps in
 * kd_* fields of `out` (n = 1).  Returns 0, or -1 if the builder throws
 * ("Key ... has been visited more than once", RelationMultiMap.java:236-238). */
int or_keydeps_build(uint32_t nadds, const uint32_t *keys, const uint32_t *vals,
                     uint32_t ntbl, const uint64_t *tbl_msb, const uint64_t *tbl_lsb, const int32_t *tbl_node,
                     or_deps *out);

/* RelationMultiMap.linearUnion for KeyDeps (RelationMultiMap.java:561-816) of txn a of `x`
 * and txn b of `y` (values are indices into the same table, compared via the table). */
int or_keydeps_union(const or_deps *x, uint32_t a, const or_deps *y, uint32_t b,
                     const uint64_t *tbl_msb, const uint64_t *tbl_lsb, const int32_t *tbl_node,
                     or_deps *out);

/* SearchableRangeList brute-force stabbing oracle (SearchableRangeListTest.java:61-115):
 * ranges sorted by (start,end); writes the indices of the ranges containing `key`
 * ((s,e] semantics) in ascending index order; returns the count. */
uint32_t or_stab_key(uint32_t nr, const uint32_t *rs, const uint32_t *re, uint32_t key, uint32_t *out);

/* WaitingOn levelling over the deps of a stream whose executeAt ==
 * txnId and none applied: level[i] = 0 if no dep executes before i, else 1 + max level(dep).
 * Also writes the WaitingOn bitset words (Command.java:1426-1437: range-dep txn bits then
 * keyDeps key bits) into wo_words at wo_off[i] (in 64-bit words). */
int or_waiting_on(const or_deps *d, uint32_t n, uint32_t *level,
                  uint32_t *wo_off /* [n+1] */, uint64_t **wo_words /* malloc'd */);

/* Levelling alone over a predecessor CSR in txn order (every pred p of i has p < i): level[i] = 0
 * without preds, else 1 + max level(p).  The CPU baseline of the device levelling of config 5's
 * reduced DAG (bench.py --config 5); returns -1 when a pred does not precede its txn. */
int or_levels_csr(uint32_t n, const uint32_t *pred_off, const uint32_t *preds, uint32_t *level);

/* Commands.initialiseWaitingOn (local/Commands.java:735-753) with its initial updateWaitingOn
 * (:755-830; WaitingOn.Update, local/Command.java:1403-1600) for the n txns of one batch of a
 * registered-status store: deps d hold global positions; status/emsb/elsb/enode give every
 * position's InternalStatus ordinal (CommandsForKey.java:194-203; 8 = SaveStatus Erased) and
 * executeAt at the moment the WaitingOn is built; own_* is each txn's own executeAt.
 *   bits [0, R)     RangeDeps txnIds, set; then each dep that hasBeen(PreCommitted) (>= COMMITTED):
 *                   truncated / invalidated (>= INVALID_OR_TRUNCATED) -> setAppliedOrInvalidated;
 *                   else executeAt > own executeAt (own kind not awaitsOnlyDeps) -> removeWaitingOn;
 *                   else APPLIED -> setAppliedAndPropagate (the dep's own appliedOrInvalidated
 *                   taken as empty); else still waiting
 *   bits [R, R+K)   KeyDeps keys, set (initialiseWaiting; CommandsForKey.notify clears them later)
 *   aoi_words       appliedOrInvalidated (same word layout; Range-domain txns only, null for keys)
 * Words and aoi are malloc'd.  0 ok. */
int or_initialise_waiting_on(const or_deps *d, uint32_t n, const uint64_t *lsb, const uint64_t *own_msb,
                             const uint64_t *own_lsb, const int32_t *own_node, const uint8_t *status,
                             const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                             uint32_t *wo_off /* [n+1] */, uint64_t **wo_words, uint64_t **aoi_words);

/* Event-driven readiness simulation (bits cleared by applies, CFK notify per key); round[i] is the
 * synchronous round in which txn i executes.  Must equal or_waiting_on's level.  0 ok, -7 stuck. */
int or_waiting_on_events(const or_deps *d, uint32_t n, uint32_t *round_out);
/* The same rounds restated from the CommandsForKey side: per-key CFK notify with the missing[]
 * counts for managed txns, registerUnmanaged/notifyUnmanaged for range and EphemeralRead txns, and
 * range-dep bits cleared on apply.  Uses the stream's keys/kinds; deps only for the WaitingOn bits,
 * the unmanaged waitingUntil bounds and range deps.  0 ok, -7 stuck. */
int or_levels_cfk(const or_stream *s, const or_deps *d, uint32_t *round_out);

/* ---- deps-set operations over every txn of a set; values index one
 * TxnId table sorted ascending (index order == Timestamp order) ---- */
/* Deps.merge / linearUnion of G sets of the same n txns (KeyDeps + RangeDeps; keys may overlap) */
int or_deps_union(uint32_t G, const or_deps *parts, or_deps *out);
/* The node-level deps of a stream over the S CommandStores of one node (SURVEY.md §7 "Hard parts"
 * 5): store j owns the IntKey range (bounds[j]-1, bounds[j+1]-1] (bounds[0] == 0 open below,
 * bounds[S] == 0xFFFFFFFF open above); each store computes the PartialDeps of every txn over its
 * keys and its Minimal slices of every range (InMemoryCommandStore.java:757-760, 886;
 * AbstractRanges.sliceMinimal :339-377) -- literal (1) or fast (0) restatement -- and the result
 * is their union (PreAccept.reduce, messages/PreAccept.java:140-156). */
int or_stream_deps_stores(const or_stream *s, uint32_t nstores, const uint32_t *bounds, int literal, or_deps *out);
/* RedundantBefore.collectDeps of every txn of the stream (local/RedundantBefore.java:181-190,
 * 418-421; ReducingRangeMap.foldl, inclusiveEnds): m entries (es, ee] ascending and disjoint with
 * [sep, eep) epochs and bound stream positions (0xFFFFFFFF = NONE); min_epoch = minUnsyncedEpoch.
 * The redundant PartialDeps (RangeDeps only); PreAccept returns or_deps_union(deps, it). */
int or_redundant_collect(const or_stream *s, uint32_t m, const uint32_t *es, const uint32_t *ee, const uint64_t *sep,
                         const uint64_t *eep, const uint32_t *bound, uint64_t min_epoch, or_deps *out);
/* KeyDeps.slice + RangeDeps.slice (+ trimUnusedValues) to select ranges (s,e]: per txn
 * sel_off[n+1] CSR, or sel_off NULL = the same nsel ranges for every txn */
int or_deps_slice(const or_deps *d, const uint32_t *sel_off, const uint32_t *sel_start, const uint32_t *sel_end,
                  uint32_t nsel, or_deps *out);
/* RelationMultiMap.invert of keysToTxnIds (range 0) / rangesToTxnIds (range 1) of every txn */
int or_deps_invert(const or_deps *d, int range, uint32_t *off /* [n+1] */, int32_t **out /* malloc'd */);

/* ---- stream segments (multi-GPU ownership by TxnId range) ----
 * or_cfk_reachable: per key, the CommandsForKey entries of txns [lo, hi) that a txn at position
 * >= thr + W can still reach under the status-at-time model -- the run from the last Write with
 * position < thr on, or the key's whole run when it has none (mapReduceActive's maxCommittedBefore
 * bound, local/CommandsForKey.java:620-645).  Key-domain txns' entries (EphemeralReads included, as
 * the device history keeps them; no kind witnesses them).  Key-major, positions ascending:
 * key[] absolute ordinals, ent[] = kind << 29 | position.  A segment's summary is
 * or_cfk_reachable(s, a, b, b - W); the CommandsForKey state at the start of segment r is
 * or_cfk_reachable(s, 0, a_r, a_r - W).
 * or_cfk_fold: that state from the summaries of segments 0..r-1 (stream order) with thr = a_r - W.
 * Outputs malloc'd (or_free). */
int or_cfk_reachable(const or_stream *s, uint32_t lo, uint32_t hi, uint32_t thr, uint32_t *n_out,
                     uint32_t **key, uint32_t **ent);
int or_cfk_fold(uint32_t nparts, const uint32_t *part_n, const uint32_t *const *keys, const uint32_t *const *ents,
                uint32_t thr, uint32_t *n_out, uint32_t **key, uint32_t **ent);
void or_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
