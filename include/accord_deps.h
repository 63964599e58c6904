/*
 * accord_deps.h -- C ABI of the MI355X-native Accord dependency-calculation path.
 *
 * This is the drop-in boundary for ONE hot path of ifesdjeen/cassandra-accord (accord-core):
 * the replica-side deps calculation behind SafeCommandStore.mapReduceActive
 * (local/SafeCommandStore.java:274) as driven by PreAccept.calculatePartialDeps
 * (messages/PreAccept.java:245-265), producing KeyDeps/RangeDeps in their exact serialised
 * layout (KeyDeps.SerializerSupport.create, primitives/KeyDeps.java:69-72;
 * RangeDeps.SerializerSupport.create, primitives/RangeDeps.java:69-72).
 *
 * Conventions (mirroring the reference, see INTEGRATION.md for the Panama FFM binding):
 *  - one accord_store handle == one CommandStore == one HIP stream.  Handles are not
 *    thread-safe; different handles may be used concurrently (the reference's one thread per
 *    store: impl/InMemoryCommandStore.java:1131-1158).
 *  - every call returns an int32 status; nonzero maps to IllegalStateException /
 *    IllegalArgumentException on the Java side (utils/Invariants.java:43-60), with the message
 *    from accord_last_error().
 *  - TxnIds are exchanged as SoA (msb, lsb, node) exactly as the Java fields
 *    (primitives/Timestamp.java:77-79); Java re-materialises them with TxnId.fromBits
 *    (primitives/TxnId.java:37-40).  Deps values are u32 indices into the batch's TxnId table.
 *  - keys are u32 ordinals of the store's sorted key dictionary (ordinal order ==
 *    Key.compareTo order); ranges are (start, end] ordinal pairs (Range.EndInclusive,
 *    primitives/Range.java:40-88).
 *  - input buffers are borrowed for the duration of a call; outputs are owned by the
 *    library until accord_deps_release().
 *  - there is no CPU fallback: without a usable HIP device every compute call fails with
 *    ACCORD_ERR_HIP.
 */
#ifndef ACCORD_DEPS_H
#define ACCORD_DEPS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACCORD_OK               0
#define ACCORD_ERR_ARG         -1   /* bad argument */
#define ACCORD_ERR_UNSORTED    -2   /* batch TxnIds not strictly ascending (Timestamp.compareTo) */
#define ACCORD_ERR_KIND        -3   /* a txn kind whose witnesses() throws (LocalOnly, bad ordinal) */
#define ACCORD_ERR_KEYS        -4   /* keys not sorted-unique, or outside the store's key range */
#define ACCORD_ERR_DOMAIN      -5   /* domain bit inconsistent with keys/ranges payload */
#define ACCORD_ERR_RANGES      -6   /* ranges not sorted / de-overlapped / empty */
#define ACCORD_ERR_CAPACITY    -7   /* a size limit of this build was exceeded */
#define ACCORD_ERR_HIP         -8   /* HIP runtime error / no device */
#define ACCORD_ERR_OOM         -9   /* host or device allocation failed */
#define ACCORD_ERR_STATE      -10   /* call out of sequence */

/* Version of this ABI: raised on every change of a struct layout or of a result's form that a
 * binding must follow.  6: KeyDeps txnIds of compute results are gapped (accord_deps.kd_val_cnt,
 * round 5); stream segments (accord_segment_*).  A binding compares accord_abi_version() with the
 * value it was written against and refuses to run on a mismatch. */
#define ACCORD_ABI_VERSION 6u
uint32_t accord_abi_version(void);

#define ACCORD_STORE_PROFILE   1u   /* record HIP events around every kernel */
/* The store keeps its CommandsForKey state across batches (CommandStore semantics: every batch
 * continues the store's stream; see accord_store_resident below).  Without it every uploaded
 * batch is a stream of its own. */
#define ACCORD_STORE_RESIDENT  2u

typedef struct accord_store accord_store;

typedef struct {
    int32_t  device;        /* HIP device ordinal */
    uint32_t key_lo;        /* store owns key ordinals [key_lo, key_hi) (CommandStores slice) */
    uint32_t key_hi;
    uint32_t window;        /* W of the status-at-time model; ACCORD_WINDOW_NONE: none
                               (statuses from accord_txn_register, resident stores) */
    uint32_t flags;         /* ACCORD_STORE_PROFILE | ACCORD_STORE_RESIDENT */
    /* The CommandStores this handle hosts, as nstores + 1 ascending key-ordinal bounds: store j owns
     * ordinals [store_bounds[j], store_bounds[j+1]), i.e. the IntKey range
     * (store_bounds[j] - 1, store_bounds[j+1] - 1]; store_bounds[0] == 0 is open below and
     * store_bounds[nstores] == ACCORD_KEY_END open above.  Every range of an uploaded batch is
     * sliced Minimal to these stores -- the range command each store registers
     * (InMemoryCommandStore.update, impl/InMemoryCommandStore.java:757-760: ranges.slice(storeRanges,
     * Minimal)) and the query it answers (mapReduceRangesInternal :886) -- so a range spanning
     * stores yields one RangeDeps entry per store slice (primitives/RangeDeps.java:462-465) and the
     * handle's result is the union of its stores' PartialDeps (PreAccept.reduce,
     * messages/PreAccept.java:140-156); pieces outside every store are dropped.  [key_lo, key_hi)
     * must lie inside the stores.  nstores = 0 (store_bounds NULL): one store over the whole key
     * domain, ranges unsliced. */
    uint32_t nstores;
    const uint32_t *store_bounds;   /* [nstores + 1], borrowed for the call */
} accord_store_cfg;

#define ACCORD_KEY_END 0xFFFFFFFFu   /* an open upper store bound */

/* A batch of transactions in TxnId order (the PreAccept stream of SURVEY.md §8d).  Key txns
 * (TxnId domain bit 0) carry sorted unique key ordinals; range txns (domain bit 1) carry sorted,
 * de-overlapped (start, end] ranges (AbstractRanges.sortAndDeoverlap, MERGE_OVERLAPPING).
 * Pointers are host pointers unless a call says otherwise. */
typedef struct {
    uint32_t        n;
    const uint64_t *msb;        /* [n] Timestamp.msb */
    const uint64_t *lsb;        /* [n] Timestamp.lsb (hlc low bits << 16 | flags) */
    const int32_t  *node;       /* [n] Node.Id.id */
    const uint32_t *key_off;    /* [n+1] CSR into key_ord */
    const uint32_t *key_ord;    /* [key_off[n]] */
    const uint32_t *rng_off;    /* [n+1] CSR into rng_start/rng_end, or NULL (no range txns) */
    const uint32_t *rng_start;
    const uint32_t *rng_end;
    /* [n] global stream position of each txn, strictly ascending, or NULL (= 0..n-1).  A store
     * that receives only the txns intersecting its keys (CommandStores.mapReduce,
     * local/CommandStores.java:575-592) passes their positions so the status-at-time window and
     * the deps values (txnIds) stay in global stream coordinates.  Key txns only. */
    const uint32_t *txn_index;
    /* Accept batches (Accept.calculatePartialDeps, messages/Accept.java:113-117): [n] the
     * executeAt of each txn (a Timestamp: msb, lsb, node), passed as startedBefore to
     * mapReduceActive, with p1 = txnId excluded unless executeAt.equals(txnId)
     * (messages/PreAccept.java:253-259).  Every txn of the batch started before a txn's executeAt
     * is registered when it computes (PREACCEPTED inside the window, as SURVEY.md §8d).  All three
     * NULL = a PreAccept batch (startedBefore = txnId).  executeAt < txnId -> ACCORD_ERR_ARG. */
    const uint64_t *exec_msb;
    const uint64_t *exec_lsb;
    const int32_t  *exec_node;
} accord_batch;

/* Per-txn PartialDeps, exact reference layout (KeyDeps.java:150-187, RangeDeps.java:81-99):
 * for txn i
 *   KeyDeps.keys         = kd_keys[kd_key_off[i] .. kd_key_off[i+1])
 *   KeyDeps.txnIds       = batch txns kd_vals[kd_val_off[i] .. kd_val_off[i] + kd_val_cnt[i])  (TxnId order)
 *                          (kd_val_cnt == NULL: kd_vals[kd_val_off[i] .. kd_val_off[i+1]), dense)
 *   KeyDeps.keysToTxnIds = kd_k2v[kd_k2v_off[i] .. kd_k2v_off[i+1])   (the int[] verbatim)
 * and the same for RangeDeps (ranges as (rd_rng_start, rd_rng_end] pairs, always dense).
 * The txnIds of a compute result (accord_deps_compute / _batch / _download) are gapped: each txn's
 * list starts at an upper bound of the lists before it (the union of its keys' witnessed entries is
 * only known once built) and kd_val_cnt gives its length -- the reader (KeyDeps.SerializerSupport
 * .create per txn) takes each txn's txnIds by (start, count) and never sees the gaps.
 * kd_vals_total is the length of the kd_vals array (= kd_val_off[n]); the deps-set operations
 * (union, slice, invert, merge, exchange, waiting-on) accept either form and produce dense sets. */
typedef struct {
    uint32_t  n;
    uint32_t  reserved;
    uint64_t  kd_keys_total, kd_vals_total, kd_k2v_total;
    uint64_t  rd_rngs_total, rd_vals_total, rd_r2v_total;
    uint32_t *kd_key_off, *kd_keys, *kd_val_off, *kd_vals, *kd_k2v_off;
    int32_t  *kd_k2v;
    uint32_t *rd_rng_off, *rd_rng_start, *rd_rng_end, *rd_val_off, *rd_vals, *rd_r2v_off;
    int32_t  *rd_r2v;
    uint32_t *kd_val_cnt;       /* [n] KeyDeps.txnIds length per txn, or NULL (dense, see above) */
    void     *owner;            /* library-private */
} accord_deps;

/* Per-stage device time of the last accord_deps_compute (ms, HIP events on the store's
 * stream; zero unless the store was created with ACCORD_STORE_PROFILE). */
typedef struct {
    float validate_ms, sort_ms, segment_ms, count_ms, scan_ms, fill_ms, range_ms, total_ms;
    float compact_ms, reserved_ms;   /* txnIds compaction (gapped -> dense CSR) */
    uint64_t pairs, hist_entries;
    /* the count stage by kernel: range txns' key checkpoints, their key counts (+ offsets scan),
     * key txns' sizes, range txns' KeyDeps counts, RangeDeps counts */
    float count_rk_cp_ms, count_rk_nkeys_ms, count_kd_sizes_ms, count_rk_ms, count_rd_ms, reserved2_ms;
    /* every decoupled look-back scan of the compute: spin iterations spent waiting on a predecessor
     * tile's status, and look-backs that gave up waiting and summed the inputs themselves */
    uint64_t scan_spins, scan_fallbacks;
} accord_timing;

/* ---- store lifecycle (CommandStore; impl/InMemoryCommandStore.java:89) ---- */
int32_t     accord_store_create(const accord_store_cfg *cfg, accord_store **out);
int32_t     accord_store_destroy(accord_store *store);
const char *accord_last_error(const accord_store *store);   /* NULL store: last global error */
void       *accord_store_stream(accord_store *store);        /* the store's hipStream_t */

/* ---- resident CommandsForKey state (ACCORD_STORE_RESIDENT) ----
 * A resident store is one CommandStore over its whole life: batch b continues the stream of
 * batches 0..b-1 (its first TxnId must follow the last one registered, ACCORD_ERR_UNSORTED
 * otherwise), every txn keeps its global stream position (txn_index given, or next_global + t),
 * and deps values are global positions -- the output of b consecutive batches is the output of
 * one batch over their concatenation.  Between batches the store keeps, per key, the history
 * entries a later txn can reach (CommandsForKey.txns from the last Write before the window on;
 * older entries are pruned for good, as committed entries below maxCommittedBefore are,
 * local/CommandsForKey.java:620-645,1654-1684).  A rejected batch leaves the state unchanged.
 * Range txns: the store also keeps the range commands a later txn's window can reach (owner
 * position >= next_global - W; the range-command scan of impl/InMemoryCommandStore.java:883-1016
 * over the commands still live), so RangeDeps and the range txns' KeyDeps continue across batches
 * too.  In a registered-status store (ACCORD_WINDOW_NONE) every range command stays until an event
 * gives it ACCORD_ST_ERASED, and a range txn's KeyDeps run the full mapReduceActive filter on the
 * keys of its ranges. */
/* Real status events (SURVEY.md §8b accord_txn_register): a resident store created with window
 * ACCORD_WINDOW_NONE has no status-at-time model -- every txn enters its keys' CommandsForKey
 * PREACCEPTED when its batch is computed (CommandsForKey.insert, local/CommandsForKey.java:880-944)
 * and keeps that status until an event changes it: CommandsForKey.update(prev, next) with the new
 * InternalStatus and executeAt (:652-706; ordinals below, :194-203).  mapReduceActive then runs in
 * full (:614-650): maxCommittedBefore over the COMMITTED/STABLE/APPLIED Writes' executeAt, the
 * prune of committed entries below it, TRANSITIVELY_KNOWN / INVALID_OR_TRUNCATED never emitted.
 * Events name txns the store holds by TxnId (strictly ascending within a call); statuses never go
 * back and a committed executeAt never changes (ACCORD_ERR_STATE; the checkState of :674-690); an
 * event for ACCEPTED..APPLIED carries an executeAt >= TxnId.  A rejected call applies nothing.
 * An entry leaves the resident state when its txn becomes INVALID_OR_TRUNCATED (CommandsForKey drops
 * truncated txns, :1654-1684). */
#define ACCORD_WINDOW_NONE          0xFFFFFFFFu
#define ACCORD_ST_TRANSITIVELY_KNOWN 0
#define ACCORD_ST_HISTORICAL         1
#define ACCORD_ST_PREACCEPTED        2
#define ACCORD_ST_ACCEPTED           3
#define ACCORD_ST_COMMITTED          4
#define ACCORD_ST_STABLE             5
#define ACCORD_ST_APPLIED            6
#define ACCORD_ST_INVALID_OR_TRUNCATED 7
/* SaveStatus Erased / Invalidated (local/SaveStatus.java:86-87): INVALID_OR_TRUNCATED for
 * CommandsForKey, and a range command with it leaves the range-command scan (SaveStatus >= Erased,
 * impl/InMemoryCommandStore.java:891).  A range command at INVALID_OR_TRUNCATED (ErasedOrInvalidated,
 * Truncated*: before Erased in SaveStatus order, :80-85) is still visited. */
#define ACCORD_ST_ERASED             8
/* SaveStatus TruncatedApply / TruncatedApplyWithOutcome / TruncatedApplyWithDeps (local/SaveStatus.java:
 * 79-81): INVALID_OR_TRUNCATED for CommandsForKey (InternalStatus.convert, local/CommandsForKey.java:
 * 222-224) and still visited by the range-command scan (before Erased), but its executeAt is known
 * (ExecuteAtKnown) and the event carries it: Commands.updateWaitingOn feeds it to an awaitsOnlyDeps
 * waiter's updateExecuteAtLeast before taking the truncation branch (local/Commands.java:782-783), and
 * checks executeAt < the waiter's executeAt for every other waiter (:789-791; a violation fails
 * accord_waiting_on_initialise / accord_ready_update with ACCORD_ERR_STATE).  Statuses advance in
 * SaveStatus order: ... APPLIED < TRUNCATED_APPLY < INVALID_OR_TRUNCATED < ERASED. */
#define ACCORD_ST_TRUNCATED_APPLY    9
int32_t accord_txn_register(accord_store *store, uint32_t n, const uint64_t *msb, const uint64_t *lsb,
                            const int32_t *node, const uint8_t *status, const uint64_t *exec_msb,
                            const uint64_t *exec_lsb, const int32_t *exec_node);

typedef struct {
    uint64_t next_global;       /* global position of the next txn */
    uint64_t carry_entries;     /* history entries kept for later batches */
    uint64_t txns_registered;   /* == next_global unless batches carried txn_index gaps */
    uint64_t reserved;
} accord_store_state_info;
int32_t accord_store_state(accord_store *store, accord_store_state_info *info);
int32_t accord_store_reset(accord_store *store);               /* back to an empty CommandStore */

/* ---- RedundantBefore.collectDeps (local/RedundantBefore.java:181-190, 418-421) ----
 * PreAccept.calculatePartialDeps returns builder.build().with(redundant) (messages/PreAccept.java:
 * 260-263), where `redundant` holds (entry.range, shardAppliedOrInvalidatedBefore) for every entry of
 * the store's RedundantBefore map the txn's keys / ranges touch (ReducingRangeMap.foldl,
 * utils/ReducingRangeMap.java:111-194: each entry once) unless Entry.outOfBounds(minEpoch, executeAt)
 * (executeAt.epoch() < startEpoch || minEpoch >= endEpoch, :260-263) or the bound is NONE.
 * The map is given as its m non-null entries: (start, end] ascending and disjoint, [start_epoch,
 * end_epoch), and shardAppliedOrInvalidatedBefore as the GLOBAL STREAM POSITION of that TxnId in
 * this store (ACCORD_NO_TXN = Timestamp.NONE).  The bound TxnIds are sync points the store has
 * processed itself, so TxnId order is position order and deps values keep one value space.
 * min_epoch = the message's minUnsyncedEpoch (EpochSupplier.constant, messages/PreAccept.java:103).
 * Every later accord_deps_compute / accord_deps_batch returns the union; m = 0 clears the map
 * (RedundantBefore.EMPTY).  A txn touching more than 64 entries is ACCORD_ERR_CAPACITY; entries
 * not ascending / disjoint or empty are ACCORD_ERR_RANGES. */
#define ACCORD_NO_TXN 0xFFFFFFFFu
int32_t accord_redundant_before_set(accord_store *store, uint32_t m, const uint32_t *start, const uint32_t *end,
                                    const uint64_t *start_epoch, const uint64_t *end_epoch, const uint32_t *bound,
                                    uint64_t min_epoch);
/* The same map with the rest of each Entry (local/RedundantBefore.java:63-110):
 * locallyAppliedOrInvalidatedBefore and bootstrappedAt as stream positions of this store
 * (ACCORD_NO_TXN = TxnId.NONE; a TxnId the stream does not hold is given as the first position whose
 * TxnId follows it -- the comparisons below only ask which positions precede it), and
 * staleUntilAtLeast != null as stale[e] = 1 (NULL arrays: NONE, NONE, not stale -- accord_redundant_
 * before_set).  The entries are the map's values as the reference holds them (Entry.merge has already
 * cleared a locallyAppliedOrInvalidatedBefore at or below bootstrappedAt).  Readiness (accord_waiting_on_
 * initialise, accord_ready_update) then applies Commands.updateWaitingOn's removal step
 * (local/Commands.java:755-761): when CommandStore.hasLocallyRedundantDependencies(minWaitingOnTxnId,
 * executeAt, participants) holds (RedundantBefore.status >= PARTIALLY_PRE_BOOTSTRAP_OR_STALE,
 * local/CommandStore.java:672-678), CommandStore.removeRedundantDependencies (:601-670) stops waiting on
 * the range deps in [bootstrappedAt, locallyAppliedOrInvalidatedBefore) of every entry their ranges
 * meet, and on those before bootstrappedAt whose ranges the bootstrapping entries cover completely
 * (RangeState.isFullyBootstrapping).  No size limit: a waiting txn with more than 4096 RangeDeps
 * txnIds, or whose participants touch more than 64 entries, is evaluated by a second pass with its
 * scratch in HBM instead of LDS. */
int32_t accord_redundant_before_set_ex(accord_store *store, uint32_t m, const uint32_t *start, const uint32_t *end,
                                       const uint64_t *start_epoch, const uint64_t *end_epoch, const uint32_t *shard_bound,
                                       const uint32_t *locally_applied_before, const uint32_t *bootstrapped_at,
                                       const uint8_t *stale, uint64_t min_epoch);

/* ---- synchronous batch entry: host in, host out ----
 * CommandStore.calculateDepsBatch(TxnId[], Seekables[], Timestamp[] executeAt, ...) ->
 * PartialDeps[]: identical to calling PreAccept.calculatePartialDeps (messages/PreAccept.java:
 * 245-265; via Accept.calculatePartialDeps, messages/Accept.java:113-117, when the batch carries
 * executeAt) for every txn in TxnId order under the status-at-time model with window cfg.window. */
int32_t accord_deps_batch(accord_store *store, const accord_batch *batch, accord_deps *out);
void    accord_deps_release(accord_deps *deps);

/* SafeCommandStore.mapReduceActive for ONE txn of a host deps set (accord_deps_download /
 * accord_deps_batch output): replays the visitor in the contract order of
 * local/SafeCommandStore.java:269-273 -- keys first, then ranges, both ascending; within each, the
 * txnIds ascending -- as fn(ctx, is_range, key or range start, range end, txn value).  The
 * reference's CommandFunction.apply(p1, keyOrRange, txnId, executeAt, in) (:58-61) feeding
 * Deps.AbstractBuilder.add rebuilds exactly this txn's PartialDeps.  A nonzero return from fn stops
 * the visit and is returned.  Host-only (no device work). */
typedef int32_t (*accord_visit_fn)(void *ctx, uint32_t is_range, uint32_t key_or_start, uint32_t range_end,
                                   uint32_t txn_value);
int32_t accord_deps_visit(const accord_deps *deps, uint32_t txn, accord_visit_fn fn, void *ctx);

/* ---- device-resident pipeline (inputs already in HBM; used by the bench) ---- */
/* H2D.  The host arrays are consumed before it returns (a batch of <= 8 MiB is staged in page-locked
 * memory and its copy left running on the store's stream, ordered before the compute; a larger one is
 * copied and waited for); a failure of the copy itself is reported by the next call on the store. */
int32_t accord_batch_upload(accord_store *store, const accord_batch *host_batch);
int32_t accord_deps_compute(accord_store *store);          /* enqueue + run the whole pipeline */
int32_t accord_deps_device_view(accord_store *store, accord_deps *dev);  /* device pointers */
int32_t accord_deps_download(accord_store *store, accord_deps *out);     /* D2H copy, host-owned */
int32_t accord_store_timing(accord_store *store, accord_timing *t);
/* profiling events on (1) or off (0) from the next call on -- ACCORD_STORE_PROFILE at creation
 * switches them on.  Operational, no reference counterpart: the bench times its steps without the
 * events (their records cost host time and marker packets) and takes the stage split from a
 * profiled pass.  Timings read after calls made without events are those of the last profiled one. */
int32_t accord_store_set_profile(accord_store *store, uint32_t on);

/* ---- union of per-store partials (K6; PreAccept.reduce, messages/PreAccept.java:140-156) ----
 * parts: G device views (accord_deps_device_view of stores on this GPU, or received buffers) of
 * the same n txns, with key-disjoint parts ordered by key (CommandStores partition the keyspace).
 * The union becomes this store's current deps (read with device_view / download); txnIds are
 * global stream positions and txn_lo is the global position of txn 0 of the parts.  Parts with
 * RangeDeps (a range txn spanning several stores is in each store's RangeDeps under the same range
 * key) are unioned with RelationMultiMap.linearUnion on both sides (accord_deps_union). */
int32_t accord_deps_merge(accord_store *store, uint32_t nparts, const accord_deps *parts, uint32_t txn_lo);

/* ---- multi-GPU: one store per rank over RCCL (xGMI) ----
 * Rank r holds the partial deps of its key block for the txns intersecting it (batch txn_index =
 * global stream positions).  accord_deps_exchange_merge sends every partial to the rank owning
 * the txn (txn g -> rank floor(g*G/n_total)) with one grouped RCCL send/recv and unions the G parts
 * there; afterwards the store's current deps are the full (node-level) deps of its own txns.  Both
 * KeyDeps and RangeDeps travel (6 offset + 7 data arrays per destination); when any received part
 * holds RangeDeps the owner unions with accord_deps_union, else with the key-disjoint merge.
 * The exchange is plan (device offsets + one all-gather of the G x G count table, the only host
 * read) -> transport -> union (sized by the received counts; its totals are read, and a merge
 * error reported, when the result is first used: accord_deps_device_view / _download).
 *
 * accord_deps_exchange_local: the same plan and union for G stores of ONE device acting as ranks
 * 0..G-1 (stores[r] = rank r, no communicator), with the transport replaced by device copies of the
 * identical segment lists -- the multi-rank exchange exercised on one GPU (tests, rank simulation).
 * Each store afterwards holds the node-level deps of its own txns, as after accord_deps_exchange_merge. */
int32_t accord_comm_unique_id(void *id128);                  /* ncclGetUniqueId, 128 bytes */
int32_t accord_comm_init(accord_store *store, int32_t nranks, int32_t rank, const void *id128);
/* the communicator's size and this store's rank as RCCL reports them (ncclCommCount / ncclCommUserRank) */
int32_t accord_comm_size(accord_store *store, int32_t *nranks, int32_t *rank);
int32_t accord_deps_exchange_merge(accord_store *store, uint32_t n_total);
int32_t accord_deps_exchange_local(accord_store *const *stores, uint32_t nranks, uint32_t n_total);
int32_t accord_shard_timing(accord_store *store, float *exchange_ms, float *merge_ms);

/* ---- multi-GPU by stream segments (config 4) ----
 * The node's stream of TxnIds is cut into G consecutive segments; rank r owns segment r -- positions
 * [a_r, b_r) -- of EVERY CommandStore the node hosts and computes the node-level deps of those txns in
 * full (what PreAccept.reduce would have assembled from the per-store partials, messages/
 * PreAccept.java:140-156), so no partial deps cross the links.  What a segment needs from before it
 * is the CommandsForKey state at a_r: per key the entries a txn >= a_r can still reach, i.e. the run
 * from the last Write before a_r - W on (mapReduceActive's maxCommittedBefore bound,
 * local/CommandsForKey.java:620-645; earlier entries are pruned for good, as withRedundantBefore
 * does, :1654-1684).  That state is built on each rank from the small summaries of the earlier
 * segments (one all-gather):
 *   accord_segment_begin    resident status-at-time store: reset, the segment starts at stream
 *                           position seg_base; then accord_batch_upload of the segment (PreAccept
 *                           batch of key txns, positions seg_base + t);
 *   accord_segment_summary  per key, the segment's entries from its last Write before b - W on (all
 *                           of them when it has none), in stream order (positions ascending, a txn's
 *                           keys ascending), in device memory owned by the store (valid until the
 *                           next summary / begin);
 *                           accord_segment_summary_copy copies them into caller buffers (device,
 *                           or host memory for an exchange staged through the host);
 *   accord_segment_carry    the CommandsForKey state at seg_base from the summaries of segments
 *                           0..r-1 (device memory, stream order): per key, every entry at or after
 *                           the key's last Write before seg_base - W over all parts (the walk back from
 *                           the newest part that stops at that Write).
 *                           The store then stands at seg_base with that state, and accord_deps_compute
 *                           gives the segment's deps -- equal to one store computing the whole stream
 *                           (tests/test_gpu_segments.py).  Calling it again rewinds the store to the
 *                           segment's start (a bench step is carry + compute).
 * Every rank's store must cover the same key range; keys in a part are relative to key_lo. */
typedef struct {
    uint64_t        n;      /* entries */
    const uint32_t *key;    /* [n] device: key ordinal - key_lo */
    const uint32_t *ent;    /* [n] device: Txn.Kind ordinal << 29 | global stream position, ascending */
} accord_cfk_part;
int32_t accord_segment_begin(accord_store *store, uint32_t seg_base);
int32_t accord_segment_summary(accord_store *store, accord_cfk_part *out);
int32_t accord_segment_summary_copy(accord_store *store, uint32_t *key_dst, uint32_t *ent_dst, uint64_t cap);
int32_t accord_segment_carry(accord_store *store, uint32_t nparts, const accord_cfk_part *parts);
/* device ms of the last summary and carry (ACCORD_STORE_PROFILE stores, else 0) */
int32_t accord_segment_timing(accord_store *store, float *summary_ms, float *carry_ms);

/* ---- deps-set operations on device ----
 * Sources are device views (accord_deps_device_view) of stores on this store's device; the values
 * of all sources index the same TxnId table sorted ascending (the batch / stream), so TxnId order
 * is index order.  union and slice make their result this store's current deps (read it with
 * accord_deps_device_view / accord_deps_download; a source may be this store's own current deps).
 *
 * accord_deps_union: Deps.merge / PartialDeps.with of nparts (>= 1; 64 per pass) sets of the same n txns, KeyDeps
 *   and RangeDeps, keys may overlap -- RelationMultiMap.linearUnion (utils/RelationMultiMap.java:
 *   561-816) via KeyDeps.merge (primitives/KeyDeps.java:115-140) / RangeDeps.merge
 *   (primitives/RangeDeps.java:101-126): the coordinator-side merge of replica replies
 *   (coordinate/CoordinateTransaction.java:75,81) and the general PreAccept.reduce. */
int32_t accord_deps_union(accord_store *store, uint32_t nparts, const accord_deps *parts);

/* accord_deps_upload: a host PartialDeps set (e.g. the replies a coordinator received, decoded with
 *   KeyDeps/RangeDeps.SerializerSupport) becomes this store's current deps (H2D copy, sync). */
int32_t accord_deps_upload(accord_store *store, const accord_deps *host);

/* accord_deps_slice: KeyDeps.slice (primitives/KeyDeps.java:189-236) and RangeDeps.slice
 *   (primitives/RangeDeps.java:545-565, incl. trimUnusedValues, utils/RelationMultiMap.java:491-532)
 *   of every txn of src to Ranges: (sel_start, sel_end] sorted and de-overlapped, host pointers;
 *   sel_off[n+1] gives each txn its own ranges, or sel_off == NULL applies the same nsel ranges to
 *   every txn (Accept/Commit message construction per destination shard, messages/Accept.java:65-72). */
int32_t accord_deps_slice(accord_store *store, const accord_deps *src, const uint32_t *sel_off,
                          const uint32_t *sel_start, const uint32_t *sel_end, uint32_t nsel);

/* accord_deps_invert: txnIdsToKeys (KeyDeps.java:350-362) and txnIdsToRanges (RangeDeps.java:537-543)
 *   of every txn of src -- RelationMultiMap.invert (utils/RelationMultiMap.java:907-938): per txn
 *   |txnIds| end offsets (absolute, the first starting at |txnIds|), then per txnId its key (range)
 *   indices ascending.  Computed on device, returned in host memory owned by the library. */
typedef struct {
    uint32_t  n;
    uint32_t  reserved;
    uint64_t  kd_total, rd_total;
    uint32_t *kd_t2k_off;       /* [n+1] */
    int32_t  *kd_t2k;           /* [kd_total] */
    uint32_t *rd_t2r_off;       /* [n+1] */
    int32_t  *rd_t2r;           /* [rd_total] */
    void     *owner;            /* library-private */
} accord_deps_inverse;

int32_t accord_deps_invert(accord_store *store, const accord_deps *src, accord_deps_inverse *out);
void    accord_deps_inverse_release(accord_deps_inverse *inv);
/* accord_deps_range_stab: SearchableRangeList over every txn's RangeDeps (RangeDeps.ensureSearchable,
 *   primitives/RangeDeps.java:709-720; SearchableRangeList.build, utils/SearchableRangeList.java:79-133)
 *   built on the device, then for each query of txn i -- queries [q_off[i], q_off[i+1]), each
 *   (q_start, q_end] (a key k is (k-1, k]), host arrays -- the txnIds of txn i's RangeDeps ranges
 *   intersecting it, ascending unique (RangeDeps.forEach(range) / computeTxnIds(key),
 *   primitives/RangeDeps.java:158-189; CheckpointIntervalArray.forEach, utils/CheckpointIntervalArray.java:
 *   100-221).  txn values are src's rd_vals entries (stream positions).  A txn with more than 65536
 *   RangeDeps ranges or 32768 RangeDeps txnIds is ACCORD_ERR_CAPACITY.  Result in library-owned
 *   host memory: off[nq+1], txn[total]. */
typedef struct {
    uint32_t  nq;
    uint32_t  reserved;
    uint64_t  total;
    uint32_t *off;
    uint32_t *txn;
    void     *owner;            /* library-private */
} accord_range_stab;
int32_t accord_deps_range_stab(accord_store *store, const accord_deps *src, const uint32_t *q_off,
                               const uint32_t *q_start, const uint32_t *q_end, accord_range_stab *out);
void    accord_range_stab_release(accord_range_stab *r);

/* device ms of the last union / slice / invert (ACCORD_STORE_PROFILE stores, else 0) */
int32_t accord_ops_timing(accord_store *store, float *ms);

/* ---- MaxConflicts fold ----
 * Replaces, for the uploaded batch of key and range txns in stream order, the per-PreAccept
 *   Timestamp minNonConflicting = maxConflicts.get(keys)          (local/CommandStore.java:344,
 *                                                                  local/MaxConflicts.java:46-49)
 *   permitFastPath && txnId.compareTo(minNonConflicting) >= 0     (local/CommandStore.java:345)
 * followed by CommandStore.updateMaxConflicts(prev, updated) with the command's executeAt
 * (local/CommandStore.java:280-289, local/SafeCommandStore.java:192-210: globally visible kinds
 * only).  The map lives on the device with the store (CommandStore.maxConflicts, empty at create)
 * and carries over between batches.  present[i] = 0 means Timestamp.NONE (no entry on any key).
 * The epoch check and rejectBefore/preAcceptTimeout expiry (:328-331) are time-dependent and stay
 * in Java.
 *
 * executeAt of txn t = the batch's exec_* (Accept batch), else txnId when t takes the fast path.  A
 * globally visible txn that takes the slow path in a PreAccept batch gets
 * time.uniqueNow(minNonConflicting) (:348), a clock value only the caller can choose, and every
 * later txn of the batch depends on it.  The fold therefore stops there: out->folded = the first
 * such txn f (n when none).  Txns [first, f) are merged into the map; the outputs of txns
 * [first, f] are final (f's own reading does not depend on f's executeAt).  The caller picks f's
 * executeAt and continues with accord_max_conflicts_fold_from(store, f, executeAt, out), which
 * merges it and folds on from there.  Folding a batch again from an earlier txn is ACCORD_ERR_STATE.
 * Range txns read and write the store keys their ranges (s, e] cover, clipped to [key_lo, key_hi)
 * (an IntKey ReducingRangeMap has no points between keys); ranges must be non-empty, sorted and
 * non-overlapping (ACCORD_ERR_KEYS).  A range-domain ExclusiveSyncPoint returns txnId without reading
 * the map (markExclusiveSyncPoint, :335-339: present = 0, fast = 1; rejectBefore stays in Java) and
 * merges its executeAt; in the key domain it is ACCORD_ERR_KIND (preaccept casts its keys to Ranges). */
typedef struct {
    uint64_t *msb, *lsb;        /* [n] minNonConflicting (host arrays, caller-owned; NULL = skip) */
    int32_t  *node;
    uint8_t  *present;          /* [n] */
    uint8_t  *fast;             /* [n] txnId >= minNonConflicting */
    uint32_t  folded;           /* out: txns of the batch merged so far (see above) */
    uint32_t  reserved;
} accord_max_conflicts_out;
int32_t accord_max_conflicts_fold(accord_store *store, accord_max_conflicts_out *out);
int32_t accord_max_conflicts_fold_from(accord_store *store, uint32_t first, uint64_t exec_msb, uint64_t exec_lsb,
                                       int32_t exec_node, accord_max_conflicts_out *out);
int32_t accord_max_conflicts_reset(accord_store *store);     /* MaxConflicts.EMPTY */
/* the per-key map, [key_hi - key_lo] entries (present = 0: no entry) */
int32_t accord_max_conflicts_state(accord_store *store, uint64_t *msb, uint64_t *lsb, int32_t *node,
                                   uint8_t *present);

/* ---- WaitingOn + execution levelling (config 5) ----
 * Over the store's current computed deps (full stream: no txn_index, not merged), with every txn
 * STABLE, executeAt = txnId and none applied:
 *   WaitingOn of txn i (Commands.initialiseWaitingOn, local/Commands.java:735-753; bit layout of
 *   Command.WaitingOn, local/Command.java:1403-1437): bits [0, R_i) = its RangeDeps txnIds,
 *   [R_i, R_i + K_i) = its KeyDeps keys, as u64 words words[wo_off[i] .. wo_off[i+1]);
 *   level[i] = 0 without deps, else 1 + max level over its deps (the order in which CFK notify,
 *   local/CommandsForKey.java:1501-1635, releases txns to ReadyToExecute). */
typedef struct {
    uint32_t  n;
    uint32_t  max_level;
    uint64_t  words_total;
    uint64_t  preds_total;      /* edges of the reduced DAG the levelling ran on */
    uint32_t *level;            /* [n] */
    uint32_t *wo_off;           /* [n+1] word offsets */
    uint64_t *words;            /* [words_total] */
    void     *owner;            /* library-private */
    /* accord_waiting_on_initialise only (else NULL): WaitingOn.appliedOrInvalidated in the words'
     * layout -- bits [0, R_i) of Range-domain txns; all zero for Key-domain txns (null there) */
    uint64_t *applied_or_invalidated;
} accord_waiting_on;

int32_t accord_waiting_on_compute(accord_store *store);                 /* device-resident */
/* Commands.initialiseWaitingOn (local/Commands.java:735-753) with its initial updateWaitingOn
 * (:755-830; WaitingOn.Update, local/Command.java:1403-1600) for every txn of the last computed batch
 * of a registered-status store (resident, ACCORD_WINDOW_NONE), against the statuses registered at
 * the time of the call (register the batch's txns COMMITTED/STABLE with their executeAt first; a txn
 * without an executeAt is taken at its TxnId).  words: bits [0, R_i) = RangeDeps txnIds, set unless
 * the dep hasBeen(PreCommitted) and is truncated / invalidated (INVALID_OR_TRUNCATED, ERASED:
 * setAppliedOrInvalidated), executes after the txn (dep executeAt > own executeAt, own kind not
 * awaitsOnlyDeps: removeWaitingOn) or is APPLIED (setAppliedAndPropagate); bits [R_i, R_i + K_i) =
 * KeyDeps keys, set (CommandsForKey.notify clears them as the keys' predecessors apply).  The
 * propagation of an applied dep's own appliedOrInvalidated set is not modelled (taken as empty).  With a
 * RedundantBefore map set by accord_redundant_before_set_ex the removal step of updateWaitingOn
 * (removeRedundantDependencies) runs first: a removed dep is not waited on and not visited.  hasBeen(PreCommitted)
 * is read from the InternalStatus (>= COMMITTED): a dep at SaveStatus PreCommitted* (InternalStatus
 * PREACCEPTED / ACCEPTED, local/CommandsForKey.java:213-215) is treated as uncommitted -- the bit stays
 * set until the dep commits (conservative: never released earlier than the reference).  level = 0,
 * max_level = 0, preds_total = 0 (levelling is accord_waiting_on_compute's model).  Download with
 * accord_waiting_on_download (applied_or_invalidated set).  The deps are the batch's computed deps,
 * united with RedundantBefore.collectDeps when the store has a RedundantBefore map (the deps
 * PreAccept returns, messages/PreAccept.java:262-263); a union / slice result is refused. */
int32_t accord_waiting_on_initialise(accord_store *store);

/* ---- execution readiness: CommandsForKey.notify / notifyUnmanaged and
 * Commands.updateWaitingOn on the device ----
 * accord_waiting_on_initialise also puts the batch's txns into the store's waiting set (with a copy
 * of their deps).  accord_ready_update re-evaluates the waiting txns whose inputs changed (all of
 * them after a new batch or truncation) against the statuses registered so far (accord_txn_register) and returns the txns that became ReadyToExecute (Commands.maybeExecute,
 * local/Commands.java:656-733: no WaitingOn bit left and status STABLE), ascending global positions;
 * they leave the set (the caller executes them and registers them APPLIED, which in turn releases
 * their dependents at a later call).  Per waiting txn:
 *   range-dep bits   Commands.updateWaitingOn (:769-830) as in accord_waiting_on_initialise;
 *   key bits, managed txns (key domain, globally visible; STABLE): CommandsForKey.notify's test
 *                    (local/CommandsForKey.java:1512-1635) expectMissingCount == |missing|: no
 *                    unapplied committed txn of a kind it witnesses executes before it on the key and
 *                    none of its deps on the key is uncommitted;
 *   key bits, unmanaged txns (range domain, EphemeralRead; hasBeen Stable): registerUnmanaged
 *                    (:1406-1498), COMMIT records re-evaluated by updatePending once minUncommitted
 *                    passes them (:1315-1360), APPLY records released by notifyUnmanaged(APPLY,
 *                    next.executeAt) (:1264-1283).
 *   removal          with a map from accord_redundant_before_set_ex, each evaluation first applies
 *                    updateWaitingOn's removeRedundantDependencies step (see there) to the range deps;
 *   executeAtLeast   awaitsOnlyDeps kinds (ExclusiveSyncPoint, EphemeralRead): WaitingOn.updateExecuteAtLeast
 *                    (local/Command.java:1511-1514) with the executeAt of every range dep visited while
 *                    committed or TruncatedApply with a known executeAt after the txn's TxnId
 *                    (local/Commands.java:782-783; an INVALID_OR_TRUNCATED / ERASED event carries none), and
 *                    of the dep executing last
 *                    when registerUnmanaged / updatePending leave an APPLY record (local/CommandsForKey.java:
 *                    1370-1380, 1470-1478).
 * The reference evaluates the key tests when an event reaches the key (notifyAndUpdatePending,
 * :1163-1215); every call here evaluates them for every waiting txn whose inputs changed, so a txn is
 * reported at the first call at which its test holds -- never later than the reference releases it
 * (tests/test_ready.py compares with an event-driven restatement).  A waiting txn that is invalidated
 * or truncated leaves the set unreported.  An applied Range-domain dep propagates its own
 * appliedOrInvalidated (setAppliedAndPropagate, local/Command.java:1569-1583) in updateWaitingOn's
 * reverse walk.
 * The arrays stay valid until the next call on the store; `waiting` = txns still in the set. */
typedef struct {
    uint32_t  n;
    uint32_t  reserved;
    uint64_t  waiting;
    const uint32_t *txn;        /* [n] ascending global positions */
    /* [n] Command.executesAtLeast() of each (local/Command.java:1145-1150): executeAtLeast for
     * awaitsOnlyDeps kinds when it was updated, else the registered executeAt */
    const uint64_t *eal_msb, *eal_lsb;
    const int32_t  *eal_node;
} accord_ready;
int32_t accord_ready_update(accord_store *store, accord_ready *out);
/* Readiness mode of a registered-status store (set while its waiting set is empty).
 * ACCORD_READY_POLL (default): every accord_ready_update call re-evaluates the key tests of the
 *   waiting txns whose inputs changed, so a txn is released at the first call at which its test
 *   holds (never later than the reference).
 * ACCORD_READY_EVENTS: event-exact -- a key bit clears only when one of
 *   CommandsForKey.notifyAndUpdatePending's events reaches the key (local/CommandsForKey.java:
 *   1163-1215): accord_txn_register replays its events in order on the device, each against the
 *   state after it (the key's minUncommitted / next / nextWrite, :432-461; notify over committed[]
 *   in the executeAt range the change selects, :1501-1511; the unmanaged COMMIT / APPLY records,
 *   :1264-1283, 1315-1360; registerUnmanaged at the Stable transition); accord_waiting_on_initialise
 *   gives the txns already Stable their transition's step; a truncation notifies the unmanaged
 *   records of the keys it took entries from.  accord_ready_update then evaluates the range-dep bits
 *   and releases.  Releases equal the event-driven restatement (oracle or_lstore_event_mode) call by
 *   call.  The replay is one wave per registration (a correctness mode, not a throughput one).
 * The mode is a setting of the store: accord_store_reset empties the waiting set and keeps it. */
#define ACCORD_READY_POLL   0u
#define ACCORD_READY_EVENTS 1u
int32_t accord_ready_set_mode(accord_store *store, uint32_t mode);
int32_t accord_waiting_on_download(accord_store *store, accord_waiting_on *out);
void    accord_waiting_on_release(accord_waiting_on *wo);
/* device ms of the last accord_waiting_on_compute: bitsets, reduced predecessors, levelling */
int32_t accord_waiting_on_timing(accord_store *store, float *bits_ms, float *preds_ms, float *level_ms);
/* how the last accord_waiting_on_compute levelled: the stripe length of the striped levelling (0 =
 * the serial resolver alone, ACCORD_LV_MODE=serial) and whether its sweeps fell back to the serial
 * resolver (1) -- the levels are the same either way */
int32_t accord_waiting_on_levelling(accord_store *store, uint32_t *stripe, uint32_t *fallback);

/* ---- synthetic workload (SURVEY.md §8d stream; splitmix64 + Zipf rejection-inversion) ---- */
typedef struct {
    uint32_t n;               /* txns */
    uint32_t keys_per_txn;    /* k distinct keys per key txn */
    uint32_t keyspace;        /* key ordinals [0, keyspace) */
    uint32_t ranges_max;      /* range txns carry 1..ranges_max ranges */
    double   zipf_s;          /* 0 = uniform */
    double   write_frac;      /* P(Write) */
    double   range_frac;      /* fraction of range-domain txns */
    uint32_t range_len_max;   /* (s, s+len], len ~ U[1, range_len_max] */
    uint32_t node_mod;        /* node = 1 + (i mod node_mod) */
    uint64_t seed;
} accord_workload_cfg;

/* arrays are malloc'd; free with accord_workload_free */
int32_t accord_workload_generate(const accord_workload_cfg *cfg, accord_batch *out);
void    accord_workload_free(accord_batch *b);

#ifdef __cplusplus
}
#endif
#endif
