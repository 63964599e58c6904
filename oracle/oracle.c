/*
 * oracle.c -- CPU restatement of the reference dependency-calculation path.
 * TEST INFRASTRUCTURE ONLY (see oracle.h header).  All file:line citations are relative to
 * /root/reference/accord-core/src/main/java/accord/.
 */
#include "oracle.h"

#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------
 * Timestamp / TxnId  (primitives/Timestamp.java, primitives/TxnId.java, local/Node.java)
 * ------------------------------------------------------------------------------------------ */

#define IDENTITY_FLAGS 0x1EULL                   /* Timestamp.java:42 */
#define IDENTITY_LSB   0xFFFFFFFFFFFF001EULL     /* Timestamp.java:41 */

int or_ts_compare(uint64_t amsb, uint64_t alsb, int32_t anode, uint64_t bmsb, uint64_t blsb, int32_t bnode)
{
    /* Timestamp.compareTo: Long.compareUnsigned(msb), then Long.compare(lowHlc(lsb)) where
     * lowHlc = lsb >>> 16 (always non-negative), then flags & IDENTITY_FLAGS, then
     * Node.Id.compareTo = Integer.compare (Node.java:134-137). */
    if (amsb != bmsb) return amsb < bmsb ? -1 : 1;
    uint64_t ah = alsb >> 16, bh = blsb >> 16;
    if (ah != bh) return ah < bh ? -1 : 1;
    uint64_t af = alsb & IDENTITY_FLAGS, bf = blsb & IDENTITY_FLAGS;
    if (af != bf) return af < bf ? -1 : 1;
    if (anode != bnode) return anode < bnode ? -1 : 1;
    return 0;
}

int or_ts_equals(uint64_t amsb, uint64_t alsb, int32_t anode, uint64_t bmsb, uint64_t blsb, int32_t bnode)
{
    return amsb == bmsb && ((alsb ^ blsb) & IDENTITY_LSB) == 0 && anode == bnode;
}

typedef struct { uint64_t msb, lsb; int32_t node; } ts_t;

static inline int ts_cmp(const ts_t *a, const ts_t *b)
{
    return or_ts_compare(a->msb, a->lsb, a->node, b->msb, b->lsb, b->node);
}

/* Txn.Kind ordinals (primitives/Txn.java:53-118) and TxnId flag decoding (TxnId.java:129-157) */
enum { K_READ = 0, K_WRITE = 1, K_EPHEMERAL_READ = 2, K_SYNC_POINT = 3, K_EXCL_SYNC_POINT = 4, K_LOCAL_ONLY = 5 };
static inline int kind_of(uint64_t lsb)   { return (int)((lsb >> 1) & 7); }
static inline int domain_of(uint64_t lsb) { return (int)(lsb & 1); }      /* 0 Key, 1 Range */

/* Kind.isGloballyVisible (Txn.java:187-201); -1 = AssertionError */
static int is_globally_visible(int k)
{
    switch (k) {
    case K_EPHEMERAL_READ: case K_LOCAL_ONLY: return 0;
    case K_WRITE: case K_READ: case K_EXCL_SYNC_POINT: case K_SYNC_POINT: return 1;
    default: return -1;
    }
}

/* Kind.witnesses() (Txn.java:221-235) as a Kinds code, and Kinds.test (Txn.java:140-152) */
enum { WS = 0, RS_OR_WS = 1, ANY_GLOBALLY_VISIBLE = 2 };
static int witnesses_of(int k)
{
    switch (k) {
    case K_EPHEMERAL_READ: case K_READ: return WS;
    case K_WRITE: return RS_OR_WS;
    case K_SYNC_POINT: case K_EXCL_SYNC_POINT: return ANY_GLOBALLY_VISIBLE;
    default: return -1;            /* LocalOnly: AssertionError */
    }
}
static int kinds_test(int kinds, int k)
{
    switch (kinds) {
    case WS: return k == K_WRITE;
    case RS_OR_WS: return k == K_READ || k == K_WRITE;
    case ANY_GLOBALLY_VISIBLE: return is_globally_visible(k) == 1;
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * Small growable arrays
 * ------------------------------------------------------------------------------------------ */
typedef struct { uint32_t *p; size_t n, cap; } u32v;
typedef struct { int32_t *p; size_t n, cap; } i32v;

static int u32v_push(u32v *v, uint32_t x)
{
    if (v->n == v->cap) {
        size_t nc = v->cap ? v->cap * 2 : 64;
        uint32_t *np = (uint32_t *)realloc(v->p, nc * sizeof(uint32_t));
        if (!np) return -1;
        v->p = np; v->cap = nc;
    }
    v->p[v->n++] = x;
    return 0;
}
static int i32v_push(i32v *v, int32_t x)
{
    if (v->n == v->cap) {
        size_t nc = v->cap ? v->cap * 2 : 64;
        int32_t *np = (int32_t *)realloc(v->p, nc * sizeof(int32_t));
        if (!np) return -1;
        v->p = np; v->cap = nc;
    }
    v->p[v->n++] = x;
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * RelationMultiMap.AbstractBuilder  (utils/RelationMultiMap.java:88-271)
 *
 * Keys are 64-bit comparable codes: a key ordinal (IntKey, Integer.compare: IntKey.java:161-165)
 * or a range packed as start<<32|end, which orders exactly like Range.compare (start, then end:
 * Range.java:310-317).  Values are indices into a TxnId table compared with Timestamp.compareTo
 * and de-duplicated with Timestamp.equals.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
    const ts_t *tbl;          /* value table */
    uint64_t *keys;  uint32_t *key_limits; size_t kcap;
    uint32_t *k2v;   size_t vcap;        /* keysToValues buffer: values in add order */
    uint32_t key_count, key_offset, total_count;
    int has_ordered_keys, has_ordered_values;
} mm_builder;

static void mmb_init(mm_builder *b, const ts_t *tbl)
{
    memset(b, 0, sizeof(*b));
    b->tbl = tbl;
    b->has_ordered_keys = 1;
    b->has_ordered_values = 1;
}
static void mmb_reset(mm_builder *b)
{
    b->key_count = b->key_offset = b->total_count = 0;
    b->has_ordered_keys = b->has_ordered_values = 1;
}
static void mmb_free(mm_builder *b)
{
    free(b->keys); free(b->key_limits); free(b->k2v);
    memset(b, 0, sizeof(*b));
}

static inline int vcmp(const ts_t *tbl, uint32_t a, uint32_t b) { return ts_cmp(&tbl[a], &tbl[b]); }

/* stable insertion/merge sort of value indices by TxnId (Arrays.sort on objects is a stable
 * TimSort; equal-identity duplicates keep add order, and de-dup keeps the first) */
static void stable_sort_vals(const ts_t *tbl, uint32_t *a, uint32_t n, uint32_t *tmp)
{
    if (n < 2) return;
    if (n <= 16) {
        for (uint32_t i = 1; i < n; ++i) {
            uint32_t x = a[i]; uint32_t j = i;
            while (j > 0 && vcmp(tbl, a[j - 1], x) > 0) { a[j] = a[j - 1]; --j; }
            a[j] = x;
        }
        return;
    }
    uint32_t h = n / 2;
    stable_sort_vals(tbl, a, h, tmp);
    stable_sort_vals(tbl, a + h, n - h, tmp);
    uint32_t i = 0, j = h, o = 0;
    while (i < h && j < n) tmp[o++] = (vcmp(tbl, a[j], a[i]) < 0) ? a[j++] : a[i++];
    while (i < h) tmp[o++] = a[i++];
    while (j < n) tmp[o++] = a[j++];
    memcpy(a, tmp, n * sizeof(uint32_t));
}

static int mmb_finish_key(mm_builder *b)       /* finishKey(): RelationMultiMap.java:147-173 */
{
    if (b->total_count == b->key_offset && b->key_count > 0) { --b->key_count; return 0; }
    if (b->key_count == 0) return 0;
    if (!b->has_ordered_values) {
        uint32_t n = b->total_count - b->key_offset;
        uint32_t *tmp = (uint32_t *)malloc((size_t)n * sizeof(uint32_t) + 4);
        if (!tmp) return -1;
        stable_sort_vals(b->tbl, b->k2v + b->key_offset, n, tmp);
        free(tmp);
        uint32_t removed = 0;
        for (uint32_t i = b->key_offset + 1; i < b->total_count; ++i) {
            const ts_t *p = &b->tbl[b->k2v[i - 1]], *q = &b->tbl[b->k2v[i]];
            if (or_ts_equals(p->msb, p->lsb, p->node, q->msb, q->lsb, q->node)) ++removed;
            else if (removed > 0) b->k2v[i - removed] = b->k2v[i];
        }
        b->total_count -= removed;
    }
    b->key_limits[b->key_count - 1] = b->total_count;
    b->key_offset = b->total_count;
    return 0;
}

static int mmb_next_key(mm_builder *b, uint64_t key)   /* nextKey(): :125-145 */
{
    if (b->key_count > 0 && b->keys[b->key_count - 1] >= key) b->has_ordered_keys = 0;
    if (mmb_finish_key(b)) return -1;
    if (b->key_count == b->kcap) {
        size_t nc = b->kcap ? b->kcap * 2 : 16;
        uint64_t *nk = (uint64_t *)realloc(b->keys, nc * sizeof(uint64_t));
        uint32_t *nl = nk ? (uint32_t *)realloc(b->key_limits, nc * sizeof(uint32_t)) : NULL;
        if (!nk || !nl) { if (nk) b->keys = nk; return -1; }
        b->keys = nk; b->key_limits = nl; b->kcap = nc;
    }
    b->keys[b->key_count++] = key;
    b->has_ordered_values = 1;
    return 0;
}

static int mmb_add_value(mm_builder *b, uint32_t v)   /* add(V): :185-199 */
{
    if (b->has_ordered_values && b->total_count > b->key_offset
        && vcmp(b->tbl, b->k2v[b->total_count - 1], v) >= 0)
        b->has_ordered_values = 0;
    if (b->total_count >= b->vcap) {
        size_t nc = b->vcap ? b->vcap * 2 : 64;
        uint32_t *nv = (uint32_t *)realloc(b->k2v, nc * sizeof(uint32_t));
        if (!nv) return -1;
        b->k2v = nv; b->vcap = nc;
    }
    b->k2v[b->total_count++] = v;
    return 0;
}

static int mmb_add(mm_builder *b, uint64_t key, uint32_t v)   /* add(K, V): :175-180 */
{
    if (b->key_count == 0 || b->keys[b->key_count - 1] != key)
        if (mmb_next_key(b, key)) return -1;
    return mmb_add_value(b, v);
}

/* Output accumulator for a sequence of per-txn multimaps */
typedef struct {
    u32v key_off, keys_lo, keys_hi, val_off, vals, k2v_off;
    i32v k2v;
} mm_out;

static int mmo_init(mm_out *o)
{
    memset(o, 0, sizeof(*o));
    if (u32v_push(&o->key_off, 0) || u32v_push(&o->val_off, 0) || u32v_push(&o->k2v_off, 0)) return -1;
    return 0;
}
static void mmo_free(mm_out *o)
{
    free(o->key_off.p); free(o->keys_lo.p); free(o->keys_hi.p); free(o->val_off.p);
    free(o->vals.p); free(o->k2v_off.p); free(o->k2v.p);
    memset(o, 0, sizeof(*o));
}
static int mmo_close_txn(mm_out *o)
{
    if (u32v_push(&o->key_off, (uint32_t)o->keys_lo.n)) return -1;
    if (u32v_push(&o->val_off, (uint32_t)o->vals.n)) return -1;
    if (u32v_push(&o->k2v_off, (uint32_t)o->k2v.n)) return -1;
    return 0;
}

static int cmp_u64(const void *a, const void *b)
{
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* build(): :201-260.  Appends one multimap to `o` (possibly empty = none()).  is_range selects
 * how a key code is split into the output key arrays.  Returns -1 on a builder exception. */
static int mmb_build(mm_builder *b, mm_out *o, int is_range)
{
    if (b->total_count == 0) return mmo_close_txn(o);                 /* none() */
    if (mmb_finish_key(b)) return -1;

    uint32_t total = b->total_count;
    uint32_t *uniq = (uint32_t *)malloc((size_t)total * sizeof(uint32_t) + 4);
    uint32_t *tmp = (uint32_t *)malloc((size_t)total * sizeof(uint32_t) + 4);
    if (!uniq || !tmp) { free(uniq); free(tmp); return -1; }
    memcpy(uniq, b->k2v, total * sizeof(uint32_t));
    stable_sort_vals(b->tbl, uniq, total, tmp);
    uint32_t value_count = 1;
    for (uint32_t i = 1; i < total; ++i) {
        const ts_t *p = &b->tbl[uniq[value_count - 1]], *q = &b->tbl[uniq[i]];
        if (!or_ts_equals(p->msb, p->lsb, p->node, q->msb, q->lsb, q->node)) uniq[value_count++] = uniq[i];
    }
    free(tmp);

    uint32_t kc = b->key_count;
    uint64_t *sorted_keys = (uint64_t *)malloc((size_t)kc * sizeof(uint64_t) + 8);
    uint32_t *sorted_idx = NULL;
    if (!sorted_keys) { free(uniq); return -1; }
    memcpy(sorted_keys, b->keys, kc * sizeof(uint64_t));
    if (!b->has_ordered_keys) {
        sorted_idx = (uint32_t *)malloc((size_t)kc * sizeof(uint32_t) + 4);
        if (!sorted_idx) { free(uniq); free(sorted_keys); return -1; }
        qsort(sorted_keys, kc, sizeof(uint64_t), cmp_u64);
        for (uint32_t i = 1; i < kc; ++i)
            if (sorted_keys[i - 1] == sorted_keys[i]) {   /* "Key ... has been visited more than once" */
                free(uniq); free(sorted_keys); free(sorted_idx); return -1;
            }
        for (uint32_t i = 0; i < kc; ++i) {
            uint32_t lo = 0, hi = kc;
            while (lo < hi) { uint32_t m = (lo + hi) / 2; if (sorted_keys[m] < b->keys[i]) lo = m + 1; else hi = m; }
            sorted_idx[lo] = i;
        }
    }

    /* emit keys, values, then result[keyCount + totalCount] */
    for (uint32_t ki = 0; ki < kc; ++ki) {
        uint64_t k = sorted_keys[ki];
        if (u32v_push(&o->keys_lo, is_range ? (uint32_t)(k >> 32) : (uint32_t)k)) goto fail;
        if (u32v_push(&o->keys_hi, is_range ? (uint32_t)k : 0)) goto fail;
    }
    for (uint32_t v = 0; v < value_count; ++v)
        if (u32v_push(&o->vals, uniq[v])) goto fail;

    size_t base = o->k2v.n;
    for (uint32_t i = 0; i < kc; ++i) if (i32v_push(&o->k2v, 0)) goto fail;
    int32_t offset = (int32_t)kc;
    for (uint32_t ki = 0; ki < kc; ++ki) {
        uint32_t k = sorted_idx ? sorted_idx[ki] : ki;
        uint32_t from = k == 0 ? 0 : b->key_limits[k - 1];
        uint32_t to = b->key_limits[k];
        /* SortedArrays.foldlIntersection(values, keysToValues[from,to)) -> result[offset++] = li */
        uint32_t li = 0;
        for (uint32_t r = from; r < to; ++r) {
            uint32_t lo = li, hi = value_count;
            while (lo < hi) { uint32_t m = (lo + hi) / 2; if (vcmp(b->tbl, uniq[m], b->k2v[r]) < 0) lo = m + 1; else hi = m; }
            if (lo < value_count && vcmp(b->tbl, uniq[lo], b->k2v[r]) == 0) {
                if (i32v_push(&o->k2v, (int32_t)lo)) goto fail;
                ++offset;
                li = lo + 1;
            }
        }
        o->k2v.p[base + ki] = offset;
    }
    free(uniq); free(sorted_keys); free(sorted_idx);
    return mmo_close_txn(o);
fail:
    free(uniq); free(sorted_keys); free(sorted_idx);
    return -1;
}

/* ------------------------------------------------------------------------------------------
 * CommandsForKey (local/CommandsForKey.java) -- literal restatement of the state and of
 * mapReduceActive.  InternalStatus ordinals: :194-203.
 * ------------------------------------------------------------------------------------------ */
enum { S_TRANSITIVELY_KNOWN = 0, S_HISTORICAL, S_PREACCEPTED, S_ACCEPTED, S_COMMITTED, S_STABLE,
       S_APPLIED, S_INVALID_OR_TRUNCATED };

typedef struct {
    uint32_t txn;            /* index into the stream table (TxnId) */
    uint8_t  status;
    ts_t     execute_at;
} txninfo_t;

typedef struct {
    txninfo_t *txns;   uint32_t n;     /* sorted by TxnId, :415 */
    uint32_t *committed; uint32_t nc;  /* indices into txns, sorted by executeAt, :419 */
    uint32_t redundant_before;         /* shardRedundantBefore as a position (0: none), :413 */
} cfk_t;

static __thread const ts_t *g_sort_tbl;   /* qsort context (thread-local: one thread per store) */
static __thread const txninfo_t *g_sort_txns;
static int cmp_committed(const void *a, const void *b)
{
    const txninfo_t *x = &g_sort_txns[*(const uint32_t *)a], *y = &g_sort_txns[*(const uint32_t *)b];
    int c = ts_cmp(&x->execute_at, &y->execute_at);
    if (c) return c;
    /* Arrays.sort(Object[], Comparator) is stable: keep TxnId order among equal executeAt */
    return (*(const uint32_t *)a < *(const uint32_t *)b) ? -1 : 1;
}

/* CommandsForKey(...) constructor: rebuild committed[] by a full pass + sort (:422-470).
 * The reference allocates a brand new TxnInfo[] on every update (insert :880-944,
 * update :652-706); the copy is restated so the CPU baseline pays the same O(n) per change. */
static int cfk_rebuild(cfk_t *c, txninfo_t *new_txns, uint32_t new_n)
{
    free(c->txns);
    c->txns = new_txns; c->n = new_n;
    uint32_t count = 0;
    for (uint32_t i = 0; i < new_n; ++i)
        if (new_txns[i].status >= S_COMMITTED && new_txns[i].status != S_INVALID_OR_TRUNCATED) ++count;
    free(c->committed);
    c->committed = (uint32_t *)malloc((size_t)count * sizeof(uint32_t) + 4);
    if (!c->committed) return -1;
    c->nc = 0;
    for (uint32_t i = 0; i < new_n; ++i)
        if (new_txns[i].status >= S_COMMITTED && new_txns[i].status != S_INVALID_OR_TRUNCATED) c->committed[c->nc++] = i;
    /* stable sort by executeAt (Arrays.sort of objects is stable); committed entries arrive in TxnId
     * order and executeAt >= TxnId, so the array is nearly sorted: insertion sort, O(n + inversions) */
    g_sort_txns = new_txns;
    for (uint32_t a = 1; a < c->nc; ++a) {
        const uint32_t x = c->committed[a];
        uint32_t b = a;
        while (b > 0 && cmp_committed(&c->committed[b - 1], &x) > 0) { c->committed[b] = c->committed[b - 1]; --b; }
        c->committed[b] = x;
    }
    return 0;
}

/* Arrays.binarySearch(txns, ts): returns index of an equal element, else -(ins)-1 */
static long cfk_search(const cfk_t *c, const ts_t *tbl, const ts_t *ts)
{
    long lo = 0, hi = (long)c->n - 1;
    while (lo <= hi) {
        long m = (lo + hi) >> 1;
        int r = ts_cmp(&tbl[c->txns[m].txn], ts);
        if (r < 0) lo = m + 1; else if (r > 0) hi = m - 1; else return m;
    }
    return -(lo + 1);
}

static int cfk_insert(cfk_t *c, const ts_t *tbl, uint32_t txn, uint8_t status)
{
    long pos = cfk_search(c, tbl, &tbl[txn]);
    if (pos >= 0) return -1;                 /* already present: not expected in the model */
    pos = -1 - pos;
    txninfo_t *nt = (txninfo_t *)malloc(((size_t)c->n + 1) * sizeof(txninfo_t));
    if (!nt) return -1;
    memcpy(nt, c->txns, (size_t)pos * sizeof(txninfo_t));
    nt[pos].txn = txn; nt[pos].status = status; nt[pos].execute_at = tbl[txn];
    memcpy(nt + pos + 1, c->txns + pos, ((size_t)c->n - pos) * sizeof(txninfo_t));
    return cfk_rebuild(c, nt, c->n + 1);
}

static int cfk_update_status(cfk_t *c, const ts_t *tbl, uint32_t txn, uint8_t status, const ts_t *execute_at)
{
    long pos = cfk_search(c, tbl, &tbl[txn]);
    if (pos < 0) return -1;
    txninfo_t *nt = (txninfo_t *)malloc((size_t)c->n * sizeof(txninfo_t) + sizeof(txninfo_t));
    if (!nt) return -1;
    memcpy(nt, c->txns, (size_t)c->n * sizeof(txninfo_t));
    nt[pos].status = status; nt[pos].execute_at = *execute_at;
    return cfk_rebuild(c, nt, c->n);
}

/* CommandsForKey.mapReduceActive (:614-650), emitting (key, txn) into the builder */
static int cfk_map_reduce_active(const cfk_t *c, const ts_t *tbl, const ts_t *started_before, int test_kinds,
                                 uint64_t key, mm_builder *b, long exclude_txn)
{
    const ts_t *max_committed_before = NULL;
    {
        /* SortedArrays.binarySearch(committed, ..., (f, v) -> f.compareTo(v.executeAt), FAST) */
        long lo = 0, hi = (long)c->nc - 1, found = -1;
        while (lo <= hi) {
            long m = (lo + hi) >> 1;
            int r = ts_cmp(started_before, &c->txns[c->committed[m]].execute_at);
            if (r > 0) lo = m + 1; else if (r < 0) hi = m - 1; else { found = m; break; }
        }
        long i = found >= 0 ? found - 1 : lo - 1;            /* i<0 ? -2-i : --i */
        while (i >= 0 && kind_of(tbl[c->txns[c->committed[i]].txn].lsb) != K_WRITE) --i;
        max_committed_before = i < 0 ? NULL : &c->txns[c->committed[i]].execute_at;
    }
    long end = cfk_search(c, tbl, started_before);           /* insertPos(0, startedBefore) */
    if (end < 0) end = -1 - end;

    for (long i = 0; i < end; ++i) {
        const txninfo_t *t = &c->txns[i];
        if (!kinds_test(test_kinds, kind_of(tbl[t->txn].lsb))) continue;
        switch (t->status) {
        case S_COMMITTED: case S_STABLE: case S_APPLIED:
            if (max_committed_before == NULL || ts_cmp(&t->execute_at, max_committed_before) >= 0) break;
            continue;
        case S_TRANSITIVELY_KNOWN: case S_INVALID_OR_TRUNCATED:
            continue;
        default: break;
        }
        /* PreAccept.calculatePartialDeps lambda (messages/PreAccept.java:255-258): p1 filter */
        if (exclude_txn >= 0 && (uint32_t)exclude_txn == t->txn) continue;
        if (mmb_add(b, key, t->txn)) return -1;
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * Range commands (impl/InMemoryCommandStore.java:100 TreeMap<TxnId,RangeCommand>, registered
 * at :739-762, scanned at :883-1016).  SaveStatus is collapsed to {live, Erased}.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
    uint32_t txn;
    int erased;
    uint32_t r0, r1;                 /* its ranges: stream rng_* [r0, r1) */
} rangecmd_t;

typedef struct { uint64_t range; uint32_t *txns; uint32_t n, cap; } collect_t;

static int range_intersects_key(uint32_t s, uint32_t e, uint32_t key) { return s < key && key <= e; }
static int range_intersects_range(uint32_t s, uint32_t e, uint32_t s2, uint32_t e2) { return s < e2 && s2 < e; }

/* ------------------------------------------------------------------------------------------
 * Stream driver (status-at-time model)
 * ------------------------------------------------------------------------------------------ */

static int alloc_out(or_deps *out, mm_out *kd, mm_out *rd, uint32_t n)
{
    memset(out, 0, sizeof(*out));
    out->n = n;
#define TAKE(dst, v) do { out->dst = (v).p ? (v).p : (__typeof__(out->dst))malloc(4); (v).p = NULL; if (!out->dst) return -1; } while (0)
    TAKE(kd_key_off, kd->key_off); TAKE(kd_keys, kd->keys_lo); TAKE(kd_val_off, kd->val_off);
    TAKE(kd_vals, kd->vals); TAKE(kd_k2v_off, kd->k2v_off); TAKE(kd_k2v, kd->k2v);
    TAKE(rd_rng_off, rd->key_off); TAKE(rd_rng_start, rd->keys_lo); TAKE(rd_rng_end, rd->keys_hi);
    TAKE(rd_val_off, rd->val_off); TAKE(rd_vals, rd->vals); TAKE(rd_r2v_off, rd->k2v_off); TAKE(rd_r2v, rd->k2v);
#undef TAKE
    return 0;
}

void or_deps_free(or_deps *d)
{
    if (!d) return;
    free(d->kd_key_off); free(d->kd_keys); free(d->kd_val_off); free(d->kd_vals); free(d->kd_k2v_off); free(d->kd_k2v);
    free(d->rd_rng_off); free(d->rd_rng_start); free(d->rd_rng_end); free(d->rd_val_off); free(d->rd_vals);
    free(d->rd_r2v_off); free(d->rd_r2v);
    memset(d, 0, sizeof(*d));
}

static uint32_t max_key(const or_stream *s, uint32_t n)
{
    uint32_t m = 0;
    for (uint32_t p = 0; p < s->key_off[n]; ++p) if (s->key_ord[p] > m) m = s->key_ord[p];
    if (s->rng_off)
        for (uint32_t r = 0; r < s->rng_off[n]; ++r) if (s->rng_end[r] > m) m = s->rng_end[r];
    return m;
}

/* validation shared by both restatements: TxnId strictly ascending, keys sorted unique,
 * ranges sorted and de-overlapped (AbstractRanges.sortAndDeoverlap MERGE_OVERLAPPING:
 * AbstractRanges.java:696-782), domain consistent with the payload, no LocalOnly query. */
static int validate(const or_stream *s, uint32_t n)
{
    for (uint32_t i = 0; i < n; ++i) {
        if (i > 0 && or_ts_compare(s->msb[i - 1], s->lsb[i - 1], s->node[i - 1], s->msb[i], s->lsb[i], s->node[i]) >= 0) return -2;
        if (witnesses_of(kind_of(s->lsb[i])) < 0) return -3;
        for (uint32_t p = s->key_off[i] + 1; p < s->key_off[i + 1]; ++p) if (s->key_ord[p - 1] >= s->key_ord[p]) return -4;
        if (s->key_ord && s->key_off[i + 1] > s->key_off[i] && s->key_ord[s->key_off[i + 1] - 1] >= 0x80000000u) return -4;
        uint32_t nr = s->rng_off ? s->rng_off[i + 1] - s->rng_off[i] : 0;
        if (domain_of(s->lsb[i]) == 0 && nr) return -5;
        if (domain_of(s->lsb[i]) == 1 && s->key_off[i + 1] != s->key_off[i]) return -5;
        for (uint32_t r = 0; r < nr; ++r) {
            uint32_t a = s->rng_off[i] + r;
            if (s->rng_start[a] >= s->rng_end[a]) return -6;
            if (r > 0 && s->rng_end[a - 1] > s->rng_start[a]) return -6;
        }
    }
    return 0;
}

/* Accept batches: startedBefore of txn i (executeAt for Accept, messages/Accept.java:113-117;
 * the txnId itself for PreAccept, messages/PreAccept.java:245-265) */
static ts_t started_before(const or_stream *s, uint32_t i)
{
    ts_t t;
    if (s->exec_msb) { t.msb = s->exec_msb[i]; t.lsb = s->exec_lsb[i]; t.node = s->exec_node[i]; }
    else { t.msb = s->msb[i]; t.lsb = s->lsb[i]; t.node = s->node[i]; }
    return t;
}

/* p1 of calculatePartialDeps: executeAt.equals(txnId) ? null : txnId (PreAccept.java:259) */
static long p1_of(const or_stream *s, uint32_t i)
{
    if (!s->exec_msb) return -1;
    return or_ts_equals(s->exec_msb[i], s->exec_lsb[i], s->exec_node[i], s->msb[i], s->lsb[i], s->node[i]) ? -1 : (long)i;
}

/* number of stream txns j < n with txnId_j < ts (TxnIds are strictly ascending): the txns a
 * startedBefore bound admits (CommandsForKey.insertPos, :1698-1703) */
static uint32_t bound_of(const or_stream *s, uint32_t n, const ts_t *ts, uint32_t i)
{
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        uint32_t m = (lo + hi) / 2;
        if (or_ts_compare(s->msb[m], s->lsb[m], s->node[m], ts->msb, ts->lsb, ts->node) < 0) lo = m + 1; else hi = m;
    }
    /* batch by batch: txns of later batches are not registered yet */
    if (s->batch_end && lo > s->batch_end[i]) lo = s->batch_end[i];
    return lo;
}

/* an Accept's executeAt never precedes its txnId (Commands.accept, local/Commands.java) */
static int validate_exec(const or_stream *s, uint32_t n)
{
    if (!s->exec_msb) return 0;
    for (uint32_t i = 0; i < n; ++i)
        if (or_ts_compare(s->exec_msb[i], s->exec_lsb[i], s->exec_node[i], s->msb[i], s->lsb[i], s->node[i]) < 0) return -1;
    return 0;
}

static int stream_literal(const or_stream *s, uint32_t n, or_deps *out)
{
    int rc = validate(s, n);
    if (!rc) rc = validate_exec(s, n);
    if (rc) return rc;
    ts_t *tbl = (ts_t *)malloc((size_t)(n ? n : 1) * sizeof(ts_t));
    if (!tbl) return -1;
    for (uint32_t i = 0; i < n; ++i) { tbl[i].msb = s->msb[i]; tbl[i].lsb = s->lsb[i]; tbl[i].node = s->node[i]; }
    g_sort_tbl = tbl;
    uint32_t nkeys = max_key(s, n) + 1;
    cfk_t *cfks = (cfk_t *)calloc(nkeys, sizeof(cfk_t));
    rangecmd_t *rcs = (rangecmd_t *)calloc(n ? n : 1, sizeof(rangecmd_t));
    uint32_t nrc = 0, rc_erase_cursor = 0;
    mm_builder kb, rb;
    mm_out kd, rd;
    collect_t *coll = NULL; uint32_t ncoll = 0, capcoll = 0;
    mmb_init(&kb, tbl); mmb_init(&rb, tbl);
    rc = -1;
    if (!cfks || !rcs || mmo_init(&kd) || mmo_init(&rd)) goto done;

    uint32_t reg = 0;                        /* txns [0, reg) are registered */
    for (uint32_t i = 0; i < n; ++i) {
        const ts_t sb_i = started_before(s, i);
        const long p1 = p1_of(s, i);
        uint32_t reg_to = bound_of(s, n, &sb_i, i);  /* an Accept sees every txn started before executeAt */
        if (reg_to < i + 1) reg_to = i + 1;
        /* 1. status at time i: txn j = i-W-1 leaves the window -> APPLIED (executeAt=txnId) if a
         *    key txn, Erased if a range txn. */
        if ((uint64_t)i >= (uint64_t)s->window + 1) {
            uint32_t j = (uint32_t)((uint64_t)i - s->window - 1);
            if (domain_of(s->lsb[j]) == 0) {
                if (is_globally_visible(kind_of(s->lsb[j])) == 1)
                    for (uint32_t p = s->key_off[j]; p < s->key_off[j + 1]; ++p)
                        if (cfk_update_status(&cfks[s->key_ord[p]], tbl, j, S_APPLIED, &tbl[j])) goto done;
            } else {
                while (rc_erase_cursor < nrc && rcs[rc_erase_cursor].txn <= j) {
                    if (rcs[rc_erase_cursor].txn == j) rcs[rc_erase_cursor].erased = 1;
                    ++rc_erase_cursor;
                }
            }
        }
        /* 2. register txns [reg, reg_to) -- txn i, and for an Accept every txn started before its
         *    executeAt -- as PREACCEPTED (SafeCommandStore.updateCommandsForKey :212-239 ->
         *    CommandsForKey.insert; range txns -> InMemoryCommandStore rangeCommands :739-762) */
        for (; reg < reg_to; ++reg) {
            const uint32_t g = reg;
            const int kind_g = kind_of(s->lsb[g]);
            if (domain_of(s->lsb[g]) == 0) {
                if (is_globally_visible(kind_g) == 1)
                    for (uint32_t p = s->key_off[g]; p < s->key_off[g + 1]; ++p)
                        if (cfk_insert(&cfks[s->key_ord[p]], tbl, g, S_PREACCEPTED)) goto done;
            } else {
                rcs[nrc].txn = g; rcs[nrc].erased = 0; rcs[nrc].r0 = s->rng_off[g]; rcs[nrc].r1 = s->rng_off[g + 1];
                ++nrc;
            }
        }

        /* 3. calculatePartialDeps (messages/PreAccept.java:245-265): startedBefore = executeAt
         *    (= txnId for PreAccept, the Accept's executeAt otherwise), p1 = txnId unless they are
         *    equal, keys first then ranges (SafeCommandStore.java:269-274). */
        int kind_i = kind_of(s->lsb[i]);
        int test_kinds = witnesses_of(kind_i);
        mmb_reset(&kb); mmb_reset(&rb);
        const ts_t *sb = &sb_i;
        if (domain_of(s->lsb[i]) == 0) {
            for (uint32_t p = s->key_off[i]; p < s->key_off[i + 1]; ++p) {
                uint32_t key = s->key_ord[p];
                if (cfk_map_reduce_active(&cfks[key], tbl, sb, test_kinds, key, &kb, p1)) goto done;
            }
        } else {
            /* mapReduceForKey Range case (InMemoryCommandStore.java:274-289): every CFK key in
             * each (start,end] in ascending order */
            for (uint32_t r = s->rng_off[i]; r < s->rng_off[i + 1]; ++r)
                for (uint32_t key = s->rng_start[r] + 1; key <= s->rng_end[r] && key < nkeys; ++key)
                    if (cfks[key].n && cfk_map_reduce_active(&cfks[key], tbl, sb, test_kinds, key, &kb, p1)) goto done;
        }
        /* mapReduceRangesInternal: TreeMap<Range, List<TxnInfo>> collect by Range.compare */
        ncoll = 0;
        for (uint32_t c = 0; c < nrc; ++c) {
            const rangecmd_t *cmd = &rcs[c];
            if (cmd->erased) continue;                                         /* :891 */
            if (ts_cmp(&tbl[cmd->txn], sb) >= 0) continue;                     /* :901-902 */
            if (p1 >= 0 && (uint32_t)p1 == cmd->txn) continue;                 /* p1 filter */
            if (!kinds_test(test_kinds, kind_of(s->lsb[cmd->txn]))) continue;  /* :927 */
            for (uint32_t a = cmd->r0; a < cmd->r1; ++a) {                     /* foldl :953-959 */
                uint32_t rs = s->rng_start[a], re = s->rng_end[a];
                int hit = 0;
                if (domain_of(s->lsb[i]) == 0) {
                    for (uint32_t p = s->key_off[i]; p < s->key_off[i + 1] && !hit; ++p)
                        hit = range_intersects_key(rs, re, s->key_ord[p]);
                } else {
                    for (uint32_t r = s->rng_off[i]; r < s->rng_off[i + 1] && !hit; ++r)
                        hit = range_intersects_range(rs, re, s->rng_start[r], s->rng_end[r]);
                }
                if (!hit) continue;
                uint64_t code = ((uint64_t)rs << 32) | re;
                uint32_t ci = 0;
                while (ci < ncoll && coll[ci].range != code) ++ci;
                if (ci == ncoll) {
                    if (ncoll == capcoll) {
                        uint32_t nc = capcoll ? capcoll * 2 : 16;
                        collect_t *np = (collect_t *)realloc(coll, nc * sizeof(collect_t));
                        if (!np) goto done;
                        memset(np + capcoll, 0, (nc - capcoll) * sizeof(collect_t));
                        coll = np; capcoll = nc;
                    }
                    coll[ncoll].range = code; coll[ncoll].n = 0;
                    ++ncoll;
                }
                collect_t *cl = &coll[ci];
                if (cl->n == 0 || cl->txns[cl->n - 1] != cmd->txn) {
                    if (cl->n == cl->cap) {
                        uint32_t nc = cl->cap ? cl->cap * 2 : 8;
                        uint32_t *np = (uint32_t *)realloc(cl->txns, nc * sizeof(uint32_t));
                        if (!np) goto done;
                        cl->txns = np; cl->cap = nc;
                    }
                    cl->txns[cl->n++] = cmd->txn;
                }
            }
        }
        /* replay in Range.compare order */
        for (uint32_t a = 1; a < ncoll; ++a) {
            collect_t x = coll[a]; uint32_t b2 = a;
            while (b2 > 0 && coll[b2 - 1].range > x.range) { coll[b2] = coll[b2 - 1]; --b2; }
            coll[b2] = x;
        }
        for (uint32_t a = 0; a < ncoll; ++a)
            for (uint32_t t = 0; t < coll[a].n; ++t)
                if (mmb_add(&rb, coll[a].range, coll[a].txns[t])) goto done;

        if (mmb_build(&kb, &kd, 0)) goto done;
        if (mmb_build(&rb, &rd, 1)) goto done;
    }
    if (alloc_out(out, &kd, &rd, n)) goto done;
    rc = 0;
done:
    if (cfks) { for (uint32_t k = 0; k < nkeys; ++k) { free(cfks[k].txns); free(cfks[k].committed); } }
    free(cfks); free(rcs);
    if (coll) { for (uint32_t a = 0; a < capcoll; ++a) free(coll[a].txns); }
    free(coll);
    mmb_free(&kb); mmb_free(&rb);
    mmo_free(&kd); mmo_free(&rd);
    free(tbl);
    return rc;
}

int or_stream_deps_literal(const or_stream *s, or_deps *out) { return stream_literal(s, s->n, out); }
int or_stream_deps_literal_prefix(const or_stream *s, uint32_t limit, or_deps *out)
{
    return stream_literal(s, limit < s->n ? limit : s->n, out);
}

/* ------------------------------------------------------------------------------------------
 * Fast restatement.  Under the status-at-time model the a3 filter for (txn i, key) reduces to
 * the witnessed entries of the key's history in [lcw, i) where lcw is the last Write entry
 * j < i-W (else the start of the history): CommandsForKey.java:620-645 with every j < i-W
 * APPLIED at executeAt=txnId (so committed[] is the history prefix before i-W) and every
 * i-W <= j < i PREACCEPTED.  Range commands: live iff j >= i-W, no pruning (InMemoryCommandStore
 * .java:883-1016).  Accept batches replace the upper bound i by `bound` = the txns started before
 * executeAt (all registered, PREACCEPTED when j >= i-W) and drop the txn itself (p1); every
 * APPLIED entry still precedes executeAt, so lcw is unchanged.
 * ------------------------------------------------------------------------------------------ */
static int cmp_u32(const void *a, const void *b)
{
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return x < y ? -1 : x > y;
}

int or_stream_deps_fast(const or_stream *s, or_deps *out)
{
    uint32_t n = s->n;
    int rc = validate(s, n);
    if (!rc) rc = validate_exec(s, n);
    if (rc) return rc;
    uint32_t nkeys = max_key(s, n) + 1;
    uint32_t P = s->key_off[n];
    uint32_t *hoff = (uint32_t *)calloc((size_t)nkeys + 1, sizeof(uint32_t));
    uint32_t *hist = (uint32_t *)malloc((size_t)(P ? P : 1) * sizeof(uint32_t));
    uint32_t *cur = (uint32_t *)malloc((size_t)(nkeys + 1) * sizeof(uint32_t));
    mm_out kd, rd;
    u32v lists = {0}, lens = {0}, heads = {0}, uni = {0}, rcmd = {0};
    rc = -1;
    if (!hoff || !hist || !cur || mmo_init(&kd) || mmo_init(&rd)) goto done;

    /* histories: stable counting sort of registered (key, txn) pairs */
    for (uint32_t i = 0; i < n; ++i)
        if (domain_of(s->lsb[i]) == 0 && is_globally_visible(kind_of(s->lsb[i])) == 1)
            for (uint32_t p = s->key_off[i]; p < s->key_off[i + 1]; ++p) hoff[s->key_ord[p] + 1]++;
    for (uint32_t k = 0; k < nkeys; ++k) hoff[k + 1] += hoff[k];
    memcpy(cur, hoff, (size_t)(nkeys + 1) * sizeof(uint32_t));
    for (uint32_t i = 0; i < n; ++i)
        if (domain_of(s->lsb[i]) == 0 && is_globally_visible(kind_of(s->lsb[i])) == 1)
            for (uint32_t p = s->key_off[i]; p < s->key_off[i + 1]; ++p) hist[cur[s->key_ord[p]]++] = i;

    /* range commands in TxnId order */
    for (uint32_t i = 0; i < n; ++i) if (domain_of(s->lsb[i]) == 1) if (u32v_push(&rcmd, i)) goto done;
    size_t rc_first = 0;

    for (uint32_t i = 0; i < n; ++i) {
        int tk = witnesses_of(kind_of(s->lsb[i]));
        int64_t applied_before = s->applied_before ? (int64_t)s->applied_before[i]
                                                   : (int64_t)i - (int64_t)s->window;    /* j < i-W are applied */
        const ts_t sb_i = started_before(s, i);
        const uint32_t bound = bound_of(s, n, &sb_i, i);     /* candidates j < bound (= i: PreAccept) */
        const long p1 = p1_of(s, i);                       /* excluded (Accept: the txn itself) */
        lists.n = 0; lens.n = 0; heads.n = 0;
        u32v qkeys = {0};
        /* keys queried: own keys, or every key inside own ranges (CFKs that exist) */
        if (domain_of(s->lsb[i]) == 0) {
            for (uint32_t p = s->key_off[i]; p < s->key_off[i + 1]; ++p) if (u32v_push(&qkeys, s->key_ord[p])) goto done;
        } else {
            for (uint32_t r = s->rng_off[i]; r < s->rng_off[i + 1]; ++r)
                for (uint32_t key = s->rng_start[r] + 1; key <= s->rng_end[r] && key < nkeys; ++key)
                    if (hoff[key + 1] > hoff[key]) if (u32v_push(&qkeys, key)) goto done;
        }
        uint32_t kc = 0;
        for (uint32_t q = 0; q < qkeys.n; ++q) {
            uint32_t key = qkeys.p[q];
            uint32_t a = hoff[key], b = hoff[key + 1];
            uint32_t lo = a, hi = b;                      /* p = lower_bound(bound) */
            while (lo < hi) { uint32_t m = (lo + hi) / 2; if (hist[m] < bound) lo = m + 1; else hi = m; }
            uint32_t p = lo;
            uint32_t start = a;
            if (applied_before > 0) {
                uint32_t l2 = a, h2 = p;                  /* last entry < i-W */
                while (l2 < h2) { uint32_t m = (l2 + h2) / 2; if ((int64_t)hist[m] < applied_before) l2 = m + 1; else h2 = m; }
                long w = (long)l2 - 1;
                while (w >= (long)a && kind_of(s->lsb[hist[w]]) != K_WRITE) --w;
                if (w >= (long)a) start = (uint32_t)w;
            }
            if (s->floor && key > 0) {                    /* withRedundantBefore: entries < floor gone */
                uint32_t l2 = a, h2 = p;
                while (l2 < h2) { uint32_t m = (l2 + h2) / 2; if (hist[m] < s->floor[i]) l2 = m + 1; else h2 = m; }
                if (l2 > start) start = l2;
            }
            uint32_t before = (uint32_t)lists.n;
            for (uint32_t e = start; e < p; ++e)
                if (kinds_test(tk, kind_of(s->lsb[hist[e]])) && (p1 < 0 || hist[e] != (uint32_t)p1))
                    if (u32v_push(&lists, hist[e])) goto done;
            uint32_t c = (uint32_t)lists.n - before;
            if (c) { if (u32v_push(&lens, c) || u32v_push(&heads, key)) goto done; ++kc; }
        }
        free(qkeys.p);
        /* KeyDeps: keys = heads, values = sorted union, k2v = header + remapped body */
        uni.n = 0;
        for (size_t e = 0; e < lists.n; ++e) if (u32v_push(&uni, lists.p[e])) goto done;
        qsort(uni.p, uni.n, sizeof(uint32_t), cmp_u32);
        size_t un = 0;
        for (size_t e = 0; e < uni.n; ++e) if (un == 0 || uni.p[un - 1] != uni.p[e]) uni.p[un++] = uni.p[e];
        for (uint32_t q = 0; q < kc; ++q) if (u32v_push(&kd.keys_lo, heads.p[q])) goto done;
        for (size_t e = 0; e < un; ++e) if (u32v_push(&kd.vals, uni.p[e])) goto done;
        int32_t off = (int32_t)kc;
        for (uint32_t q = 0; q < kc; ++q) { off += (int32_t)lens.p[q]; if (i32v_push(&kd.k2v, off)) goto done; }
        for (size_t e = 0; e < lists.n; ++e) {
            uint32_t *f = (uint32_t *)bsearch(&lists.p[e], uni.p, un, sizeof(uint32_t), cmp_u32);
            if (i32v_push(&kd.k2v, (int32_t)(f - uni.p))) goto done;
        }
        if (mmo_close_txn(&kd)) goto done;

        /* RangeDeps: live witnessed range commands j in [i-W, i) whose ranges intersect */
        {
            mm_builder rb; mmb_init(&rb, NULL);
            /* collect (range code, txn) pairs then build canonical multimap directly */
            u32v rlo = {0}, rhi = {0}, rtx = {0};
            while (rc_first < rcmd.n && (int64_t)rcmd.p[rc_first] < applied_before) ++rc_first;   /* monotone in i */
            for (size_t c = rc_first; c < rcmd.n; ++c) {
                uint32_t j = rcmd.p[c];
                if (j >= bound) break;
                if (p1 >= 0 && j == (uint32_t)p1) continue;
                if (!kinds_test(tk, kind_of(s->lsb[j]))) continue;
                for (uint32_t a = s->rng_off[j]; a < s->rng_off[j + 1]; ++a) {
                    uint32_t rs = s->rng_start[a], re = s->rng_end[a];
                    int hit = 0;
                    if (domain_of(s->lsb[i]) == 0) {
                        uint32_t lo = s->key_off[i], hi = s->key_off[i + 1];   /* first key > rs */
                        while (lo < hi) { uint32_t m = (lo + hi) / 2; if (s->key_ord[m] <= rs) lo = m + 1; else hi = m; }
                        hit = lo < s->key_off[i + 1] && s->key_ord[lo] <= re;
                    } else {
                        for (uint32_t r = s->rng_off[i]; r < s->rng_off[i + 1] && !hit; ++r)
                            hit = range_intersects_range(rs, re, s->rng_start[r], s->rng_end[r]);
                    }
                    if (hit) { if (u32v_push(&rlo, rs) || u32v_push(&rhi, re) || u32v_push(&rtx, j)) goto done; }
                }
            }
            /* ranges sorted by (start,end); values per range are ascending txn (j ascending) */
            size_t m = rtx.n;
            uint32_t *ord = (uint32_t *)malloc((m ? m : 1) * sizeof(uint32_t));
            uint64_t *codes = (uint64_t *)malloc((m ? m : 1) * sizeof(uint64_t));
            if (!ord || !codes) { free(ord); free(codes); goto done; }
            for (size_t e = 0; e < m; ++e) codes[e] = ((uint64_t)rlo.p[e] << 32) | rhi.p[e];
            for (size_t e = 0; e < m; ++e) ord[e] = (uint32_t)e;
            /* stable insertion by code (m is small) */
            for (size_t e = 1; e < m; ++e) {
                uint32_t x = ord[e]; size_t f = e;
                while (f > 0 && codes[ord[f - 1]] > codes[x]) { ord[f] = ord[f - 1]; --f; }
                ord[f] = x;
            }
            u32v rv = {0};
            for (size_t e = 0; e < m; ++e) if (u32v_push(&rv, rtx.p[e])) goto done;
            qsort(rv.p, rv.n, sizeof(uint32_t), cmp_u32);
            size_t rvn = 0;
            for (size_t e = 0; e < rv.n; ++e) if (rvn == 0 || rv.p[rvn - 1] != rv.p[e]) rv.p[rvn++] = rv.p[e];
            size_t nk = 0;
            for (size_t e = 0; e < m; ++e) if (e == 0 || codes[ord[e]] != codes[ord[e - 1]]) ++nk;
            size_t hdr = rd.k2v.n;
            for (size_t e = 0; e < nk; ++e) if (i32v_push(&rd.k2v, 0)) goto done;
            size_t ki = 0;
            for (size_t e = 0; e < m; ++e) {
                if (e == 0 || codes[ord[e]] != codes[ord[e - 1]]) {
                    if (u32v_push(&rd.keys_lo, rlo.p[ord[e]]) || u32v_push(&rd.keys_hi, rhi.p[ord[e]])) goto done;
                    if (e > 0) { rd.k2v.p[hdr + ki] = (int32_t)(rd.k2v.n - hdr); ++ki; }
                }
                uint32_t *f = (uint32_t *)bsearch(&rtx.p[ord[e]], rv.p, rvn, sizeof(uint32_t), cmp_u32);
                if (i32v_push(&rd.k2v, (int32_t)(f - rv.p))) goto done;
            }
            if (nk) rd.k2v.p[hdr + ki] = (int32_t)(rd.k2v.n - hdr);
            for (size_t e = 0; e < rvn; ++e) if (u32v_push(&rd.vals, rv.p[e])) goto done;
            if (mmo_close_txn(&rd)) goto done;
            free(ord); free(codes); free(rv.p); free(rlo.p); free(rhi.p); free(rtx.p);
            mmb_free(&rb);
        }
    }
    if (alloc_out(out, &kd, &rd, n)) goto done;
    rc = 0;
done:
    free(hoff); free(hist); free(cur);
    free(lists.p); free(lens.p); free(heads.p); free(uni.p); free(rcmd.p);
    mmo_free(&kd); mmo_free(&rd);
    return rc;
}

/* ------------------------------------------------------------------------------------------
 * Primitive entry points for the restated reference property tests
 * ------------------------------------------------------------------------------------------ */
int or_keydeps_build(uint32_t nadds, const uint32_t *keys, const uint32_t *vals,
                     uint32_t ntbl, const uint64_t *tbl_msb, const uint64_t *tbl_lsb, const int32_t *tbl_node,
                     or_deps *out)
{
    ts_t *tbl = (ts_t *)malloc((size_t)(ntbl ? ntbl : 1) * sizeof(ts_t));
    if (!tbl) return -1;
    for (uint32_t i = 0; i < ntbl; ++i) { tbl[i].msb = tbl_msb[i]; tbl[i].lsb = tbl_lsb[i]; tbl[i].node = tbl_node[i]; }
    mm_builder b; mm_out kd, rd;
    int rc = -1;
    mmb_init(&b, tbl);
    if (mmo_init(&kd) || mmo_init(&rd)) goto done;
    for (uint32_t a = 0; a < nadds; ++a) if (mmb_add(&b, keys[a], vals[a])) goto done;
    if (mmb_build(&b, &kd, 0)) goto done;
    if (mmo_close_txn(&rd)) goto done;
    if (alloc_out(out, &kd, &rd, 1)) goto done;
    rc = 0;
done:
    mmb_free(&b); mmo_free(&kd); mmo_free(&rd); free(tbl);
    return rc;
}

/* linearUnion general path (RelationMultiMap.java:733-801).  The pass-through paths
 * (:583-730) return one input unchanged only when it already equals the union, so the
 * value-level result is the general merge's in every case. */
int or_keydeps_union(const or_deps *x, uint32_t a, const or_deps *y, uint32_t b,
                     const uint64_t *tbl_msb, const uint64_t *tbl_lsb, const int32_t *tbl_node,
                     or_deps *out)
{
    const uint32_t *lk = x->kd_keys + x->kd_key_off[a], *rk = y->kd_keys + y->kd_key_off[b];
    uint32_t lkn = x->kd_key_off[a + 1] - x->kd_key_off[a], rkn = y->kd_key_off[b + 1] - y->kd_key_off[b];
    const uint32_t *lv = x->kd_vals + x->kd_val_off[a], *rv = y->kd_vals + y->kd_val_off[b];
    uint32_t lvn = x->kd_val_off[a + 1] - x->kd_val_off[a], rvn = y->kd_val_off[b + 1] - y->kd_val_off[b];
    const int32_t *l = x->kd_k2v + x->kd_k2v_off[a], *r = y->kd_k2v + y->kd_k2v_off[b];
    mm_out kd, rd;
    int rc = -1;
    uint32_t *ov = NULL, *rl = NULL, *rr = NULL;
    if (mmo_init(&kd) || mmo_init(&rd)) goto done;
    /* SortedArrays.linearUnion of values (left wins on ties) */
    ov = (uint32_t *)malloc(((size_t)lvn + rvn + 1) * sizeof(uint32_t));
    rl = (uint32_t *)malloc(((size_t)lvn + 1) * sizeof(uint32_t));
    rr = (uint32_t *)malloc(((size_t)rvn + 1) * sizeof(uint32_t));
    if (!ov || !rl || !rr) goto done;
    uint32_t i = 0, j = 0, o = 0;
    while (i < lvn && j < rvn) {
        int c = or_ts_compare(tbl_msb[lv[i]], tbl_lsb[lv[i]], tbl_node[lv[i]], tbl_msb[rv[j]], tbl_lsb[rv[j]], tbl_node[rv[j]]);
        if (c == 0) { rl[i++] = o; rr[j++] = o; ov[o++] = lv[i - 1]; }
        else if (c < 0) { rl[i++] = o; ov[o++] = lv[i - 1]; }
        else { rr[j++] = o; ov[o++] = rv[j - 1]; }
    }
    while (i < lvn) { rl[i++] = o; ov[o++] = lv[i - 1]; }
    while (j < rvn) { rr[j++] = o; ov[o++] = rv[j - 1]; }
    for (uint32_t v = 0; v < o; ++v) if (u32v_push(&kd.vals, ov[v])) goto done;
    /* keys union + per-key union of remapped indices */
    uint32_t lki = 0, rki = 0, lp = lkn, rp = rkn;
    u32v okeys = {0};
    i32v body = {0}; i32v hdr = {0};
    while (lki < lkn || rki < rkn) {
        int which = (lki < lkn && rki < rkn) ? (lk[lki] < rk[rki] ? -1 : lk[lki] > rk[rki] ? 1 : 0) : (lki < lkn ? -1 : 1);
        if (which <= 0 && which != 0) {
            if (u32v_push(&okeys, lk[lki])) goto done;
            while (lp < (uint32_t)l[lki]) if (i32v_push(&body, (int32_t)rl[l[lp++]])) goto done;
            ++lki;
        } else if (which > 0) {
            if (u32v_push(&okeys, rk[rki])) goto done;
            while (rp < (uint32_t)r[rki]) if (i32v_push(&body, (int32_t)rr[r[rp++]])) goto done;
            ++rki;
        } else {
            if (u32v_push(&okeys, lk[lki])) goto done;
            while (lp < (uint32_t)l[lki] && rp < (uint32_t)r[rki]) {
                int32_t nl = (int32_t)rl[l[lp]], nr = (int32_t)rr[r[rp]];
                if (nl <= nr) { if (i32v_push(&body, nl)) goto done; lp++; if (nl == nr) rp++; }
                else { if (i32v_push(&body, nr)) goto done; rp++; }
            }
            while (lp < (uint32_t)l[lki]) if (i32v_push(&body, (int32_t)rl[l[lp++]])) goto done;
            while (rp < (uint32_t)r[rki]) if (i32v_push(&body, (int32_t)rr[r[rp++]])) goto done;
            ++lki; ++rki;
        }
        if (i32v_push(&hdr, (int32_t)body.n)) goto done;
    }
    for (size_t k = 0; k < okeys.n; ++k) if (u32v_push(&kd.keys_lo, okeys.p[k])) goto done;
    for (size_t k = 0; k < hdr.n; ++k) if (i32v_push(&kd.k2v, hdr.p[k] + (int32_t)okeys.n)) goto done;
    for (size_t k = 0; k < body.n; ++k) if (i32v_push(&kd.k2v, body.p[k])) goto done;
    free(okeys.p); free(body.p); free(hdr.p);
    if (mmo_close_txn(&kd) || mmo_close_txn(&rd)) goto done;
    if (alloc_out(out, &kd, &rd, 1)) goto done;
    rc = 0;
done:
    free(ov); free(rl); free(rr);
    mmo_free(&kd); mmo_free(&rd);
    return rc;
}

uint32_t or_stab_key(uint32_t nr, const uint32_t *rs, const uint32_t *re, uint32_t key, uint32_t *out)
{
    uint32_t c = 0;
    for (uint32_t i = 0; i < nr; ++i) if (range_intersects_key(rs[i], re[i], key)) out[c++] = i;
    return c;
}

/* WaitingOn + levelling under "all STABLE, executeAt = txnId, none
 * applied" (config 5): Command.WaitingOn.Update (local/Command.java:1426-1437) sets bits
 * [0, |rangeDeps.txnIds|) for range deps and [R, R + |keyDeps.keys|) for key deps;
 * Commands.updateWaitingOn (local/Commands.java:755-830) clears none because every dep j < i
 * executes before i and none is applied.  Level: 0 if no dep executes before, else 1 + max. */
int or_waiting_on(const or_deps *d, uint32_t n, uint32_t *level, uint32_t *wo_off, uint64_t **wo_words)
{
    size_t total = 0;
    wo_off[0] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t bits = (d->rd_val_off[i + 1] - d->rd_val_off[i]) + (d->kd_key_off[i + 1] - d->kd_key_off[i]);
        total += (bits + 63) / 64;
        wo_off[i + 1] = (uint32_t)total;
    }
    uint64_t *w = (uint64_t *)calloc(total ? total : 1, sizeof(uint64_t));
    if (!w) return -1;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t bits = (d->rd_val_off[i + 1] - d->rd_val_off[i]) + (d->kd_key_off[i + 1] - d->kd_key_off[i]);
        for (uint32_t b = 0; b < bits; ++b) w[wo_off[i] + b / 64] |= 1ULL << (b & 63);
        uint32_t lv = 0;
        for (uint32_t v = d->kd_val_off[i]; v < d->kd_val_off[i + 1]; ++v) if (level[d->kd_vals[v]] + 1 > lv) lv = level[d->kd_vals[v]] + 1;
        for (uint32_t v = d->rd_val_off[i]; v < d->rd_val_off[i + 1]; ++v) if (level[d->rd_vals[v]] + 1 > lv) lv = level[d->rd_vals[v]] + 1;
        level[i] = lv;
    }
    *wo_words = w;
    return 0;
}

int or_levels_csr(uint32_t n, const uint32_t *pred_off, const uint32_t *preds, uint32_t *level)
{
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t lv = 0;
        for (uint32_t q = pred_off[i]; q < pred_off[i + 1]; ++q) {
            const uint32_t p = preds[q];
            if (p >= i) return -1;
            if (level[p] + 1 > lv) lv = level[p] + 1;
        }
        level[i] = lv;
    }
    return 0;
}

/* Commands.initialiseWaitingOn + the initial updateWaitingOn (see oracle.h).  Txn.Kind.awaitsOnlyDeps
 * (primitives/Txn.java:211-214): ExclusiveSyncPoint, EphemeralRead. */
int or_initialise_waiting_on(const or_deps *d, uint32_t n, const uint64_t *lsb, const uint64_t *own_msb,
                             const uint64_t *own_lsb, const int32_t *own_node, const uint8_t *status,
                             const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode,
                             uint32_t *wo_off, uint64_t **wo_words, uint64_t **aoi_words)
{
    enum { COMMITTED = 4, APPLIED = 6, INVALID_OR_TRUNCATED = 7 };
    size_t total = 0;
    wo_off[0] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t bits = (d->rd_val_off[i + 1] - d->rd_val_off[i]) + (d->kd_key_off[i + 1] - d->kd_key_off[i]);
        total += (bits + 63) / 64;
        wo_off[i + 1] = (uint32_t)total;
    }
    uint64_t *w = (uint64_t *)calloc(total ? total : 1, sizeof(uint64_t));
    uint64_t *a = (uint64_t *)calloc(total ? total : 1, sizeof(uint64_t));
    if (!w || !a) { free(w); free(a); return -1; }
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t kind = (uint32_t)(lsb[i] >> 1) & 7u;
        const int awaits_only_deps = kind == 4u || kind == 2u;      /* ExclusiveSyncPoint, EphemeralRead */
        const int range_domain = (int)(lsb[i] & 1u);                 /* Routable.Domain.Range */
        const uint32_t r0 = d->rd_val_off[i], R = d->rd_val_off[i + 1] - r0;
        const uint32_t K = d->kd_key_off[i + 1] - d->kd_key_off[i];
        uint64_t *wi = w + wo_off[i], *ai = a + wo_off[i];
        /* WaitingOn.Update(txnId, deps): the waiting set starts with every txnId and key */
        for (uint32_t b = 0; b < R + K; ++b) wi[b / 64] |= 1ULL << (b & 63);
        /* forEachWaitingOnId: txnId bits in reverse order */
        for (uint32_t j = R; j-- > 0;) {
            const uint32_t g = d->rd_vals[r0 + j];
            const uint32_t st = status[g];
            if (st < COMMITTED) continue;                            /* !hasBeen(PreCommitted) */
            const uint64_t bit = 1ULL << (j & 63);
            if (st >= INVALID_OR_TRUNCATED) {                        /* hasBeen(Truncated): setAppliedOrInvalidated */
                if (wi[j / 64] & bit) { wi[j / 64] &= ~bit; if (range_domain) ai[j / 64] |= bit; }
            } else if (!awaits_only_deps &&
                       or_ts_compare(emsb[g], elsb[g], enode[g], own_msb[i], own_lsb[i], own_node[i]) > 0) {
                wi[j / 64] &= ~bit;                                  /* executes after us: removeWaitingOn */
            } else if (st == APPLIED) {                              /* setAppliedAndPropagate */
                if (wi[j / 64] & bit) { wi[j / 64] &= ~bit; if (range_domain) ai[j / 64] |= bit; }
            }
        }
    }
    *wo_words = w;
    *aoi_words = a;
    return 0;
}

/* Event-driven restatement of execution readiness (validates the levelling abstraction, SURVEY.md
 * §8a a13): every txn starts with its WaitingOn bits (Commands.initialiseWaitingOn,
 * local/Commands.java:735-753).  A range-dep bit clears when that dep applies
 * (Commands.updateWaitingOn -> WaitingOn.setAppliedOrInvalidated, :755-830); a key bit clears when
 * every dep of that key executing before this txn has applied (CommandsForKey.notify,
 * local/CommandsForKey.java:1501-1635 -> Commands.removeWaitingOnKeyAndMaybeExecute, :859-876).
 * A txn with no bits left executes (maybeExecute, :656-733).  Synchronous rounds: all txns ready at
 * round r execute and apply together; round[i] = r.  Independent of or_waiting_on's recurrence. */
int or_waiting_on_events(const or_deps *d, uint32_t n, uint32_t *round_out)
{
    uint32_t *bits_left = (uint32_t *)calloc(n ? n : 1, sizeof(uint32_t));
    uint32_t *radj_off = (uint32_t *)calloc((size_t)n + 1, sizeof(uint32_t));
    uint32_t nkslot = d->kd_key_off[n];
    uint32_t *slot_left = (uint32_t *)calloc(nkslot ? nkslot : 1, sizeof(uint32_t));
    if (!bits_left || !radj_off || !slot_left) { free(bits_left); free(radj_off); free(slot_left); return -1; }
    /* reverse edges: dep j -> (waiter i, slot); slot >= 0 key slot (global index), ~r range bit */
    size_t E = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t kc = d->kd_key_off[i + 1] - d->kd_key_off[i];
        const int32_t *k2v = d->kd_k2v + d->kd_k2v_off[i];
        for (uint32_t q = 0; q < kc; ++q) {
            uint32_t b = q == 0 ? kc : (uint32_t)k2v[q - 1], e = (uint32_t)k2v[q];
            for (uint32_t x = b; x < e; ++x) radj_off[d->kd_vals[d->kd_val_off[i] + (uint32_t)k2v[x]] + 1]++;
            slot_left[d->kd_key_off[i] + q] = e - b;
            E += e - b;
        }
        for (uint32_t v = d->rd_val_off[i]; v < d->rd_val_off[i + 1]; ++v) { radj_off[d->rd_vals[v] + 1]++; ++E; }
        bits_left[i] = kc + (d->rd_val_off[i + 1] - d->rd_val_off[i]);
    }
    for (uint32_t j = 0; j < n; ++j) radj_off[j + 1] += radj_off[j];
    uint32_t *rw = (uint32_t *)malloc((E ? E : 1) * sizeof(uint32_t));
    int64_t *rs = (int64_t *)malloc((E ? E : 1) * sizeof(int64_t));
    uint32_t *fill = (uint32_t *)malloc(((size_t)n + 1) * sizeof(uint32_t));
    uint32_t *frontier = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    uint32_t *nextf = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    if (!rw || !rs || !fill || !frontier || !nextf) {
        free(bits_left); free(radj_off); free(slot_left); free(rw); free(rs); free(fill); free(frontier); free(nextf);
        return -1;
    }
    memcpy(fill, radj_off, ((size_t)n + 1) * sizeof(uint32_t));
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t kc = d->kd_key_off[i + 1] - d->kd_key_off[i];
        const int32_t *k2v = d->kd_k2v + d->kd_k2v_off[i];
        for (uint32_t q = 0; q < kc; ++q) {
            uint32_t b = q == 0 ? kc : (uint32_t)k2v[q - 1], e = (uint32_t)k2v[q];
            for (uint32_t x = b; x < e; ++x) {
                uint32_t j = d->kd_vals[d->kd_val_off[i] + (uint32_t)k2v[x]];
                rw[fill[j]] = i; rs[fill[j]] = (int64_t)(d->kd_key_off[i] + q); fill[j]++;
            }
        }
        for (uint32_t v = d->rd_val_off[i]; v < d->rd_val_off[i + 1]; ++v) {
            uint32_t j = d->rd_vals[v];
            rw[fill[j]] = i; rs[fill[j]] = -1; fill[j]++;
        }
    }
    uint32_t nf = 0;
    for (uint32_t i = 0; i < n; ++i) if (bits_left[i] == 0) frontier[nf++] = i;
    uint32_t done = 0, r = 0;
    while (nf) {
        uint32_t nn = 0;
        for (uint32_t f = 0; f < nf; ++f) round_out[frontier[f]] = r;     /* execute + apply */
        for (uint32_t f = 0; f < nf; ++f) {
            uint32_t j = frontier[f];
            for (uint32_t x = radj_off[j]; x < radj_off[j + 1]; ++x) {
                uint32_t i = rw[x];
                int clear = 1;
                if (rs[x] >= 0) clear = --slot_left[rs[x]] == 0;
                if (clear && --bits_left[i] == 0) nextf[nn++] = i;
            }
        }
        done += nf;
        uint32_t *t = frontier; frontier = nextf; nextf = t;
        nf = nn;
        ++r;
    }
    free(bits_left); free(radj_off); free(slot_left); free(rw); free(rs); free(fill); free(frontier); free(nextf);
    return done == n ? 0 : -7;   /* -7: a txn never became ready (cycle / missing dep) */
}

/* Execution readiness restated from the CommandsForKey side, independent of
 * the deps values of managed txns: each key keeps a CFK of the managed txns on it (key domain and
 * Kind.isGloballyVisible, SafeCommandStore.java:219-233), all STABLE with executeAt = txnId.
 *  - managed txn t clears its key-k WaitingOn bit when CommandsForKey.notify (:1512-1635) finds
 *    expectMissingCount == |missing| at t: the unapplied committed txns before t in executeAt order,
 *    counted per kind (Write: reads + writes; Read: writes; SyncPoints: all three), against its
 *    missing[] -- empty here, because every txn is registered STABLE in TxnId order and update()
 *    elides committed txns from missing (:1103-1109).  notify runs over [next, nextWrite] of the key
 *    (:1199-1203) whenever a txn on it applies, and once at registration (:1176-1186);
 *  - unmanaged txns (range domain, EphemeralRead) go through registerUnmanaged (:1406-1498): key k
 *    is pending until every committed txn on k executing at or before waitingUntil (the max
 *    executeAt of its deps on k) has applied, released by notifyUnmanaged(APPLY, next.executeAt)
 *    (:1211-1212);
 *  - a range-dep bit clears when that dep applies (Commands.updateWaitingOn, Commands.java:755-830).
 * Synchronous rounds as or_waiting_on_events.  0 ok, -7 stuck, -8 deps name a txn the CFK lacks. */
int or_levels_cfk(const or_stream *s, const or_deps *d, uint32_t *round_out)
{
    const uint32_t n = s->n;
    int rc = 0;
    uint32_t nkeys = 0;
    for (uint32_t x = 0; x < s->key_off[n]; ++x) if (s->key_ord[x] + 1 > nkeys) nkeys = s->key_ord[x] + 1;
    for (uint32_t x = 0; x < d->kd_key_off[n]; ++x) if (d->kd_keys[x] + 1 > nkeys) nkeys = d->kd_keys[x] + 1;
    uint8_t *managed = (uint8_t *)calloc(n ? n : 1, 1), *applied = (uint8_t *)calloc(n ? n : 1, 1);
    uint8_t *dirty = (uint8_t *)calloc(nkeys ? nkeys : 1, 1);
    uint32_t *cfk_off = (uint32_t *)calloc((size_t)nkeys + 1, sizeof(uint32_t));
    uint32_t *nextp = (uint32_t *)calloc(nkeys ? nkeys : 1, sizeof(uint32_t));
    uint32_t *dlist = (uint32_t *)calloc(nkeys ? nkeys : 1, sizeof(uint32_t));
    uint32_t *pend_off = (uint32_t *)calloc((size_t)nkeys + 1, sizeof(uint32_t));
    uint32_t *bits_left = (uint32_t *)calloc(n ? n : 1, sizeof(uint32_t));
    uint32_t *radj_off = (uint32_t *)calloc((size_t)n + 1, sizeof(uint32_t));
    uint32_t *frontier = (uint32_t *)malloc((n ? n : 1) * sizeof(uint32_t));
    uint32_t nslot = d->kd_key_off[n];
    uint8_t *slot_clear = (uint8_t *)calloc(nslot ? nslot : 1, 1);
    uint32_t *cfk = NULL, *fill = NULL, *pend_slot = NULL, *pend_txn = NULL, *pend_until = NULL, *pend_head = NULL,
             *rw = NULL;
    if (!managed || !applied || !dirty || !cfk_off || !nextp || !dlist || !pend_off || !bits_left || !radj_off || !frontier ||
        !slot_clear) { rc = -1; goto out; }
    for (uint32_t i = 0; i < n; ++i) {
        managed[i] = domain_of(s->lsb[i]) == 0 && is_globally_visible(kind_of(s->lsb[i])) == 1;
        if (managed[i])
            for (uint32_t x = s->key_off[i]; x < s->key_off[i + 1]; ++x) cfk_off[s->key_ord[x] + 1]++;
        else
            for (uint32_t x = d->kd_key_off[i]; x < d->kd_key_off[i + 1]; ++x) pend_off[d->kd_keys[x] + 1]++;
        for (uint32_t v = d->rd_val_off[i]; v < d->rd_val_off[i + 1]; ++v) radj_off[d->rd_vals[v] + 1]++;
        bits_left[i] = (d->kd_key_off[i + 1] - d->kd_key_off[i]) + (d->rd_val_off[i + 1] - d->rd_val_off[i]);
    }
    for (uint32_t k = 0; k < nkeys; ++k) { cfk_off[k + 1] += cfk_off[k]; pend_off[k + 1] += pend_off[k]; }
    for (uint32_t j = 0; j < n; ++j) radj_off[j + 1] += radj_off[j];
    cfk = (uint32_t *)malloc(((size_t)cfk_off[nkeys] + 1) * sizeof(uint32_t));
    fill = (uint32_t *)malloc(((size_t)(nkeys > n ? nkeys : n) + 1) * sizeof(uint32_t));
    pend_slot = (uint32_t *)malloc(((size_t)pend_off[nkeys] + 1) * sizeof(uint32_t));
    pend_until = (uint32_t *)malloc(((size_t)pend_off[nkeys] + 1) * sizeof(uint32_t));
    pend_txn = (uint32_t *)malloc(((size_t)pend_off[nkeys] + 1) * sizeof(uint32_t));
    pend_head = (uint32_t *)calloc(nkeys ? nkeys : 1, sizeof(uint32_t));
    rw = (uint32_t *)malloc(((size_t)radj_off[n] + 1) * sizeof(uint32_t));
    if (!cfk || !fill || !pend_slot || !pend_txn || !pend_until || !pend_head || !rw) { rc = -1; goto out; }
    /* CFK txns[] per key in TxnId (= executeAt) order */
    memcpy(fill, cfk_off, (size_t)nkeys * sizeof(uint32_t));
    for (uint32_t i = 0; i < n; ++i)
        if (managed[i])
            for (uint32_t x = s->key_off[i]; x < s->key_off[i + 1]; ++x) cfk[fill[s->key_ord[x]]++] = i;
    /* registerUnmanaged: one pending APPLY record per (txn, key of its keyDeps), waitingUntil = the
     * max executeAt of its deps on the key (all committed, all before it: :1427-1449) */
    memcpy(fill, pend_off, (size_t)nkeys * sizeof(uint32_t));
    for (uint32_t i = 0; i < n; ++i) {
        if (managed[i]) continue;
        const int32_t *k2v = d->kd_k2v + d->kd_k2v_off[i];
        uint32_t kc = d->kd_key_off[i + 1] - d->kd_key_off[i];
        for (uint32_t q = 0; q < kc; ++q) {
            uint32_t b = q == 0 ? kc : (uint32_t)k2v[q - 1], e = (uint32_t)k2v[q], until = 0;
            for (uint32_t x = b; x < e; ++x) {
                uint32_t j = d->kd_vals[d->kd_val_off[i] + (uint32_t)k2v[x]];
                if (j > until) until = j;
            }
            uint32_t k = d->kd_keys[d->kd_key_off[i] + q];
            pend_slot[fill[k]] = d->kd_key_off[i] + q;
            pend_txn[fill[k]] = i;
            pend_until[fill[k]++] = until;
        }
    }
    /* pending records of a key in waitingUntil order (released as a prefix) */
    for (uint32_t k = 0; k < nkeys; ++k)
        for (uint32_t a = pend_off[k] + 1; a < pend_off[k + 1]; ++a)
            for (uint32_t b = a; b > pend_off[k] && pend_until[b - 1] > pend_until[b]; --b) {
                uint32_t t = pend_until[b]; pend_until[b] = pend_until[b - 1]; pend_until[b - 1] = t;
                t = pend_slot[b]; pend_slot[b] = pend_slot[b - 1]; pend_slot[b - 1] = t;
                t = pend_txn[b]; pend_txn[b] = pend_txn[b - 1]; pend_txn[b - 1] = t;
            }
    memcpy(fill, radj_off, (size_t)n * sizeof(uint32_t));
    for (uint32_t i = 0; i < n; ++i)
        for (uint32_t v = d->rd_val_off[i]; v < d->rd_val_off[i + 1]; ++v) rw[fill[d->rd_vals[v]]++] = i;
    for (uint32_t k = 0; k < nkeys; ++k) { nextp[k] = cfk_off[k]; pend_head[k] = pend_off[k]; dirty[k] = 1; }

    uint32_t done = 0, r = 0, nf = 0, ndirty = nkeys;
    for (uint32_t k = 0; k < nkeys; ++k) dlist[k] = k;
    for (;;) {
        /* CFK side: notify + notifyUnmanaged on every key whose state changed */
        for (uint32_t dk = 0; dk < ndirty; ++dk) {
            const uint32_t k = dlist[dk];
            dirty[k] = 0;
            while (nextp[k] < cfk_off[k + 1] && applied[cfk[nextp[k]]]) nextp[k]++;
            uint32_t ur = 0, uw = 0, usp = 0;
            for (uint32_t p = nextp[k]; p < cfk_off[k + 1]; ++p) {
                uint32_t t = cfk[p];
                if (applied[t]) continue;
                int kind = kind_of(s->lsb[t]);
                uint32_t expect = kind == K_READ ? uw : kind == K_WRITE ? uw + ur : uw + ur + usp;
                if (expect == 0) {           /* |missing| == 0: removeWaitingOn(t, key) */
                    const uint32_t *ks = d->kd_keys + d->kd_key_off[t];
                    uint32_t lo = 0, hi = d->kd_key_off[t + 1] - d->kd_key_off[t];
                    while (lo < hi) { uint32_t m = (lo + hi) / 2; if (ks[m] < k) lo = m + 1; else hi = m; }
                    uint32_t slot = d->kd_key_off[t] + lo;
                    if (lo < d->kd_key_off[t + 1] - d->kd_key_off[t] && ks[lo] == k && !slot_clear[slot]) {
                        slot_clear[slot] = 1;
                        if (--bits_left[t] == 0) frontier[nf++] = t;
                    }
                }
                if (kind == K_WRITE) { ++uw; break; }          /* notify stops at nextWrite */
                if (kind == K_READ) ++ur; else ++usp;
            }
            uint32_t next = nextp[k] < cfk_off[k + 1] ? cfk[nextp[k]] : UINT32_MAX;
            while (pend_head[k] < pend_off[k + 1] && pend_until[pend_head[k]] < next) {
                uint32_t slot = pend_slot[pend_head[k]], t = pend_txn[pend_head[k]++];
                if (!slot_clear[slot]) {
                    slot_clear[slot] = 1;
                    if (--bits_left[t] == 0) frontier[nf++] = t;
                }
            }
        }
        ndirty = 0;
        if (r == 0)
            for (uint32_t i = 0; i < n; ++i)
                if (d->kd_key_off[i + 1] == d->kd_key_off[i] && d->rd_val_off[i + 1] == d->rd_val_off[i]) frontier[nf++] = i;
        if (!nf) break;
        /* execute + apply this round's frontier */
        uint32_t cur = nf;
        for (uint32_t f = 0; f < cur; ++f) {
            uint32_t j = frontier[f];
            round_out[j] = r;
            applied[j] = 1;
            if (managed[j])
                for (uint32_t x = s->key_off[j]; x < s->key_off[j + 1]; ++x)
                    if (!dirty[s->key_ord[x]]) { dirty[s->key_ord[x]] = 1; dlist[ndirty++] = s->key_ord[x]; }
        }
        done += cur;
        nf = 0;
        /* range-dep bits (frontier is reused for the next round: copy out this round's first) */
        memcpy(fill, frontier, (size_t)cur * sizeof(uint32_t));
        for (uint32_t f = 0; f < cur; ++f) {
            uint32_t j = fill[f];
            for (uint32_t x = radj_off[j]; x < radj_off[j + 1]; ++x)
                if (--bits_left[rw[x]] == 0) frontier[nf++] = rw[x];
        }
        ++r;
    }
    rc = done == n ? 0 : -7;
out:
    free(managed); free(applied); free(dirty); free(cfk_off); free(nextp); free(dlist); free(pend_off); free(bits_left);
    free(radj_off); free(frontier); free(slot_clear); free(cfk); free(fill); free(pend_slot); free(pend_txn);
    free(pend_until); free(pend_head); free(rw);
    return rc;
}

/* ==========================================================================================
 * Deps-set operations over every txn of an or_deps set.
 * Values are indices into one TxnId table sorted ascending (the stream the deps were computed
 * from, whose order the stream drivers validate), so Timestamp.compareTo order == index order.
 * Keys are u64 codes as in the builder: a key ordinal, or start<<32|end for a range (Range.compare
 * order, Range.java:310-317).
 * ========================================================================================== */

typedef struct {
    uint64_t *keys; uint32_t nk;
    const uint32_t *vals; uint32_t nv;
    const int32_t *k2v; uint32_t nx;        /* keysToValues: nk end offsets + body */
} mm_view;

static int view_of(const or_deps *d, uint32_t i, int range, mm_view *v)
{
    if (!range) {
        v->nk = d->kd_key_off[i + 1] - d->kd_key_off[i];
        v->vals = d->kd_vals + d->kd_val_off[i]; v->nv = d->kd_val_off[i + 1] - d->kd_val_off[i];
        v->k2v = d->kd_k2v + d->kd_k2v_off[i]; v->nx = d->kd_k2v_off[i + 1] - d->kd_k2v_off[i];
    } else {
        v->nk = d->rd_rng_off[i + 1] - d->rd_rng_off[i];
        v->vals = d->rd_vals + d->rd_val_off[i]; v->nv = d->rd_val_off[i + 1] - d->rd_val_off[i];
        v->k2v = d->rd_r2v + d->rd_r2v_off[i]; v->nx = d->rd_r2v_off[i + 1] - d->rd_r2v_off[i];
    }
    v->keys = (uint64_t *)malloc(((size_t)v->nk + 1) * sizeof(uint64_t));
    if (!v->keys) return -1;
    for (uint32_t a = 0; a < v->nk; ++a)
        v->keys[a] = range ? ((uint64_t)d->rd_rng_start[d->rd_rng_off[i] + a] << 32 | d->rd_rng_end[d->rd_rng_off[i] + a])
                           : d->kd_keys[d->kd_key_off[i] + a];
    return 0;
}

/* append one multimap (keys, vals, keysToValues verbatim) to o */
static int mmo_emit(mm_out *o, int range, const uint64_t *keys, uint32_t nk, const uint32_t *vals, uint32_t nv,
                    const int32_t *k2v, uint32_t nx)
{
    for (uint32_t a = 0; a < nk; ++a) {
        if (u32v_push(&o->keys_lo, range ? (uint32_t)(keys[a] >> 32) : (uint32_t)keys[a])) return -1;
        if (range && u32v_push(&o->keys_hi, (uint32_t)keys[a])) return -1;
    }
    for (uint32_t v = 0; v < nv; ++v) if (u32v_push(&o->vals, vals[v])) return -1;
    for (uint32_t x = 0; x < nx; ++x) if (i32v_push(&o->k2v, k2v[x])) return -1;
    return mmo_close_txn(o);
}

static uint32_t body_start(const int32_t *k2v, uint32_t nk, uint32_t a) { return a == 0 ? nk : (uint32_t)k2v[a - 1]; }

/* RelationMultiMap.linearUnion (utils/RelationMultiMap.java:561-816) of two multimaps: values are
 * SortedArrays.linearUnion'd (utils/SortedArrays.java:152-281, left wins on ties), keys are unioned
 * in key order and each key's list is the union of both sides' indices remapped into the union
 * (remapToSuperset, :1197-1223).  The pass-through branches (:583-730) return one input only when
 * it already equals the union, so this is the value-level result in every case.  isEmpty() of
 * either side returns the other (KeyDeps.with, KeyDeps.java:238-241; RangeDeps.with :567-570). */
static int mm_union2(const mm_view *l, const mm_view *r, uint64_t **ok, uint32_t *onk, u32v *ov, i32v *ox)
{
    const mm_view *only = NULL;
    if (l->nx == l->nk || r->nx == r->nk) only = l->nx == l->nk ? r : l;
    ov->n = 0; ox->n = 0;
    *ok = (uint64_t *)malloc(((size_t)l->nk + r->nk + 1) * sizeof(uint64_t));
    if (!*ok) return -1;
    if (only) {
        memcpy(*ok, only->keys, (size_t)only->nk * sizeof(uint64_t)); *onk = only->nk;
        for (uint32_t v = 0; v < only->nv; ++v) if (u32v_push(ov, only->vals[v])) return -1;
        for (uint32_t x = 0; x < only->nx; ++x) if (i32v_push(ox, only->k2v[x])) return -1;
        return 0;
    }
    uint32_t *rl = (uint32_t *)malloc(((size_t)l->nv + 1) * 4), *rr = (uint32_t *)malloc(((size_t)r->nv + 1) * 4);
    i32v body = {0};
    int rc = -1;
    if (!rl || !rr) goto done;
    {
        uint32_t i = 0, j = 0, o = 0;
        while (i < l->nv || j < r->nv) {
            if (j == r->nv || (i < l->nv && l->vals[i] < r->vals[j])) { rl[i] = o; if (u32v_push(ov, l->vals[i++])) goto done; }
            else if (i == l->nv || r->vals[j] < l->vals[i]) { rr[j] = o; if (u32v_push(ov, r->vals[j++])) goto done; }
            else { rl[i] = rr[j] = o; if (u32v_push(ov, l->vals[i])) goto done; ++i; ++j; }
            ++o;
        }
    }
    {
        uint32_t a = 0, b = 0, nk = 0;
        uint32_t *hdr = (uint32_t *)malloc(((size_t)l->nk + r->nk + 1) * 4);
        if (!hdr) goto done;
        while (a < l->nk || b < r->nk) {
            int which = a == l->nk ? 1 : b == r->nk ? -1 : (l->keys[a] < r->keys[b] ? -1 : l->keys[a] > r->keys[b] ? 1 : 0);
            uint32_t lp = 0, le = 0, rp = 0, re = 0;
            if (which <= 0) { lp = body_start(l->k2v, l->nk, a); le = (uint32_t)l->k2v[a]; }
            if (which >= 0) { rp = body_start(r->k2v, r->nk, b); re = (uint32_t)r->k2v[b]; }
            (*ok)[nk] = which <= 0 ? l->keys[a] : r->keys[b];
            while (lp < le || rp < re) {
                int32_t x = lp < le ? (int32_t)rl[l->k2v[lp]] : INT32_MAX, y = rp < re ? (int32_t)rr[r->k2v[rp]] : INT32_MAX;
                if (x <= y) { if (i32v_push(&body, x)) { free(hdr); goto done; } ++lp; if (x == y) ++rp; }
                else { if (i32v_push(&body, y)) { free(hdr); goto done; } ++rp; }
            }
            hdr[nk++] = (uint32_t)body.n;
            if (which <= 0) ++a;
            if (which >= 0) ++b;
        }
        *onk = nk;
        for (uint32_t k = 0; k < nk; ++k) if (i32v_push(ox, (int32_t)(hdr[k] + nk))) { free(hdr); goto done; }
        for (size_t x = 0; x < body.n; ++x) if (i32v_push(ox, body.p[x])) { free(hdr); goto done; }
        free(hdr);
    }
    rc = 0;
done:
    free(rl); free(rr); free(body.p);
    return rc;
}

/* Deps.merge / PartialDeps.with over G sets of the same n txns (KeyDeps.merge KeyDeps.java:115-140,
 * RangeDeps.merge RangeDeps.java:101-126: a LinearMerger == left fold of linearUnion). */
int or_deps_union(uint32_t G, const or_deps *parts, or_deps *out)
{
    if (G == 0) return -1;
    const uint32_t n = parts[0].n;
    mm_out kd, rd;
    int rc = -1;
    if (mmo_init(&kd) || mmo_init(&rd)) goto fail;
    for (uint32_t i = 0; i < n; ++i) {
        for (int range = 0; range < 2; ++range) {
            mm_view acc;
            if (view_of(&parts[0], i, range, &acc)) goto fail;
            uint64_t *akeys = acc.keys;
            u32v av = {0}; i32v ax = {0};
            for (uint32_t v = 0; v < acc.nv; ++v) if (u32v_push(&av, acc.vals[v])) goto fail;
            for (uint32_t x = 0; x < acc.nx; ++x) if (i32v_push(&ax, acc.k2v[x])) goto fail;
            for (uint32_t g = 1; g < G; ++g) {
                mm_view r, l = {akeys, acc.nk, av.p, (uint32_t)av.n, ax.p, (uint32_t)ax.n};
                if (view_of(&parts[g], i, range, &r)) goto fail;
                uint64_t *nkeys; uint32_t nnk; u32v nv = {0}; i32v nx = {0};
                int e = mm_union2(&l, &r, &nkeys, &nnk, &nv, &nx);
                free(r.keys);
                if (e) goto fail;
                free(akeys); free(av.p); free(ax.p);
                akeys = nkeys; acc.nk = nnk; av = nv; ax = nx;
            }
            int e = mmo_emit(range ? &rd : &kd, range, akeys, acc.nk, av.p, (uint32_t)av.n, ax.p, (uint32_t)ax.n);
            free(akeys); free(av.p); free(ax.p);
            if (e) goto fail;
        }
    }
    if (alloc_out(out, &kd, &rd, n)) goto fail;
    rc = 0;
fail:
    mmo_free(&kd); mmo_free(&rd);
    return rc;
}

/* ------------------------------------------------------------------------------------------
 * The CommandStores of one node (SURVEY.md §7 "Hard parts" 5, §8e).  Store j owns the IntKey
 * range (bounds[j]-1, bounds[j+1]-1] (bounds[0] == 0: open below; bounds[S] == 0xFFFFFFFF: open
 * above).  Each store sees every txn of the stream restricted to itself -- its keys
 * (Keys.slice) and its ranges sliced Minimal (AbstractRanges.sliceMinimal, primitives/
 * AbstractRanges.java:339-377: one piece (max(s, lo), min(e, hi)] per intersecting range, in
 * order) -- both as the registered range command (InMemoryCommandStore.update,
 * impl/InMemoryCommandStore.java:757-760) and as the query (mapReduceRangesInternal :886).  Each
 * computes its PartialDeps alone (literal or fast restatement, same global positions, same
 * status-at-time model) and the node's result is their union (PreAccept.reduce ->
 * PartialDeps.with, messages/PreAccept.java:140-156): a range command spanning stores stays one
 * RangeDeps entry per store slice (primitives/RangeDeps.java:462-465).
 * ------------------------------------------------------------------------------------------ */
typedef struct { uint32_t *key_off, *key_ord, *rng_off, *rng_start, *rng_end; } store_view;

static void store_view_free(store_view *v)
{
    free(v->key_off); free(v->key_ord); free(v->rng_off); free(v->rng_start); free(v->rng_end);
    memset(v, 0, sizeof(*v));
}

static int store_view_build(const or_stream *s, uint32_t blo, uint32_t bhi, store_view *v)
{
    const uint32_t n = s->n;
    const int64_t lo = (int64_t)blo - 1;                                     /* (lo, hi] */
    const int64_t hi = bhi == 0xFFFFFFFFu ? INT64_MAX : (int64_t)bhi - 1;
    const uint32_t P = s->key_off[n], R = s->rng_off ? s->rng_off[n] : 0;
    memset(v, 0, sizeof(*v));
    v->key_off = (uint32_t *)malloc(((size_t)n + 1) * 4);
    v->key_ord = (uint32_t *)malloc(((size_t)P + 1) * 4);
    v->rng_off = (uint32_t *)malloc(((size_t)n + 1) * 4);
    v->rng_start = (uint32_t *)malloc(((size_t)R + 1) * 4);
    v->rng_end = (uint32_t *)malloc(((size_t)R + 1) * 4);
    if (!v->key_off || !v->key_ord || !v->rng_off || !v->rng_start || !v->rng_end) { store_view_free(v); return -1; }
    uint32_t np = 0, nr = 0;
    v->key_off[0] = 0; v->rng_off[0] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        for (uint32_t p = s->key_off[i]; p < s->key_off[i + 1]; ++p) {
            const int64_t k = s->key_ord[p];
            if (lo < k && k <= hi) v->key_ord[np++] = s->key_ord[p];
        }
        v->key_off[i + 1] = np;
        if (s->rng_off)
            for (uint32_t r = s->rng_off[i]; r < s->rng_off[i + 1]; ++r) {
                const int64_t rs = s->rng_start[r], re = s->rng_end[r];
                if (!(rs < hi && lo < re)) continue;                            /* Range.compareIntersecting */
                v->rng_start[nr] = (uint32_t)(rs >= lo ? rs : lo);              /* cs >= 0 ? rs : ls */
                v->rng_end[nr] = (uint32_t)(re <= hi ? re : hi);                /* ce <= 0 ? re : le */
                ++nr;
            }
        v->rng_off[i + 1] = nr;
    }
    return 0;
}

int or_stream_deps_stores(const or_stream *s, uint32_t nstores, const uint32_t *bounds, int literal, or_deps *out)
{
    if (nstores == 0) return -1;
    for (uint32_t j = 0; j < nstores; ++j) if (bounds[j] >= bounds[j + 1]) return -1;
    or_deps *parts = (or_deps *)calloc(nstores, sizeof(or_deps));
    if (!parts) return -1;
    int rc = 0;
    uint32_t done = 0;
    for (uint32_t j = 0; j < nstores && !rc; ++j) {
        store_view v;
        if ((rc = store_view_build(s, bounds[j], bounds[j + 1], &v))) break;
        or_stream t = *s;
        t.key_off = v.key_off; t.key_ord = v.key_ord;
        t.rng_off = v.rng_off; t.rng_start = v.rng_start; t.rng_end = v.rng_end;
        rc = literal ? stream_literal(&t, t.n, &parts[j]) : or_stream_deps_fast(&t, &parts[j]);
        store_view_free(&v);
        if (!rc) ++done;
    }
    if (!rc) rc = or_deps_union(nstores, parts, out);
    for (uint32_t j = 0; j < done; ++j) or_deps_free(&parts[j]);
    free(parts);
    return rc;
}

/* trimUnusedValues (utils/RelationMultiMap.java:491-532): keep the values referenced by the body
 * in their order, rewrite the body to the kept positions. */
static int trim_and_emit(mm_out *o, int range, const uint64_t *keys, uint32_t nk, const uint32_t *vals, uint32_t nv,
                         int32_t *k2v, uint32_t nx)
{
    int32_t *remap = (int32_t *)malloc(((size_t)nv + 1) * sizeof(int32_t));
    uint32_t *kept = (uint32_t *)malloc(((size_t)nv + 1) * sizeof(uint32_t));
    if (!remap || !kept) { free(remap); free(kept); return -1; }
    for (uint32_t v = 0; v < nv; ++v) remap[v] = 0;
    for (uint32_t x = nk; x < nx; ++x) remap[k2v[x]] = 1;
    uint32_t m = 0;
    for (uint32_t v = 0; v < nv; ++v) { if (remap[v]) { kept[m] = vals[v]; remap[v] = (int32_t)m++; } else remap[v] = -1; }
    if (m < nv) for (uint32_t x = nk; x < nx; ++x) k2v[x] = remap[k2v[x]];
    int e = mmo_emit(o, range, keys, nk, m < nv ? kept : vals, m < nv ? m : nv, k2v, nx);
    free(remap); free(kept);
    return e;
}

static int range_contains_key(uint32_t s, uint32_t e, uint64_t key) { return (uint64_t)s < key && key <= (uint64_t)e; }

/* KeyDeps.slice (primitives/KeyDeps.java:189-236): keys.slice(ranges) keeps the keys inside the
 * select ranges ((s,e] containment), copies their lists and trims unused txnIds; an empty KeyDeps,
 * or a selection of every key, returns the input unchanged; no key selected gives the empty
 * KeyDeps (no keys, no txnIds, no ints). */
static int keydeps_slice_one(mm_out *o, const mm_view *v, const uint32_t *ss, const uint32_t *se, uint32_t ns)
{
    if (v->nx == v->nk) return mmo_emit(o, 0, v->keys, v->nk, v->vals, v->nv, v->k2v, v->nx);
    uint64_t *sk = (uint64_t *)malloc(((size_t)v->nk + 1) * sizeof(uint64_t));
    uint32_t *sa = (uint32_t *)malloc(((size_t)v->nk + 1) * sizeof(uint32_t));
    if (!sk || !sa) { free(sk); free(sa); return -1; }
    uint32_t m = 0;
    for (uint32_t a = 0; a < v->nk; ++a)
        for (uint32_t q = 0; q < ns; ++q)
            if (range_contains_key(ss[q], se[q], v->keys[a])) { sk[m] = v->keys[a]; sa[m++] = a; break; }
    int e;
    if (m == 0) e = mmo_emit(o, 0, NULL, 0, NULL, 0, NULL, 0);
    else if (m == v->nk) e = mmo_emit(o, 0, v->keys, v->nk, v->vals, v->nv, v->k2v, v->nx);
    else {
        uint32_t off = m;
        for (uint32_t j = 0; j < m; ++j) off += (uint32_t)v->k2v[sa[j]] - body_start(v->k2v, v->nk, sa[j]);
        int32_t *trg = (int32_t *)malloc(((size_t)off + 1) * sizeof(int32_t));
        if (!trg) { free(sk); free(sa); return -1; }
        off = m;
        for (uint32_t j = 0; j < m; ++j) {
            for (uint32_t x = body_start(v->k2v, v->nk, sa[j]); x < (uint32_t)v->k2v[sa[j]]; ++x) trg[off++] = v->k2v[x];
            trg[j] = (int32_t)off;
        }
        e = trim_and_emit(o, 0, sk, m, v->vals, v->nv, trg, off);
        free(trg);
    }
    free(sk); free(sa);
    return e;
}

/* RangeDeps.slice (primitives/RangeDeps.java:545-565) with the RangeAndMapCollector
 * (:727-848) driven by SearchableRangeList/CheckpointIntervalArray.forEach
 * (utils/CheckpointIntervalArray.java:100-221) once per select range with the running minIndex
 * (RangeDeps.java:192-197).  Per select range (qs, qe]:
 *   end   = first index >= minIndex whose start >= qe (CEIL on start), nothing if end <= minIndex;
 *   floor = CEIL(qs) on start within [minIndex, n) (exact: lowest equal start) or, if absent, the
 *           insertion point - 1; start = floor, stepped forward once if that range ends <= qs;
 *   the checkpoint + scan matches are {i in [minIndex, floor) : end_i > qs} (the match set the
 *           checkpoint index guarantees: SearchableRangeListTest.java:98-112), buffered
 *           out-of-order; the run [max(start,minIndex), end) is reported through forEachRange,
 *           whose accept() first flushes the buffered matches (sorted) and then copies the run;
 *   minIndex = end.
 * Buffered matches are only flushed by a later non-empty run: matches still buffered after the
 * last select range are dropped (collector has no final flush, RangeDeps.java:550-563).  The
 * output ranges are ascending by index; all ranges selected returns the input unchanged. */
static int rangedeps_slice_one(mm_out *o, const or_deps *d, uint32_t i, const mm_view *v,
                               const uint32_t *ss, const uint32_t *se, uint32_t ns)
{
    const uint32_t n = v->nk;
    const uint32_t *rs = d->rd_rng_start + d->rd_rng_off[i], *re = d->rd_rng_end + d->rd_rng_off[i];
    if (v->nx == v->nk) return mmo_emit(o, 1, NULL, 0, v->vals, v->nv, NULL, 0);   /* RangeDeps(NO_RANGES, txnIds, NO_INTS) */
    uint8_t *sel = (uint8_t *)calloc((size_t)n + 1, 1), *pend = (uint8_t *)calloc((size_t)n + 1, 1);
    if (!sel || !pend) { free(sel); free(pend); return -1; }
    uint32_t minIndex = 0;
    for (uint32_t q = 0; q < ns; ++q) {
        if (n == 0 || minIndex == n) continue;
        uint32_t end = minIndex;
        while (end < n && rs[end] < se[q]) ++end;            /* starts are ascending */
        if (end <= minIndex) continue;
        uint32_t ins = minIndex;
        while (ins < n && rs[ins] < ss[q]) ++ins;
        int64_t floor, start;
        if (ins < n && rs[ins] == ss[q]) floor = start = ins;
        else {
            floor = start = (int64_t)ins - 1;
            if (start < 0) start = floor = 0;
            else if (re[start] <= ss[q]) ++start;
        }
        if (start < minIndex) start = minIndex;
        for (int64_t x = minIndex; x < floor; ++x) if (re[x] > ss[q]) pend[x] = 1;
        if ((uint32_t)start != end) {
            for (uint32_t x = 0; x < n; ++x) if (pend[x] && x < (uint32_t)start) { sel[x] = 1; pend[x] = 0; }
            for (uint32_t x = (uint32_t)start; x < end; ++x) sel[x] = 1;
            memset(pend, 0, n);   /* buffered entries >= fromIndex are dropped (binarySearch cut) */
        }
        minIndex = end;
    }
    uint32_t m = 0;
    for (uint32_t x = 0; x < n; ++x) m += sel[x];
    int e;
    if (m == 0) e = mmo_emit(o, 1, NULL, 0, NULL, 0, NULL, 0);
    else if (m == n) e = mmo_emit(o, 1, v->keys, v->nk, v->vals, v->nv, v->k2v, v->nx);
    else {
        uint64_t *sk = (uint64_t *)malloc(((size_t)m + 1) * sizeof(uint64_t));
        uint32_t off = m;
        for (uint32_t x = 0; x < n; ++x) if (sel[x]) off += (uint32_t)v->k2v[x] - body_start(v->k2v, n, x);
        int32_t *trg = (int32_t *)malloc(((size_t)off + 1) * sizeof(int32_t));
        if (!sk || !trg) { free(sk); free(trg); free(sel); free(pend); return -1; }
        uint32_t j = 0;
        off = m;
        for (uint32_t x = 0; x < n; ++x) {
            if (!sel[x]) continue;
            sk[j] = v->keys[x];
            for (uint32_t y = body_start(v->k2v, n, x); y < (uint32_t)v->k2v[x]; ++y) trg[off++] = v->k2v[y];
            trg[j++] = (int32_t)off;
        }
        e = trim_and_emit(o, 1, sk, m, v->vals, v->nv, trg, off);
        free(sk); free(trg);
    }
    free(sel); free(pend);
    return e;
}

int or_deps_slice(const or_deps *d, const uint32_t *sel_off, const uint32_t *sel_start, const uint32_t *sel_end,
                  uint32_t nsel, or_deps *out)
{
    const uint32_t n = d->n;
    mm_out kd, rd;
    int rc = -1;
    if (mmo_init(&kd) || mmo_init(&rd)) goto fail;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t q0 = sel_off ? sel_off[i] : 0, ns = sel_off ? sel_off[i + 1] - sel_off[i] : nsel;
        mm_view v;
        if (view_of(d, i, 0, &v)) goto fail;
        int e = keydeps_slice_one(&kd, &v, sel_start + q0, sel_end + q0, ns);
        free(v.keys);
        if (e) goto fail;
        if (view_of(d, i, 1, &v)) goto fail;
        e = rangedeps_slice_one(&rd, d, i, &v, sel_start + q0, sel_end + q0, ns);
        free(v.keys);
        if (e) goto fail;
    }
    if (alloc_out(out, &kd, &rd, n)) goto fail;
    rc = 0;
fail:
    mmo_free(&kd); mmo_free(&rd);
    return rc;
}

/* RelationMultiMap.invert (utils/RelationMultiMap.java:907-938) of every txn's keysToTxnIds
 * (range = 0) or rangesToTxnIds (range = 1): txnIdsToKeys with |txnIds| end offsets (absolute,
 * first starting at |txnIds|) then, per txnId, its key indices ascending.  off[n+1] (caller) and
 * *out (malloc'd). */
int or_deps_invert(const or_deps *d, int range, uint32_t *off, int32_t **out)
{
    const uint32_t n = d->n;
    size_t total = 0;
    off[0] = 0;
    for (uint32_t i = 0; i < n; ++i) {
        mm_view v;
        if (view_of(d, i, range, &v)) return -1;
        free(v.keys);
        total += (size_t)v.nv + (v.nx - v.nk);
        off[i + 1] = (uint32_t)total;
    }
    int32_t *o = (int32_t *)calloc(total ? total : 1, sizeof(int32_t));
    if (!o) return -1;
    for (uint32_t i = 0; i < n; ++i) {
        mm_view v;
        if (view_of(d, i, range, &v)) { free(o); return -1; }
        free(v.keys);
        int32_t *trg = o + off[i];
        const int32_t *src = v.k2v;
        const uint32_t tk = v.nv, sk = v.nk, sl = v.nx;
        if (tk == 0) continue;
        for (uint32_t x = sk; x < sl; ++x) trg[src[x]]++;
        trg[0] += (int32_t)tk;
        for (uint32_t k = 1; k < tk; ++k) trg[k] += trg[k - 1];
        memmove(trg + 1, trg, (size_t)(tk - 1) * sizeof(int32_t));
        trg[0] = (int32_t)tk;
        uint32_t k = 0;
        for (uint32_t x = sk; x < sl; ++x) {
            while (x == (uint32_t)src[k]) ++k;
            trg[trg[src[x]]++] = (int32_t)k;
        }
    }
    *out = o;
    return 0;
}

/* ---- MaxConflicts fold (test infrastructure) ------------------------------------------------
 * Literal restatement of the per-PreAccept executeAt proposal input for key txns:
 *   CommandStore.preaccept reads  minNonConflicting = maxConflicts.get(keys)
 *     (local/CommandStore.java:344, MaxConflicts.get = foldl(keys, Timestamp::max, NONE),
 *      local/MaxConflicts.java:46-49; foldl visits only keys with a map entry, in key order, as
 *      fold(value, acc): utils/ReducingRangeMap.java:55-57,117-140; Timestamp.max(a, b) =
 *      a.compareTo(b) >= 0 ? a : b, primitives/Timestamp.java:265-268),
 *   fast path iff txnId.compareTo(minNonConflicting) >= 0 (:345, epoch check excluded), and then
 *   the command's executeAt is merged in (SafeCommandStore.update -> updateMaxConflicts,
 *   local/SafeCommandStore.java:192-210 only for isGloballyVisible kinds, primitives/Txn.java:187-200;
 *   CommandStore.updateMaxConflicts -> MaxConflicts.update = merge(this, create(keys, executeAt))
 *   with Timestamp::max(old, new), local/CommandStore.java:280-289, local/MaxConflicts.java:68-80).
 * The map is one entry per key ordinal (st_has = 0: no entry).  exec_* NULL: executeAt = txnId.
 * Returns 0, or -4 for a key outside [key_lo, key_lo + nkeys). */
int or_max_conflicts(uint32_t n, const uint64_t *msb, const uint64_t *lsb, const int32_t *node,
                     const uint32_t *key_off, const uint32_t *key_ord, const uint64_t *exec_msb,
                     const uint64_t *exec_lsb, const int32_t *exec_node, uint32_t key_lo, uint32_t nkeys,
                     uint64_t *st_msb, uint64_t *st_lsb, int32_t *st_node, uint8_t *st_has,
                     uint64_t *o_msb, uint64_t *o_lsb, int32_t *o_node, uint8_t *o_has, uint8_t *o_fast,
                     uint32_t first, int has_override, uint64_t ov_msb, uint64_t ov_lsb, int32_t ov_node,
                     uint32_t *folded)
{
    *folded = n;
    for (uint32_t i = first; i < n; ++i) {
        /* CommandStore.preaccept (local/CommandStore.java:320-349): ExclusiveSyncPoint returns before
         * reading maxConflicts and treats its keys as Ranges (:335-339) -- no key-domain form */
        const int kind = kind_of(lsb[i]);
        if (kind >= 4 || (lsb[i] & 1)) return (lsb[i] & 1) ? -5 : -3;
        int has = 0;
        uint64_t am = 0, al = 0;    /* Timestamp.NONE */
        int32_t an = 0;
        /* MaxConflicts.get = foldl(keys, Timestamp::max, NONE) (local/MaxConflicts.java:46-49) */
        for (uint32_t p = key_off[i]; p < key_off[i + 1]; ++p) {
            if (key_ord[p] < key_lo || key_ord[p] - key_lo >= nkeys) return -4;
            uint32_t k = key_ord[p] - key_lo;
            if (!st_has[k]) continue;
            if (!has || or_ts_compare(st_msb[k], st_lsb[k], st_node[k], am, al, an) >= 0) {
                am = st_msb[k]; al = st_lsb[k]; an = st_node[k];
            }
            has = 1;
        }
        o_msb[i] = am; o_lsb[i] = al; o_node[i] = an; o_has[i] = (uint8_t)has;
        const int fast = or_ts_compare(msb[i], lsb[i], node[i], am, al, an) >= 0;
        o_fast[i] = (uint8_t)fast;
        /* updateMaxConflicts: globally visible kinds only (local/SafeCommandStore.java:198-209) */
        if (is_globally_visible(kind) != 1) continue;
        uint64_t em, el;
        int32_t en;
        if (i == first && has_override) { em = ov_msb; el = ov_lsb; en = ov_node; }
        else if (exec_msb) { em = exec_msb[i]; el = exec_lsb[i]; en = exec_node[i]; }
        else if (fast) { em = msb[i]; el = lsb[i]; en = node[i]; }
        else { *folded = i; return 0; }   /* executeAt = time.uniqueNow(minNonConflicting) (:348): the caller's */
        for (uint32_t p = key_off[i]; p < key_off[i + 1]; ++p) {
            uint32_t k = key_ord[p] - key_lo;
            /* merge keeps the old value unless the new one is strictly greater */
            if (!st_has[k] || or_ts_compare(em, el, en, st_msb[k], st_lsb[k], st_node[k]) > 0) {
                st_msb[k] = em; st_lsb[k] = el; st_node[k] = en; st_has[k] = 1;
            }
        }
    }
    return 0;
}

/* MaxConflicts over key and range txns with the map held as a ReducingRangeMap-style list of
 * disjoint intervals (utils/ReducingIntervalMap.java, utils/ReducingRangeMap.java) rather than one
 * entry per key: a key k is the interval [k, k+1), a range (s, e] (Range.EndInclusive) the interval
 * [s+1, e+1), clipped to the store's keys [key_lo, key_lo + nkeys) ("keys sliced to those owned",
 * local/CommandStore.java:318).  get = foldl over the intersecting intervals in order with
 * Timestamp.max(value, acc) (MaxConflicts.java:46-54); update = merge with Timestamp.max(old, new)
 * (:68-80), which splits intervals at the new bounds.  ExclusiveSyncPoint in the range domain
 * returns txnId before reading the map (CommandStore.java:335-339: present = 0, fast = 1) and is
 * merged like any globally visible txn; in the key domain it is -3.  The per-key state arrays are
 * the map's point values on entry and exit.  Returns 0, -3 kind, -4 key outside the store, -6
 * ranges not sorted / overlapping / empty. */
typedef struct { uint32_t a, b; ts_t v; } mc_ivl;
typedef struct { mc_ivl *p; size_t n, cap; } mc_map;

static int mcm_push(mc_map *m, uint32_t a, uint32_t b, ts_t v)
{
    if (a >= b) return 0;
    if (m->n == m->cap) {
        size_t nc = m->cap ? m->cap * 2 : 64;
        mc_ivl *np = (mc_ivl *)realloc(m->p, nc * sizeof(mc_ivl));
        if (!np) return -1;
        m->p = np; m->cap = nc;
    }
    m->p[m->n].a = a; m->p[m->n].b = b; m->p[m->n].v = v;
    m->n++;
    return 0;
}

/* foldl(Timestamp::max(value, acc)) over the intervals intersecting [a, b) */
static void mcm_get(const mc_map *m, uint32_t a, uint32_t b, int *has, ts_t *acc)
{
    for (size_t i = 0; i < m->n; ++i) {
        const mc_ivl *x = &m->p[i];
        if (x->b <= a || x->a >= b) continue;
        if (!*has || ts_cmp(&x->v, acc) >= 0) *acc = x->v;
        *has = 1;
    }
}

/* merge(this, create([a, b), v)) with Timestamp::max(old, new): old kept unless new is greater */
static int mcm_update(mc_map *m, uint32_t a, uint32_t b, const ts_t *v)
{
    mc_map o = {0, 0, 0};
    uint32_t cur = a;            /* next uncovered point of [a, b) */
    for (size_t i = 0; i < m->n; ++i) {
        const mc_ivl x = m->p[i];
        if (x.b <= a || x.a >= b) {
            if (x.a >= b && cur < b) { if (mcm_push(&o, cur, b, *v)) goto oom; cur = b; }
            if (mcm_push(&o, x.a, x.b, x.v)) goto oom;
            continue;
        }
        if (x.a < a && mcm_push(&o, x.a, a, x.v)) goto oom;
        const uint32_t lo = x.a > a ? x.a : a, hi = x.b < b ? x.b : b;
        if (cur < lo && mcm_push(&o, cur, lo, *v)) goto oom;
        if (mcm_push(&o, lo, hi, ts_cmp(v, &x.v) > 0 ? *v : x.v)) goto oom;
        cur = hi;
        if (x.b > b && mcm_push(&o, b, x.b, x.v)) goto oom;
    }
    if (cur < b && mcm_push(&o, cur, b, *v)) goto oom;
    free(m->p);
    *m = o;
    return 0;
oom:
    free(o.p);
    return -1;
}

int or_max_conflicts_rm(uint32_t n, const uint64_t *msb, const uint64_t *lsb, const int32_t *node,
                        const uint32_t *key_off, const uint32_t *key_ord, const uint32_t *rng_off,
                        const uint32_t *rng_start, const uint32_t *rng_end, const uint64_t *exec_msb,
                        const uint64_t *exec_lsb, const int32_t *exec_node, uint32_t key_lo, uint32_t nkeys,
                        uint64_t *st_msb, uint64_t *st_lsb, int32_t *st_node, uint8_t *st_has,
                        uint64_t *o_msb, uint64_t *o_lsb, int32_t *o_node, uint8_t *o_has, uint8_t *o_fast,
                        uint32_t first, int has_override, uint64_t ov_msb, uint64_t ov_lsb, int32_t ov_node,
                        uint32_t *folded)
{
    mc_map m = {0, 0, 0};
    int rc = 0;
    *folded = n;
    for (uint32_t k = 0; k < nkeys; ++k)
        if (st_has[k]) {
            ts_t v = {st_msb[k], st_lsb[k], st_node[k]};
            if (mcm_push(&m, k, k + 1, v)) { rc = -1; goto out; }
        }
    for (uint32_t i = first; i < n; ++i) {
        const int kind = kind_of(lsb[i]), range = (int)(lsb[i] & 1);
        if (kind >= 5 || (!range && kind == K_EXCL_SYNC_POINT)) { rc = -3; goto out; }
        /* the txn's intervals, clipped to the store */
        uint32_t na = range ? rng_off[i + 1] - rng_off[i] : key_off[i + 1] - key_off[i];
        uint32_t *ia = (uint32_t *)malloc(((size_t)na + 1) * 2 * sizeof(uint32_t));
        if (!ia) { rc = -1; goto out; }
        uint32_t ni = 0;
        for (uint32_t q = 0; q < na; ++q) {
            uint64_t a, b;
            if (range) {
                const uint32_t r = rng_off[i] + q;
                if (rng_start[r] >= rng_end[r] || (q > 0 && rng_start[r] < rng_end[r - 1])) { free(ia); rc = -6; goto out; }
                a = (uint64_t)rng_start[r] + 1; b = (uint64_t)rng_end[r] + 1;
                if (a < key_lo) a = key_lo;
                if (b > (uint64_t)key_lo + nkeys) b = (uint64_t)key_lo + nkeys;
                if (a >= b) continue;
            } else {
                const uint32_t k = key_ord[key_off[i] + q];
                if (k < key_lo || k - key_lo >= nkeys) { free(ia); rc = -4; goto out; }
                a = k; b = (uint64_t)k + 1;
            }
            ia[2 * ni] = (uint32_t)(a - key_lo); ia[2 * ni + 1] = (uint32_t)(b - key_lo); ++ni;
        }
        int has = 0, fast;
        ts_t acc = {0, 0, 0};
        if (range && kind == K_EXCL_SYNC_POINT) fast = 1;     /* markExclusiveSyncPoint; return txnId */
        else {
            for (uint32_t q = 0; q < ni; ++q) mcm_get(&m, ia[2 * q], ia[2 * q + 1], &has, &acc);
            fast = or_ts_compare(msb[i], lsb[i], node[i], acc.msb, acc.lsb, acc.node) >= 0;
        }
        o_msb[i] = acc.msb; o_lsb[i] = acc.lsb; o_node[i] = acc.node; o_has[i] = (uint8_t)has;
        o_fast[i] = (uint8_t)fast;
        if (is_globally_visible(kind) == 1) {
            ts_t e;
            if (i == first && has_override) { e.msb = ov_msb; e.lsb = ov_lsb; e.node = ov_node; }
            else if (exec_msb) { e.msb = exec_msb[i]; e.lsb = exec_lsb[i]; e.node = exec_node[i]; }
            else if (fast) { e.msb = msb[i]; e.lsb = lsb[i]; e.node = node[i]; }
            else { free(ia); *folded = i; goto out; }
            for (uint32_t q = 0; q < ni; ++q)
                if (mcm_update(&m, ia[2 * q], ia[2 * q + 1], &e)) { free(ia); rc = -1; goto out; }
        }
        free(ia);
    }
out:
    if (rc == 0) {
        memset(st_has, 0, nkeys);
        for (size_t j = 0; j < m.n; ++j)
            for (uint32_t k = m.p[j].a; k < m.p[j].b; ++k) {
                st_msb[k] = m.p[j].v.msb; st_lsb[k] = m.p[j].v.lsb; st_node[k] = m.p[j].v.node; st_has[k] = 1;
            }
    }
    free(m.p);
    return rc;
}

/* ==========================================================================================
 * Stateful literal CommandStore (test infrastructure): a resident store fed batch by batch,
 * with real status events in between.  Key txns only.  Every txn a batch carries is inserted
 * into its keys' CommandsForKey as PREACCEPTED when it is processed (CommandsForKey.insert,
 * local/CommandsForKey.java:880-944, via SafeCommandStore.updateCommandsForKey :212-239); an
 * event (accord_txn_register) is CommandsForKey.update(prev, next) with the new InternalStatus
 * and executeAt on every key of the txn (:652-706, the committed[] index rebuilt by the
 * constructor :422-470).  There is no status-at-time model: a txn keeps PREACCEPTED until an
 * event changes it.  Deps values are global positions (the order txns entered the store).
 * ========================================================================================== */
struct or_lstore {
    uint32_t nkeys;
    cfk_t *cfks;
    ts_t *tbl;                 /* TxnIds by global position */
    uint32_t *koff, *kord;     /* keys of every registered txn (CSR by global position) */
    uint32_t n, cap, nk, kcap;
    uint8_t *status;           /* current InternalStatus of every txn (8: SaveStatus Erased/Invalidated) */
    ts_t *exec;
    /* range txns: InMemoryCommandStore.rangeCommands (impl/InMemoryCommandStore.java:739-762) --
     * the command's ranges (CSR by global position) and whether its SaveStatus reached Erased */
    uint32_t *roff, *rst, *ren;
    uint32_t nr, rcap;
    /* execution readiness: the txns whose WaitingOn was initialised and that are not ready yet */
    struct or_waiter *wt;
    uint32_t nwt, cwt;
    /* RedundantBefore as readiness reads it (or_lstore_redundant): entries (rr_s, rr_e] ascending and
     * disjoint, [rr_sep, rr_eep), locallyAppliedOrInvalidatedBefore / bootstrappedAt as positions
     * (0xFFFFFFFF = TxnId.NONE), staleUntilAtLeast != null */
    uint32_t rr_m;
    uint32_t *rr_s, *rr_e, *rr_local, *rr_boot;
    uint64_t *rr_sep, *rr_eep;
    uint8_t *rr_stale;
    /* event mode (or_lstore_event_mode): key bits are cleared only when notifyAndUpdatePending's events
     * reach the key; wix[g] = waiter index + 1 of the txn at position g (0: not waiting) */
    int event_mode;
    uint32_t *wix;
    uint32_t wix_cap;
    /* setAppliedAndPropagate (local/Command.java:1569-1583): the final WaitingOn.appliedOrInvalidated of
     * every released Range-domain waiter, as the positions of its RangeDeps txnIds whose bit is set
     * (pv_at[g] = 1 + start in pv_pool, pv_len[g] entries; 0 = none) */
    uint32_t *pv_at, *pv_len, pv_cap_pos;
    uint32_t *pv_pool;
    size_t pv_n, pv_cap;
};

static void or_lstore_waiters_free(or_lstore *s);
typedef struct or_waiter or_waiter;
static or_waiter *waiter_of(const or_lstore *s, uint32_t g);
static int waiter_unmanaged(const or_lstore *s, const or_waiter *x);
static void lstore_register_unmanaged(or_lstore *s, or_waiter *x);
static void lstore_event(or_lstore *s, uint32_t k, uint32_t X, uint8_t prev, uint8_t nw, const ts_t *exec);
static void cfk_nexts(const or_lstore *s, const cfk_t *c, long *min_unc, long *next, long *next_write);
static void cfk_notify_unmanaged(or_lstore *s, uint32_t k, int commit, long min_unc, long next);
static int wix_rebuild(or_lstore *s);

or_lstore *or_lstore_create(uint32_t nkeys)
{
    or_lstore *s = (or_lstore *)calloc(1, sizeof(or_lstore));
    if (!s) return NULL;
    s->nkeys = nkeys;
    s->cfks = (cfk_t *)calloc(nkeys ? nkeys : 1, sizeof(cfk_t));
    s->koff = (uint32_t *)calloc(1, sizeof(uint32_t));
    s->roff = (uint32_t *)calloc(1, sizeof(uint32_t));
    if (!s->cfks || !s->koff || !s->roff) { or_lstore_free(s); return NULL; }
    return s;
}

void or_lstore_free(or_lstore *s)
{
    if (!s) return;
    if (s->cfks) for (uint32_t k = 0; k < s->nkeys; ++k) { free(s->cfks[k].txns); free(s->cfks[k].committed); }
    free(s->cfks); free(s->tbl); free(s->koff); free(s->kord); free(s->status); free(s->exec);
    free(s->roff); free(s->rst); free(s->ren);
    or_lstore_waiters_free(s);
    free(s->rr_s); free(s->rr_e); free(s->rr_local); free(s->rr_boot); free(s->rr_sep); free(s->rr_eep); free(s->rr_stale);
    free(s->wix);
    free(s->pv_at); free(s->pv_len); free(s->pv_pool);
    free(s);
}

static int lstore_reserve(or_lstore *s, uint32_t n, uint32_t nk)
{
    if (n > s->cap) {
        uint32_t c = s->cap ? s->cap : 1024;
        while (c < n) c *= 2;
        ts_t *t = (ts_t *)realloc(s->tbl, (size_t)c * sizeof(ts_t));
        if (!t) return -1;
        s->tbl = t;
        uint32_t *ko = (uint32_t *)realloc(s->koff, ((size_t)c + 1) * sizeof(uint32_t));
        if (!ko) return -1;
        s->koff = ko;
        uint8_t *st = (uint8_t *)realloc(s->status, c);
        if (!st) return -1;
        s->status = st;
        ts_t *ex = (ts_t *)realloc(s->exec, (size_t)c * sizeof(ts_t));
        if (!ex) return -1;
        s->exec = ex;
        uint32_t *ro = (uint32_t *)realloc(s->roff, ((size_t)c + 1) * sizeof(uint32_t));
        if (!ro) return -1;
        s->roff = ro;
        s->cap = c;
    }
    if (nk > s->kcap) {
        uint32_t c = s->kcap ? s->kcap : 4096;
        while (c < nk) c *= 2;
        uint32_t *kk = (uint32_t *)realloc(s->kord, (size_t)c * sizeof(uint32_t));
        if (!kk) return -1;
        s->kord = kk;
        s->kcap = c;
    }
    return 0;
}

static int lstore_reserve_ranges(or_lstore *s, uint32_t nr)
{
    if (nr <= s->rcap) return 0;
    uint32_t c = s->rcap ? s->rcap : 1024;
    while (c < nr) c *= 2;
    uint32_t *a = (uint32_t *)realloc(s->rst, (size_t)c * sizeof(uint32_t));
    if (!a) return -1;
    s->rst = a;
    uint32_t *b = (uint32_t *)realloc(s->ren, (size_t)c * sizeof(uint32_t));
    if (!b) return -1;
    s->ren = b;
    s->rcap = c;
    return 0;
}

#define S_ERASED 8             /* SaveStatus >= Erased (Erased, Invalidated): local/SaveStatus.java:83-87 */
/* SaveStatus TruncatedApply* (local/SaveStatus.java:79-81): INVALID_OR_TRUNCATED in CommandsForKey
 * (InternalStatus.convert, local/CommandsForKey.java:222-224), before Erased (still visited by the
 * range scan), with a known executeAt (updateWaitingOn's updateExecuteAtLeast, local/Commands.java:782) */
#define S_TRUNC_APPLY 9
/* the order statuses advance in: ... Applied < TruncatedApply < ErasedOrInvalidated / Invalidated <
 * Erased (SaveStatus order) */
static int status_rank(int st) { return st == S_TRUNC_APPLY ? 13 : 2 * st; }

/* mapReduceRangesInternal (impl/InMemoryCommandStore.java:883-1016) over the store's range commands
 * [0, reg): skip SaveStatus >= Erased (:891; ErasedOrInvalidated is before Erased and still visited),
 * txnId < startedBefore (:901-902), the p1 txn, unwitnessed kinds (:927); every range of the command
 * intersecting the query -> (range, txnId) collected in a TreeMap by Range.compare and replayed. */
static int lstore_range_scan(const or_lstore *s, const or_stream *b, uint32_t i, uint32_t reg, const ts_t *sb,
                             long p1, int test_kinds, mm_builder *rb)
{
    typedef struct { uint64_t code; uint32_t txn; } hit_t;
    hit_t *h = NULL;
    size_t nh = 0, ch = 0;
    int rc = -1;
    for (uint32_t g = 0; g < reg; ++g) {
        if (s->roff[g + 1] == s->roff[g]) continue;                          /* not a range command */
        if (s->status[g] == S_ERASED) continue;
        if (ts_cmp(&s->tbl[g], sb) >= 0) continue;
        if (p1 >= 0 && (uint32_t)p1 == g) continue;
        if (!kinds_test(test_kinds, kind_of(s->tbl[g].lsb))) continue;
        for (uint32_t a = s->roff[g]; a < s->roff[g + 1]; ++a) {
            const uint32_t rs = s->rst[a], re = s->ren[a];
            int hit = 0;
            if (domain_of(b->lsb[i]) == 0) {
                for (uint32_t p = b->key_off[i]; p < b->key_off[i + 1] && !hit; ++p)
                    hit = range_intersects_key(rs, re, b->key_ord[p]);
            } else {
                for (uint32_t r = b->rng_off[i]; r < b->rng_off[i + 1] && !hit; ++r)
                    hit = range_intersects_range(rs, re, b->rng_start[r], b->rng_end[r]);
            }
            if (!hit) continue;
            if (nh == ch) {
                ch = ch ? ch * 2 : 64;
                hit_t *nhp = (hit_t *)realloc(h, ch * sizeof(hit_t));
                if (!nhp) goto done;
                h = nhp;
            }
            h[nh].code = ((uint64_t)rs << 32) | re;
            h[nh].txn = g;
            ++nh;
        }
    }
    /* TreeMap by Range.compare, each list in scan (TxnId) order: a stable insertion sort by range */
    for (size_t a = 1; a < nh; ++a) {
        hit_t x = h[a]; size_t c = a;
        while (c > 0 && h[c - 1].code > x.code) { h[c] = h[c - 1]; --c; }
        h[c] = x;
    }
    for (size_t a = 0; a < nh; ++a)
        if (mmb_add(rb, h[a].code, h[a].txn)) goto done;
    rc = 0;
done:
    free(h);
    return rc;
}

int or_lstore_batch(or_lstore *s, const or_stream *b, or_deps *out)
{
    const uint32_t n = b->n;
    int rc = validate(b, n);
    if (!rc) rc = validate_exec(b, n);
    if (rc) return rc;
    for (uint32_t i = 0; i < n; ++i) {
        if (domain_of(b->lsb[i]) != 0 && !b->rng_off) return -5;
        for (uint32_t p = b->key_off[i]; p < b->key_off[i + 1]; ++p) if (b->key_ord[p] >= s->nkeys) return -4;
    }
    if (n && s->n && or_ts_compare(s->tbl[s->n - 1].msb, s->tbl[s->n - 1].lsb, s->tbl[s->n - 1].node,
                                   b->msb[0], b->lsb[0], b->node[0]) >= 0) return -2;
    const uint32_t base = s->n;
    const uint32_t nbr = b->rng_off ? b->rng_off[n] - b->rng_off[0] : 0;
    if (lstore_reserve(s, base + n, s->koff[base] + b->key_off[n])) return -1;
    if (lstore_reserve_ranges(s, s->roff[base] + nbr)) return -1;
    for (uint32_t i = 0; i < n; ++i) {                 /* the batch's TxnIds, keys and ranges (not registered yet) */
        ts_t t = {b->msb[i], b->lsb[i], b->node[i]};
        s->tbl[base + i] = t;
        s->koff[base + i + 1] = s->koff[base + i] + (b->key_off[i + 1] - b->key_off[i]);
        memcpy(s->kord + s->koff[base + i], b->key_ord + b->key_off[i], (b->key_off[i + 1] - b->key_off[i]) * 4);
        const uint32_t r0 = b->rng_off ? b->rng_off[i] : 0, r1 = b->rng_off ? b->rng_off[i + 1] : 0;
        s->roff[base + i + 1] = s->roff[base + i] + (r1 - r0);
        if (r1 > r0) {
            memcpy(s->rst + s->roff[base + i], b->rng_start + r0, (r1 - r0) * 4);
            memcpy(s->ren + s->roff[base + i], b->rng_end + r0, (r1 - r0) * 4);
        }
        s->status[base + i] = S_PREACCEPTED;
        s->exec[base + i] = t;
    }
    mm_builder kb, rb;
    mm_out kd, rd;
    mmb_init(&kb, s->tbl);
    mmb_init(&rb, s->tbl);
    if (mmo_init(&kd) || mmo_init(&rd)) return -1;
    rc = -1;
    uint32_t reg = 0;                                  /* batch txns [0, reg) are inserted */
    for (uint32_t i = 0; i < n; ++i) {
        const ts_t sb = started_before(b, i);
        const long p1 = p1_of(b, i) >= 0 ? (long)(base + i) : -1;
        uint32_t reg_to = bound_of(b, n, &sb, i);      /* an Accept sees the batch txns started before executeAt */
        if (reg_to < i + 1) reg_to = i + 1;
        for (; reg < reg_to; ++reg) {
            const uint32_t g = base + reg;
            if (domain_of(b->lsb[reg]) == 0 && is_globally_visible(kind_of(b->lsb[reg])) == 1)
                for (uint32_t p = b->key_off[reg]; p < b->key_off[reg + 1]; ++p)
                    if (cfk_insert(&s->cfks[b->key_ord[p]], s->tbl, g, S_PREACCEPTED)) goto done;
            /* a range txn joins rangeCommands (its ranges above), not any CommandsForKey */
        }
        const int test_kinds = witnesses_of(kind_of(b->lsb[i]));
        mmb_reset(&kb); mmb_reset(&rb);
        if (domain_of(b->lsb[i]) == 0) {
            for (uint32_t p = b->key_off[i]; p < b->key_off[i + 1]; ++p) {
                const uint32_t key = b->key_ord[p];
                if (cfk_map_reduce_active(&s->cfks[key], s->tbl, &sb, test_kinds, key, &kb, p1)) goto done;
            }
        } else {
            /* mapReduceForKey Range case (impl/InMemoryCommandStore.java:274-289): every CFK key in
             * each (start, end], ascending */
            for (uint32_t r = b->rng_off[i]; r < b->rng_off[i + 1]; ++r)
                for (uint32_t key = b->rng_start[r] + 1; key <= b->rng_end[r] && key < s->nkeys; ++key)
                    if (s->cfks[key].n && cfk_map_reduce_active(&s->cfks[key], s->tbl, &sb, test_kinds, key, &kb, p1))
                        goto done;
        }
        if (lstore_range_scan(s, b, i, base + reg, &sb, p1, test_kinds, &rb)) goto done;
        if (mmb_build(&kb, &kd, 0)) goto done;
        if (mmb_build(&rb, &rd, 1)) goto done;
    }
    s->n = base + n;
    if (alloc_out(out, &kd, &rd, n)) goto done;
    rc = 0;
done:
    if (rc) s->n = base;
    mmb_free(&kb); mmb_free(&rb);
    mmo_free(&kd); mmo_free(&rd);
    return rc;
}

/* a status event for each of n txns (strictly ascending TxnIds, all known to the store):
 * InternalStatus ordinals (local/CommandsForKey.java:194-203); executeAt for ACCEPTED and above.
 * Statuses never go back; a committed executeAt never changes (the checkState of :674-690). */
int or_lstore_register(or_lstore *s, uint32_t n, const uint64_t *msb, const uint64_t *lsb, const int32_t *node,
                       const uint8_t *status, const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode)
{
    uint32_t *pos = (uint32_t *)malloc((size_t)(n ? n : 1) * sizeof(uint32_t));
    if (!pos) return -1;
    for (uint32_t r = 0; r < n; ++r) {                 /* validate everything before changing anything */
        if (r && or_ts_compare(msb[r - 1], lsb[r - 1], node[r - 1], msb[r], lsb[r], node[r]) >= 0) { free(pos); return -2; }
        if (status[r] > S_TRUNC_APPLY) { free(pos); return -1; }
        uint32_t lo = 0, hi = s->n;
        while (lo < hi) {
            uint32_t m = (lo + hi) / 2;
            if (or_ts_compare(s->tbl[m].msb, s->tbl[m].lsb, s->tbl[m].node, msb[r], lsb[r], node[r]) < 0) lo = m + 1; else hi = m;
        }
        if (lo >= s->n || !or_ts_equals(s->tbl[lo].msb, s->tbl[lo].lsb, s->tbl[lo].node, msb[r], lsb[r], node[r])) { free(pos); return -1; }
        const uint32_t g = lo;
        const uint8_t cur = s->status[g], nw = status[r];
        if (status_rank(nw) < status_rank(cur)) { free(pos); return -10; }
        const int has_info = (nw >= S_ACCEPTED && nw <= S_APPLIED) || nw == S_TRUNC_APPLY;
        if (has_info) {
            if (!emsb) { free(pos); return -1; }
            if (or_ts_compare(emsb[r], elsb[r], enode[r], s->tbl[g].msb, s->tbl[g].lsb, s->tbl[g].node) < 0) { free(pos); return -1; }
            const int cur_committed = cur >= S_COMMITTED && cur <= S_APPLIED;
            if (cur_committed && (emsb[r] != s->exec[g].msb || elsb[r] != s->exec[g].lsb || enode[r] != s->exec[g].node)) {
                free(pos); return -10;
            }
        }
        pos[r] = g;
    }
    for (uint32_t r = 0; r < n; ++r) {
        const uint32_t g = pos[r];
        const uint8_t nw = status[r];
        const int has_info = (nw >= S_ACCEPTED && nw <= S_APPLIED) || nw == S_TRUNC_APPLY;
        ts_t ex = s->exec[g];
        if (has_info) { ex.msb = emsb[r]; ex.lsb = elsb[r]; ex.node = enode[r]; }
        const uint8_t was = s->status[g];
        s->status[g] = nw;
        s->exec[g] = ex;
        if (s->event_mode && nw >= S_STABLE && nw < S_INVALID_OR_TRUNCATED && was < S_STABLE) {
            or_waiter *x = waiter_of(s, g);                  /* hasBeen(Stable): registerUnmanaged */
            if (x && waiter_unmanaged(s, x)) lstore_register_unmanaged(s, x);
        }
        if (is_globally_visible(kind_of(s->tbl[g].lsb)) != 1) continue;   /* never inserted into CFK */
        if (domain_of(s->tbl[g].lsb) != 0) continue;                       /* range command: status only */
        /* TruncatedApply, Erased and Invalidated leave CommandsForKey as INVALID_OR_TRUNCATED does */
        const uint8_t cs = nw >= S_INVALID_OR_TRUNCATED ? (uint8_t)S_INVALID_OR_TRUNCATED : nw;
        for (uint32_t p = s->koff[g]; p < s->koff[g + 1]; ++p) {
            cfk_t *c = &s->cfks[s->kord[p]];
            if (g < c->redundant_before) continue;       /* truncated from this key */
            const long at = cfk_search(c, s->tbl, &s->tbl[g]);
            const uint8_t prev = at >= 0 ? c->txns[at].status : S_TRANSITIVELY_KNOWN;
            if (cfk_update_status(c, s->tbl, g, cs, &ex)) { free(pos); return -1; }
            if (s->event_mode) lstore_event(s, s->kord[p], g, prev, cs, &ex);
        }
    }
    free(pos);
    return 0;
}

uint32_t or_lstore_size(const or_lstore *s) { return s->n; }

int or_lstore_truncate(or_lstore *s, uint32_t m, const uint32_t *start, const uint32_t *end, const uint32_t *bound)
{
    for (uint32_t e = 0; e < m; ++e) if (start[e] >= end[e] || (e && end[e - 1] > start[e])) return -1;
    uint32_t e = 0;
    for (uint32_t k = 0; k < s->nkeys; ++k) {
        while (e < m && end[e] < k) ++e;                 /* first entry with end >= k */
        if (e == m || !(start[e] < k)) continue;         /* k in (start, end] */
        if (bound[e] == 0xFFFFFFFFu) continue;           /* Timestamp.NONE */
        cfk_t *c = &s->cfks[k];
        if (bound[e] < c->redundant_before) return -1;    /* checkArgument: never goes back (:1656) */
        c->redundant_before = bound[e];
        uint32_t pos = 0;                                /* insertPos(0, bound) (:1664) */
        while (pos < c->n && c->txns[pos].txn < bound[e]) ++pos;
        if (pos == 0) continue;
        txninfo_t *nt = (txninfo_t *)malloc(((size_t)(c->n - pos) + 1) * sizeof(txninfo_t));
        if (!nt) return -1;
        memcpy(nt, c->txns + pos, (size_t)(c->n - pos) * sizeof(txninfo_t));
        if (cfk_rebuild(c, nt, c->n - pos)) return -1;
        if (s->event_mode) {                 /* notifyAndUpdatePending(safeStore, prevCfk) (:1205-1213) */
            long min_unc, next, nwr;
            cfk_nexts(s, c, &min_unc, &next, &nwr);
            if (min_unc < 0 || next >= 0) cfk_notify_unmanaged(s, k, 0, min_unc, next);
        }
    }
    return 0;
}


/* ------------------------------------------------------------------------------------------
 * Execution readiness of a registered-status store: the WaitingOn of every
 * txn whose WaitingOn was initialised (Commands.initialiseWaitingOn, local/Commands.java:735-753),
 * cleared as the store's statuses change, until the txn is ReadyToExecute (maybeExecute, :656-733).
 * Each or_lstore_ready call evaluates, against the current CommandsForKey state, the tests the
 * reference evaluates when an event reaches a key:
 *  - range-dep bits: Commands.updateWaitingOn (:769-830) for every dep that hasBeen(PreCommitted);
 *  - key bits of managed txns (key domain, globally visible; STABLE): CommandsForKey.notify's count
 *    test (local/CommandsForKey.java:1512-1635): expectMissingCount (unapplied committed txns before
 *    the txn's executeAt in committed[] plus uncommitted txns with a lower TxnId, by the kinds it
 *    witnesses) == |missing| (the uncommitted txns it witnesses with TxnId < executeAt that its
 *    deps lack: computeInfoAndAdditions :1071-1140, committed ones elided :1103-1109);
 *  - key bits of unmanaged txns (range domain, EphemeralRead; hasBeen Stable):
 *    registerUnmanaged (:1406-1498) once, then updatePending on a COMMIT record whose waitingUntil
 *    precedes minUncommitted (:1243-1262, :1315-1360) and the APPLY release of notifyUnmanaged
 *    (:1264-1283) with next / minUncommitted as the constructor derives them (:422-470).
 * The reference evaluates these tests when an event reaches the key (notifyAndUpdatePending,
 * :1163-1215); here they are evaluated for every waiting txn at every call (a txn is released at
 * the first call at which its test holds).  Ready = no bit left and status STABLE.  A waiting txn
 * that is invalidated or truncated (INVALID_OR_TRUNCATED, Erased) leaves the set unreported: the
 * reference never executes it (Commands.maybeExecute needs Stable).
 * ------------------------------------------------------------------------------------------ */
typedef struct or_waiter {
    uint32_t g, nr, nk;
    uint32_t *rdeps;             /* [nr] RangeDeps txnIds (positions) */
    uint32_t *keys;              /* [nk] KeyDeps keys */
    uint32_t *kdoff, *kdeps;     /* per key its KeyDeps txnIds (positions, ascending) */
    uint64_t *words, *aoi;       /* WaitingOn bits: [0, nr) txnIds, [nr, nr + nk) keys */
    uint8_t *pend;               /* per key (unmanaged): 0 unregistered, 1 COMMIT, 2 APPLY, 3 released */
    uint32_t *until;             /* per key: the waitingUntil txn (position) */
    uint32_t nrr;                /* its RangeDeps ranges (rrs, rre] and their txn index lists */
    uint32_t *rrs, *rre, *r2voff, *r2v;
    ts_t eal;                    /* WaitingOn.executeAtLeast (local/Command.java:1409-1513), when has_eal */
    int has_eal;
} or_waiter;

static void waiter_free(or_waiter *x)
{
    free(x->rdeps); free(x->keys); free(x->kdoff); free(x->kdeps); free(x->words); free(x->aoi);
    free(x->pend); free(x->until); free(x->rrs); free(x->rre); free(x->r2voff); free(x->r2v);
}

static void or_lstore_waiters_free(or_lstore *s)
{
    for (uint32_t w = 0; w < s->nwt; ++w) waiter_free(&s->wt[w]);
    free(s->wt);
    s->wt = NULL; s->nwt = s->cwt = 0;
}

static int lstore_remove_redundant(const or_lstore *s, struct or_waiter *x, const ts_t *ex);

int or_lstore_waiting_add(or_lstore *s, uint32_t base, const or_deps *d, uint32_t n)
{
    if (s->nwt + n > s->cwt) {
        uint32_t c = s->cwt ? s->cwt : 1024;
        while (c < s->nwt + n) c *= 2;
        or_waiter *nw = (or_waiter *)realloc(s->wt, (size_t)c * sizeof(or_waiter));
        if (!nw) return -1;
        s->wt = nw; s->cwt = c;
    }
    for (uint32_t i = 0; i < n; ++i) {
        or_waiter *x = &s->wt[s->nwt];
        memset(x, 0, sizeof(*x));
        x->g = base + i;
        x->nr = d->rd_val_off[i + 1] - d->rd_val_off[i];
        x->nk = d->kd_key_off[i + 1] - d->kd_key_off[i];
        const uint32_t nw = (x->nr + x->nk + 63) / 64;
        const int32_t *k2v = d->kd_k2v + d->kd_k2v_off[i];
        const uint32_t body = d->kd_k2v_off[i + 1] - d->kd_k2v_off[i] - x->nk;
        x->rdeps = (uint32_t *)malloc(((size_t)x->nr + 1) * 4);
        x->keys = (uint32_t *)malloc(((size_t)x->nk + 1) * 4);
        x->kdoff = (uint32_t *)malloc(((size_t)x->nk + 1) * 4);
        x->kdeps = (uint32_t *)malloc(((size_t)body + 1) * 4);
        x->words = (uint64_t *)calloc(nw + 1, 8);
        x->aoi = (uint64_t *)calloc(nw + 1, 8);
        x->pend = (uint8_t *)calloc((size_t)x->nk + 1, 1);
        x->until = (uint32_t *)calloc((size_t)x->nk + 1, 4);
        if (!x->rdeps || !x->keys || !x->kdoff || !x->kdeps || !x->words || !x->aoi || !x->pend || !x->until) return -1;
        x->nrr = d->rd_rng_off ? d->rd_rng_off[i + 1] - d->rd_rng_off[i] : 0;
        const uint32_t rbody = x->nrr ? d->rd_r2v_off[i + 1] - d->rd_r2v_off[i] - x->nrr : 0;
        x->rrs = (uint32_t *)malloc(((size_t)x->nrr + 1) * 4);
        x->rre = (uint32_t *)malloc(((size_t)x->nrr + 1) * 4);
        x->r2voff = (uint32_t *)malloc(((size_t)x->nrr + 1) * 4);
        x->r2v = (uint32_t *)malloc(((size_t)rbody + 1) * 4);
        if (!x->rrs || !x->rre || !x->r2voff || !x->r2v) return -1;
        x->r2voff[0] = 0;
        for (uint32_t q = 0; q < x->nrr; ++q) {           /* RangeDeps: ranges, then per range its txn indices */
            x->rrs[q] = d->rd_rng_start[d->rd_rng_off[i] + q];
            x->rre[q] = d->rd_rng_end[d->rd_rng_off[i] + q];
            const int32_t *blk = d->rd_r2v + d->rd_r2v_off[i];
            const uint32_t b = q == 0 ? x->nrr : (uint32_t)blk[q - 1], e = (uint32_t)blk[q];
            for (uint32_t y = b; y < e; ++y) x->r2v[x->r2voff[q] + (y - b)] = (uint32_t)blk[y];
            x->r2voff[q + 1] = x->r2voff[q] + (e - b);
        }
        for (uint32_t j = 0; j < x->nr; ++j) x->rdeps[j] = d->rd_vals[d->rd_val_off[i] + j];
        x->kdoff[0] = 0;
        for (uint32_t q = 0; q < x->nk; ++q) {
            x->keys[q] = d->kd_keys[d->kd_key_off[i] + q];
            const uint32_t b = q == 0 ? x->nk : (uint32_t)k2v[q - 1], e = (uint32_t)k2v[q];
            for (uint32_t y = b; y < e; ++y) x->kdeps[x->kdoff[q] + (y - b)] = d->kd_vals[d->kd_val_off[i] + (uint32_t)k2v[y]];
            x->kdoff[q + 1] = x->kdoff[q] + (e - b);
        }
        for (uint32_t b = 0; b < x->nr + x->nk; ++b) x->words[b / 64] |= 1ULL << (b & 63);
        ++s->nwt;
        /* initialiseWaitingOn's updateWaitingOn removes the redundant deps under the map of that time
         * (local/Commands.java:735-761); its dep visit is the first or_lstore_ready evaluation */
        if (lstore_remove_redundant(s, x, &s->exec[x->g])) return -1;
    }
    if (s->event_mode) {
        /* the WaitingOn exists from the txn's STABLE transition (initialiseWaitingOn): the txns that are
         * Stable already take that transition's CommandsForKey step now, in TxnId order */
        if (wix_rebuild(s)) return -1;
        for (uint32_t i = 0; i < n; ++i) {
            or_waiter *x = waiter_of(s, base + i);
            if (!x) continue;
            const uint32_t g = x->g;
            const uint8_t st = s->status[g];
            if (st < S_STABLE || st >= S_INVALID_OR_TRUNCATED) continue;
            if (waiter_unmanaged(s, x)) { lstore_register_unmanaged(s, x); continue; }
            if (st != S_STABLE) continue;
            for (uint32_t p = s->koff[g]; p < s->koff[g + 1]; ++p)
                if (g >= s->cfks[s->kord[p]].redundant_before) lstore_event(s, s->kord[p], g, S_STABLE, S_STABLE, &s->exec[g]);
        }
    }
    return 0;
}

uint32_t or_lstore_waiting(const or_lstore *s) { return s->nwt; }

static inline int w_test(const uint64_t *w, uint32_t b) { return (int)((w[b / 64] >> (b & 63)) & 1u); }
static inline void w_clear(uint64_t *w, uint32_t b) { w[b / 64] &= ~(1ULL << (b & 63)); }

/* the CommandsForKey constructor's minUncommitted and next (local/CommandsForKey.java:432-461):
 * positions, or -1 */
static void cfk_next(const cfk_t *c, long *min_unc, long *next)
{
    *min_unc = -1; *next = -1;
    const txninfo_t *best = NULL;
    for (uint32_t i = 0; i < c->n; ++i) {
        const txninfo_t *t = &c->txns[i];
        if (t->status == S_INVALID_OR_TRUNCATED) continue;
        if (t->status >= S_COMMITTED) {
            if (t->status < S_APPLIED && (!best || ts_cmp(&best->execute_at, &t->execute_at) > 0)) best = t;
        } else if (*min_unc < 0) *min_unc = t->txn;
    }
    if (best) *next = best->txn;
    /* next is nulled when minUncommitted precedes its executeAt (:454-455) */
    (void)0;
}

/* registerUnmanaged (:1406-1498) / updatePending (:1315-1360) over the deps of one key: returns 1 =
 * ready, 0 = pending APPLY (*until = the relevant dep executing last), -1 = pending COMMIT (*until =
 * the last dep), for a waiter at executeAt ex; `reg` = registration (uncommitted deps -> COMMIT) */
static int unmanaged_eval(const or_lstore *s, const cfk_t *c, const or_waiter *x, uint32_t q, const ts_t *ex,
                          int only_deps, int reg, uint32_t *until, long *executes_at)
{
    *executes_at = -1;
    const uint32_t *dl = x->kdeps + x->kdoff[q];
    const uint32_t nd = x->kdoff[q + 1] - x->kdoff[q];
    uint32_t i = 0;
    while (i < nd && dl[i] < c->redundant_before) ++i;          /* txnIds.find(shardRedundantBefore) */
    if (i >= nd) return 1;
    int ready = 1, to_apply = 1;
    long best = -1;
    for (; i < nd; ++i) {
        const long j = cfk_search(c, s->tbl, &s->tbl[dl[i]]);
        if (j < 0) { ready = to_apply = 0; continue; }          /* missing from this CFK */
        const txninfo_t *t = &c->txns[j];
        if (reg && t->status < S_COMMITTED) { ready = to_apply = 0; continue; }
        if (only_deps || ts_cmp(&t->execute_at, ex) < 0) {
            ready &= t->status >= S_APPLIED;
            if (best < 0 || ts_cmp(&s->exec[best], &t->execute_at) < 0) best = t->txn;
        }
    }
    if (ready) return 1;
    *executes_at = best;                                        /* executesAt: the relevant dep executing last */
    if (to_apply) { *until = best < 0 ? dl[nd - 1] : (uint32_t)best; return 0; }
    *until = dl[nd - 1];
    return -1;
}

int or_lstore_redundant(or_lstore *s, uint32_t m, const uint32_t *start, const uint32_t *end, const uint64_t *sep,
                        const uint64_t *eep, const uint32_t *local, const uint32_t *boot, const uint8_t *stale)
{
    for (uint32_t e = 0; e < m; ++e) if (start[e] >= end[e] || (e && end[e - 1] > start[e])) return -1;
    free(s->rr_s); free(s->rr_e); free(s->rr_local); free(s->rr_boot); free(s->rr_sep); free(s->rr_eep); free(s->rr_stale);
    s->rr_s = s->rr_e = s->rr_local = s->rr_boot = NULL; s->rr_sep = s->rr_eep = NULL; s->rr_stale = NULL;
    s->rr_m = 0;
    if (!m) return 0;
    s->rr_s = (uint32_t *)malloc((size_t)m * 4); s->rr_e = (uint32_t *)malloc((size_t)m * 4);
    s->rr_local = (uint32_t *)malloc((size_t)m * 4); s->rr_boot = (uint32_t *)malloc((size_t)m * 4);
    s->rr_sep = (uint64_t *)malloc((size_t)m * 8); s->rr_eep = (uint64_t *)malloc((size_t)m * 8);
    s->rr_stale = (uint8_t *)malloc(m);
    if (!s->rr_s || !s->rr_e || !s->rr_local || !s->rr_boot || !s->rr_sep || !s->rr_eep || !s->rr_stale) return -1;
    memcpy(s->rr_s, start, (size_t)m * 4); memcpy(s->rr_e, end, (size_t)m * 4);
    memcpy(s->rr_local, local, (size_t)m * 4); memcpy(s->rr_boot, boot, (size_t)m * 4);
    memcpy(s->rr_sep, sep, (size_t)m * 8); memcpy(s->rr_eep, eep, (size_t)m * 8);
    memcpy(s->rr_stale, stale, m);
    s->rr_m = m;
    return 0;
}

/* RedundantStatus (local/RedundantStatus.java) in declaration order, and its merge table (:91-141) */
enum { RS_NOT_OWNED, RS_LIVE, RS_PARTIALLY_PRE_BOOTSTRAP_OR_STALE, RS_PRE_BOOTSTRAP_OR_STALE,
       RS_REDUNDANT_PRE_BOOTSTRAP_OR_STALE, RS_LOCALLY_REDUNDANT, RS_SHARD_REDUNDANT };
static const uint8_t RS_MERGE[7][7] = {
    /* NOT_OWNED */ {0, 1, 2, 3, 4, 5, 6},
    /* LIVE      */ {1, 1, 2, 2, 4, 4, 4},
    /* PARTIALLY */ {2, 2, 2, 2, 4, 4, 4},
    /* PRE_BOOT  */ {3, 2, 2, 3, 4, 4, 4},
    /* RED_PRE   */ {4, 4, 4, 4, 4, 4, 4},
    /* LOCALLY   */ {5, 4, 4, 4, 4, 5, 5},
    /* SHARD     */ {6, 4, 4, 4, 4, 5, 6},
};

/* does the map entry (es, ee] meet the participants of the txn at position g (its keys or ranges)? */
static int rr_meets(const or_lstore *s, uint32_t g, uint32_t es, uint32_t ee)
{
    if (domain_of(s->tbl[g].lsb) != 0) {
        for (uint32_t a = s->roff[g]; a < s->roff[g + 1]; ++a)
            if (range_intersects_range(es, ee, s->rst[a], s->ren[a])) return 1;
        return 0;
    }
    for (uint32_t p = s->koff[g]; p < s->koff[g + 1]; ++p)
        if (range_intersects_key(es, ee, s->kord[p])) return 1;
    return 0;
}

/* d.txnIds().find(bound), insertion point (positions ascend with TxnIds); TxnId.NONE precedes all */
static uint32_t rr_find(const or_waiter *x, uint32_t bound)
{
    if (bound == 0xFFFFFFFFu) return 0;
    uint32_t lo = 0, hi = x->nr;
    while (lo < hi) { uint32_t m = (lo + hi) / 2; if (x->rdeps[m] < bound) lo = m + 1; else hi = m; }
    return lo;
}

typedef struct { uint32_t n, cap; uint32_t *a, *b; } rr_set;   /* disjoint intervals (a, b] */

static int rr_set_push(rr_set *r, uint32_t a, uint32_t b)
{
    if (r->n == r->cap) {
        uint32_t c = r->cap ? r->cap * 2 : 8;
        uint32_t *na = (uint32_t *)realloc(r->a, (size_t)c * 4), *nb;
        if (!na) return -1;
        r->a = na;
        nb = (uint32_t *)realloc(r->b, (size_t)c * 4);
        if (!nb) return -1;
        r->b = nb; r->cap = c;
    }
    r->a[r->n] = a; r->b[r->n] = b; ++r->n;
    return 0;
}

/* Commands.updateWaitingOn's removal step (local/Commands.java:755-761):
 * CommandStore.hasLocallyRedundantDependencies(minWaitingOnTxnId, executeAt, participants)
 * (local/CommandStore.java:672-678: RedundantBefore.status >= PARTIALLY_PRE_BOOTSTRAP_OR_STALE, folding
 * Entry.getAndMerge :157-161 / get :225-240 over the entries the participants touch), then
 * CommandStore.removeRedundantDependencies (:601-670) literally: per entry, ascending, the range deps
 * meeting its range with txnIdx in [bootstrapIdx, appliedIdx) stop being waited on, and those below
 * bootstrapIdx whose every range is covered by bootstrapping entries (RangeState.isFullyBootstrapping,
 * the remaining ranges carried across entries).  Range-dep bits only (WaitingOn.txnIds = RangeDeps). */
static int lstore_remove_redundant(const or_lstore *s, or_waiter *x, const ts_t *ex)
{
    if (!s->rr_m || !x->nr) return 0;
    uint32_t j0 = 0xFFFFFFFFu;                            /* WaitingOn.Update.minWaitingOnTxnId (:1500-1504) */
    for (uint32_t b = 0; b < x->nr + x->nk; ++b) if (w_test(x->words, b)) { j0 = b; break; }
    if (j0 >= x->nr) return 0;
    const uint32_t g = x->g, mpos = x->rdeps[j0];
    const uint64_t min_epoch = s->tbl[mpos].msb >> 15, exec_epoch = ex->msb >> 15;
    int st = RS_NOT_OWNED;
    for (uint32_t e = 0; e < s->rr_m; ++e) {
        if (!rr_meets(s, g, s->rr_s[e], s->rr_e[e])) continue;
        if (exec_epoch < s->rr_sep[e] || min_epoch >= s->rr_eep[e]) continue;        /* outOfBounds */
        int es;                                                                        /* Entry.get(minId) */
        if (s->rr_stale[e] || (s->rr_boot[e] != 0xFFFFFFFFu && s->rr_boot[e] > mpos)) es = RS_PRE_BOOTSTRAP_OR_STALE;
        else if (s->rr_local[e] != 0xFFFFFFFFu && s->rr_local[e] > mpos) es = RS_LOCALLY_REDUNDANT;   /* or SHARD_: same here */
        else es = RS_LIVE;
        st = RS_MERGE[st][es];
    }
    if (st < RS_PARTIALLY_PRE_BOOTSTRAP_OR_STALE) return 0;
    rr_set *part = (rr_set *)calloc(x->nr ? x->nr : 1, sizeof(rr_set));   /* partiallyBootstrapping */
    uint8_t *has = (uint8_t *)calloc(x->nr ? x->nr : 1, 1);
    int rc = -1;
    if (!part || !has) goto out;
    for (uint32_t e = 0; e < s->rr_m; ++e) {
        if (!rr_meets(s, g, s->rr_s[e], s->rr_e[e])) continue;
        const uint32_t es = s->rr_s[e], ee = s->rr_e[e];
        const uint32_t bidx = rr_find(x, s->rr_boot[e]), aidx = rr_find(x, s->rr_local[e]);
        if (aidx > bidx)                                   /* d.forEach(e.range): the txns of its ranges meeting it */
            for (uint32_t q = 0; q < x->nrr; ++q) {
                if (!range_intersects_range(x->rrs[q], x->rre[q], es, ee)) continue;
                for (uint32_t y = x->r2voff[q]; y < x->r2voff[q + 1]; ++y) {
                    const uint32_t j = x->r2v[y];
                    if (j >= bidx && j < aidx) w_clear(x->words, j);
                }
            }
        if (bidx > 0)
            for (uint32_t q = 0; q < x->nrr; ++q) {
                if (!range_intersects_range(x->rrs[q], x->rre[q], es, ee)) continue;
                for (uint32_t y = x->r2voff[q]; y < x->r2voff[q + 1]; ++y) {
                    const uint32_t j = x->r2v[y];
                    if (!(j < bidx && w_test(x->words, j))) continue;
                    /* isFullyBootstrapping(j): every range of j inside e.range, else j's remaining ranges
                     * (first: all of them) minus e.range, fully when none remain */
                    int fully = 1;
                    for (uint32_t q2 = 0; q2 < x->nrr && fully; ++q2)
                        for (uint32_t y2 = x->r2voff[q2]; y2 < x->r2voff[q2 + 1]; ++y2)
                            if (x->r2v[y2] == j && !(es <= x->rrs[q2] && x->rre[q2] <= ee)) { fully = 0; break; }
                    if (!fully) {
                        rr_set *r = &part[j];
                        if (!has[j]) {
                            has[j] = 1;
                            for (uint32_t q2 = 0; q2 < x->nrr; ++q2)
                                for (uint32_t y2 = x->r2voff[q2]; y2 < x->r2voff[q2 + 1]; ++y2)
                                    if (x->r2v[y2] == j && rr_set_push(r, x->rrs[q2], x->rre[q2])) goto out;
                        }
                        rr_set nr = {0, 0, NULL, NULL};
                        for (uint32_t u = 0; u < r->n; ++u) {          /* remaining.subtract(e.range) */
                            const uint32_t a = r->a[u], b = r->b[u];
                            if (a < (b < es ? b : es) && rr_set_push(&nr, a, b < es ? b : es)) { free(nr.a); free(nr.b); goto out; }
                            if ((a > ee ? a : ee) < b && rr_set_push(&nr, a > ee ? a : ee, b)) { free(nr.a); free(nr.b); goto out; }
                        }
                        free(r->a); free(r->b);
                        *r = nr;
                        fully = r->n == 0;
                    }
                    if (fully) w_clear(x->words, j);
                }
            }
    }
    rc = 0;
out:
    if (part) for (uint32_t j = 0; j < x->nr; ++j) { free(part[j].a); free(part[j].b); }
    free(part); free(has);
    return rc;
}

static void eal_merge(or_waiter *x, const ts_t *t)          /* updateExecuteAtLeast: Timestamp.nonNullOrMax */
{
    if (!x->has_eal || ts_cmp(&x->eal, t) < 0) { x->eal = *t; x->has_eal = 1; }
}

/* CommandsForKey.notify's test for the STABLE managed waiter x on its key slot q
 * (local/CommandsForKey.java:1512-1635): expectMissingCount == |missing| */
static int managed_test(const or_lstore *s, const cfk_t *c, const or_waiter *x, uint32_t q)
{
    const uint32_t g = x->g;
    const ts_t *ex = &s->exec[g];
    const int wk = witnesses_of(kind_of(s->tbl[g].lsb));
    uint32_t expect = 0, missing = 0;
    for (uint32_t a = 0; a < c->nc; ++a) {              /* committed[], executeAt order */
        const txninfo_t *t = &c->txns[c->committed[a]];
        if (ts_cmp(&t->execute_at, ex) >= 0) break;
        if (t->status == S_APPLIED) continue;
        if (kinds_test(wk, kind_of(s->tbl[t->txn].lsb))) ++expect;
    }
    const uint32_t *dl = x->kdeps + x->kdoff[q];
    const uint32_t nd = x->kdoff[q + 1] - x->kdoff[q];
    for (uint32_t a = 0; a < c->n; ++a) {               /* backfill: uncommitted, TxnId order */
        const txninfo_t *t = &c->txns[a];
        if (ts_cmp(&s->tbl[t->txn], ex) >= 0) break;
        if (t->status >= S_COMMITTED || t->txn == g) continue;
        if (!kinds_test(wk, kind_of(s->tbl[t->txn].lsb))) continue;
        ++expect;
        uint32_t lo = 0, hi = nd;                        /* in its deps? */
        while (lo < hi) { uint32_t m = (lo + hi) / 2; if (dl[m] < t->txn) lo = m + 1; else hi = m; }
        if (!(lo < nd && dl[lo] == t->txn)) ++missing;
    }
    return expect == missing;
}

/* the unmanaged waiter x's key slot q: registerUnmanaged (:1406-1498) */
static void unmanaged_register(const or_lstore *s, const cfk_t *c, or_waiter *x, uint32_t q)
{
    const int kind = kind_of(s->tbl[x->g].lsb), only_deps = kind == K_EXCL_SYNC_POINT || kind == K_EPHEMERAL_READ;
    long ea;
    const int r = unmanaged_eval(s, c, x, q, &s->exec[x->g], only_deps, 1, &x->until[q], &ea);
    if (r == 1) { x->pend[q] = 3; w_clear(x->words, x->nr + q); return; }
    x->pend[q] = r == 0 ? 2 : 1;
    if (r == 0 && only_deps && ea >= 0) eal_merge(x, &s->exec[ea]);   /* :1470-1478 */
}

/* notifyUnmanaged(COMMIT, minUncommitted) for a COMMIT record: updatePending (:1315-1360) */
static void unmanaged_commit(const or_lstore *s, const cfk_t *c, or_waiter *x, uint32_t q, long min_unc)
{
    if (x->pend[q] != 1 || !(min_unc < 0 || (uint32_t)min_unc > x->until[q])) return;
    const int kind = kind_of(s->tbl[x->g].lsb), only_deps = kind == K_EXCL_SYNC_POINT || kind == K_EPHEMERAL_READ;
    long ea;
    const int r = unmanaged_eval(s, c, x, q, &s->exec[x->g], only_deps, 0, &x->until[q], &ea);
    if (r == 1) { x->pend[q] = 3; w_clear(x->words, x->nr + q); return; }
    x->pend[q] = 2;
    if (only_deps && ea >= 0) eal_merge(x, &s->exec[ea]);                /* :1370-1380 */
}

/* notifyUnmanaged(APPLY, next.executeAt) for an APPLY record (:1264-1283); next < 0: Timestamp.MAX */
static void unmanaged_apply(const or_lstore *s, or_waiter *x, uint32_t q, long next)
{
    if (x->pend[q] == 2 && (next < 0 || ts_cmp(&s->exec[x->until[q]], &s->exec[next]) < 0)) {
        x->pend[q] = 3; w_clear(x->words, x->nr + q);
    }
}

/* ---- event mode: key bits are cleared when notifyAndUpdatePending's events reach the key ---- */
void or_lstore_event_mode(or_lstore *s, int on) { s->event_mode = on; }

static int wix_rebuild(or_lstore *s)
{
    if (s->wix_cap < s->n + 1) {
        uint32_t *w = (uint32_t *)realloc(s->wix, ((size_t)s->cap + 1) * 4);
        if (!w) return -1;
        s->wix = w; s->wix_cap = s->cap + 1;
    }
    memset(s->wix, 0, (size_t)s->wix_cap * 4);
    for (uint32_t w = 0; w < s->nwt; ++w) s->wix[s->wt[w].g] = w + 1;
    return 0;
}

static or_waiter *waiter_of(const or_lstore *s, uint32_t g)
{
    return s->wix && g < s->wix_cap && s->wix[g] ? &s->wt[s->wix[g] - 1] : NULL;
}

static long waiter_slot(const or_waiter *x, uint32_t k)          /* KeyDeps key slot of k, or -1 */
{
    uint32_t lo = 0, hi = x->nk;
    while (lo < hi) { uint32_t m = (lo + hi) / 2; if (x->keys[m] < k) lo = m + 1; else hi = m; }
    return lo < x->nk && x->keys[lo] == k ? (long)lo : -1;
}

/* the CommandsForKey constructor's minUncommitted, next, nextWrite (:432-461), positions or -1 */
static void cfk_nexts(const or_lstore *s, const cfk_t *c, long *min_unc, long *next, long *next_write)
{
    *min_unc = *next = *next_write = -1;
    for (uint32_t i = 0; i < c->n; ++i) {
        const txninfo_t *t = &c->txns[i];
        if (t->status == S_INVALID_OR_TRUNCATED) continue;
        if (t->status >= S_COMMITTED) {
            if (t->status < S_APPLIED) {
                if (kind_of(s->tbl[t->txn].lsb) == K_WRITE && (*next_write < 0 || ts_cmp(&s->exec[*next_write], &t->execute_at) > 0))
                    *next_write = t->txn;
                if (*next < 0 || ts_cmp(&s->exec[*next], &t->execute_at) > 0) *next = t->txn;
            }
        } else if (*min_unc < 0) *min_unc = t->txn;
    }
    if (*min_unc >= 0) {
        if (*next >= 0 && ts_cmp(&s->tbl[*min_unc], &s->exec[*next]) < 0) *next = -1;
        if (*next_write >= 0 && ts_cmp(&s->tbl[*min_unc], &s->exec[*next_write]) < 0) *next_write = -1;
    }
}

/* notify(kinds, from, to) (:1501-1511): the STABLE waiters in committed[] executing in [from, to]
 * (from NULL = Timestamp.NONE, to NULL = Timestamp.MAX) run the count test on key k */
static void cfk_notify(or_lstore *s, uint32_t k, const ts_t *from, const ts_t *to)
{
    const cfk_t *c = &s->cfks[k];
    uint32_t i = 0;
    if (from) while (i < c->nc && ts_cmp(&c->txns[c->committed[i]].execute_at, from) < 0) ++i;
    for (; i < c->nc; ++i) {
        const txninfo_t *t = &c->txns[c->committed[i]];
        if (to && ts_cmp(&t->execute_at, to) > 0) break;
        if (t->status != S_STABLE) continue;
        or_waiter *x = waiter_of(s, t->txn);
        if (!x || s->status[x->g] != S_STABLE) continue;
        const long q = waiter_slot(x, k);
        if (q < 0 || !w_test(x->words, x->nr + (uint32_t)q)) continue;
        if (managed_test(s, c, x, (uint32_t)q)) w_clear(x->words, x->nr + (uint32_t)q);
    }
}

static int waiter_unmanaged(const or_lstore *s, const or_waiter *x)
{
    return !(domain_of(s->tbl[x->g].lsb) == 0 && is_globally_visible(kind_of(s->tbl[x->g].lsb)) == 1);
}

/* notifyUnmanaged(COMMIT / APPLY) over the unmanaged records of key k (:1264-1283) */
static void cfk_notify_unmanaged(or_lstore *s, uint32_t k, int commit, long min_unc, long next)
{
    const cfk_t *c = &s->cfks[k];
    for (uint32_t w = 0; w < s->nwt; ++w) {
        or_waiter *x = &s->wt[w];
        if (!waiter_unmanaged(s, x)) continue;
        const long q = waiter_slot(x, k);
        if (q < 0 || !w_test(x->words, x->nr + (uint32_t)q)) continue;
        if (commit) unmanaged_commit(s, c, x, (uint32_t)q, min_unc);
        else unmanaged_apply(s, x, (uint32_t)q, next);
    }
}

/* CommandsForKey.notifyAndUpdatePending(safeStore, txnId, newStatus, newExecuteAt, prevCfk)
 * (:1163-1215) after the txn at position X moved from prev to nw on key k */
static void lstore_event(or_lstore *s, uint32_t k, uint32_t X, uint8_t prev, uint8_t nw, const ts_t *exec)
{
    long min_unc, next, nwr;
    cfk_nexts(s, &s->cfks[k], &min_unc, &next, &nwr);
    switch (nw) {
    case S_STABLE: case S_COMMITTED: {
        const int cmp = nwr < 0 ? -1 : ts_cmp(exec, &s->exec[nwr]);
        if (cmp <= 0) {
            if (nw == S_COMMITTED) break;
            cfk_notify(s, k, next >= 0 ? &s->exec[next] : NULL, exec);     /* the txn itself may execute */
        } else {
            /* waiters on us may be ready, if we execute after them, were known and not committed */
            if (prev == S_COMMITTED || ts_cmp(&s->exec[nwr], &s->tbl[X]) < 0 || ts_cmp(exec, &s->tbl[X]) == 0) break;
            cfk_notify(s, k, &s->exec[next], &s->exec[nwr]);
        }
        break;
    }
    case S_APPLIED: case S_INVALID_OR_TRUNCATED:
        if (next >= 0) cfk_notify(s, k, &s->exec[next], nwr >= 0 ? &s->exec[nwr] : NULL);
        break;
    default: break;
    }
    if (nw >= S_COMMITTED && prev < S_COMMITTED) cfk_notify_unmanaged(s, k, 1, min_unc, next);
    if (min_unc < 0 || next >= 0) cfk_notify_unmanaged(s, k, 0, min_unc, next);
}

/* an unmanaged waiter that has now been Stable: registerUnmanaged on its keys */
static void lstore_register_unmanaged(or_lstore *s, or_waiter *x)
{
    for (uint32_t q = 0; q < x->nk; ++q)
        if (w_test(x->words, x->nr + q) && x->pend[q] == 0) unmanaged_register(s, &s->cfks[x->keys[q]], x, q);
}

/* a released Range-domain waiter keeps its appliedOrInvalidated for setAppliedAndPropagate */
static int pv_save(or_lstore *s, const or_waiter *x)
{
    uint32_t cnt = 0;
    for (uint32_t j = 0; j < x->nr; ++j) cnt += w_test(x->aoi, j);
    if (!cnt) return 0;
    if (s->pv_cap_pos < s->cap) {
        uint32_t *a = (uint32_t *)realloc(s->pv_at, (size_t)s->cap * 4), *b;
        if (!a) return -1;
        s->pv_at = a;
        b = (uint32_t *)realloc(s->pv_len, (size_t)s->cap * 4);
        if (!b) return -1;
        s->pv_len = b;
        memset(s->pv_at + s->pv_cap_pos, 0, (size_t)(s->cap - s->pv_cap_pos) * 4);
        memset(s->pv_len + s->pv_cap_pos, 0, (size_t)(s->cap - s->pv_cap_pos) * 4);
        s->pv_cap_pos = s->cap;
    }
    if (s->pv_n + cnt > s->pv_cap) {
        size_t c = s->pv_cap ? s->pv_cap : 4096;
        while (c < s->pv_n + cnt) c *= 2;
        uint32_t *p = (uint32_t *)realloc(s->pv_pool, c * 4);
        if (!p) return -1;
        s->pv_pool = p; s->pv_cap = c;
    }
    s->pv_at[x->g] = (uint32_t)s->pv_n + 1;
    s->pv_len[x->g] = cnt;
    for (uint32_t j = 0; j < x->nr; ++j)
        if (w_test(x->aoi, j)) s->pv_pool[s->pv_n++] = x->rdeps[j];
    return 0;
}

/* WaitingOn.setAppliedAndPropagate(dg, dg's WaitingOn) after dg's own bit was set applied: every txnId
 * both lists hold whose appliedOrInvalidated bit dg has set takes setAppliedOrInvalidated here
 * (forEachIntersection, utils/SortedArrays.java:1231): a waiter without appliedOrInvalidated (key
 * domain) just stops waiting on it (removeWaitingOn), a Range-domain one also records it when it was
 * still waiting on it (:1551-1567).  A dep whose WaitingOn this store never initialised propagates
 * nothing. */
static void pv_propagate(const or_lstore *s, or_waiter *x, uint32_t dg, int rdom)
{
    if (!s->pv_at || dg >= s->pv_cap_pos || !s->pv_at[dg]) return;
    const uint32_t *L = s->pv_pool + (s->pv_at[dg] - 1);
    for (uint32_t a = 0, j = 0; a < s->pv_len[dg] && j < x->nr;) {   /* both ascending */
        if (L[a] < x->rdeps[j]) { ++a; continue; }
        if (L[a] > x->rdeps[j]) { ++j; continue; }
        if (w_test(x->words, j) && !(rdom && w_test(x->aoi, j))) {
            w_clear(x->words, j);
            if (rdom) x->aoi[j / 64] |= 1ULL << (j & 63);
        }
        ++a; ++j;
    }
}

int or_lstore_ready(or_lstore *s, uint32_t *ready_out, uint32_t *nready)
{
    return or_lstore_ready_ex(s, ready_out, nready, NULL, NULL, NULL);
}

int or_lstore_ready_ex(or_lstore *s, uint32_t *ready_out, uint32_t *nready, uint64_t *eal_msb, uint64_t *eal_lsb,
                       int32_t *eal_node)
{
    uint32_t nout = 0, keep = 0;
    for (uint32_t w = 0; w < s->nwt; ++w) {
        or_waiter *x = &s->wt[w];
        const uint32_t g = x->g;
        const uint8_t st = s->status[g];
        const int kind = kind_of(s->tbl[g].lsb), rdom = domain_of(s->tbl[g].lsb);
        const int only_deps = kind == K_EXCL_SYNC_POINT || kind == K_EPHEMERAL_READ;   /* awaitsOnlyDeps */
        const ts_t *ex = &s->exec[g];
        if (st >= S_INVALID_OR_TRUNCATED) {      /* invalidated / truncated: leaves the waiting set, never ready */
            waiter_free(x);
            continue;
        }
        if (lstore_remove_redundant(s, x, ex)) return -1;
        /* range-dep bits: Commands.updateWaitingOn (forEachWaitingOnId: reverse order) */
        for (uint32_t j = x->nr; j-- > 0;) {
            if (!w_test(x->words, j)) continue;
            const uint32_t dg = x->rdeps[j];
            const uint8_t ds = s->status[dg];
            if (ds < S_COMMITTED) continue;                     /* !hasBeen(PreCommitted) */
            /* updateExecuteAtLeast (:782-783): a dep with a known executeAt after the waiter's TxnId --
             * committed, or TruncatedApply (ExecuteAtKnown); an ErasedOrInvalidated / Erased /
             * Invalidated event carries none */
            const int exec_known = ds <= S_APPLIED || ds == S_TRUNC_APPLY;
            if (only_deps && exec_known && ts_cmp(&s->exec[dg], &s->tbl[g]) > 0) eal_merge(x, &s->exec[dg]);
            /* TruncatedApply: Invariants.checkState(executeAt < waitingExecuteAt || awaitsOnlyDeps) (:789-791) */
            if (ds == S_TRUNC_APPLY && !only_deps && ts_cmp(&s->exec[dg], ex) >= 0) return -10;
            if (ds >= S_INVALID_OR_TRUNCATED) { w_clear(x->words, j); if (rdom) x->aoi[j / 64] |= 1ULL << (j & 63); }
            else if (!only_deps && ts_cmp(&s->exec[dg], ex) > 0) w_clear(x->words, j);
            else if (ds == S_APPLIED) {                     /* setAppliedAndPropagate */
                w_clear(x->words, j);
                if (rdom) x->aoi[j / 64] |= 1ULL << (j & 63);
                pv_propagate(s, x, dg, rdom);
            }
        }
        const int managed = rdom == 0 && is_globally_visible(kind) == 1;
        for (uint32_t q = 0; q < x->nk && !s->event_mode; ++q) {   /* event mode: the events clear key bits */
            const uint32_t b = x->nr + q;
            if (!w_test(x->words, b)) continue;
            const cfk_t *c = &s->cfks[x->keys[q]];
            if (managed) {
                if (st == S_STABLE && managed_test(s, c, x, q)) w_clear(x->words, b);
                continue;
            }
            if (st < S_STABLE || st >= S_INVALID_OR_TRUNCATED) continue;   /* hasBeen(Stable), not truncated */
            if (x->pend[q] == 0) {                                   /* registerUnmanaged */
                unmanaged_register(s, c, x, q);
                if (x->pend[q] == 3) continue;
            }
            long min_unc, next;
            cfk_next(c, &min_unc, &next);
            if (next >= 0 && min_unc >= 0 && ts_cmp(&s->tbl[min_unc], &s->exec[next]) < 0) next = -1;
            unmanaged_commit(s, c, x, q, min_unc);                   /* COMMIT -> updatePending */
            if (x->pend[q] == 3) continue;
            if (min_unc < 0 || next >= 0) unmanaged_apply(s, x, q, next);   /* notifyUnmanaged(APPLY, next) */
        }
        int waiting = 0;
        for (uint32_t a = 0; a < (x->nr + x->nk + 63) / 64; ++a) waiting |= x->words[a] != 0;
        if (!waiting && st == S_STABLE) {
            /* Command.executesAtLeast (local/Command.java:1145-1150) */
            const ts_t *ea = only_deps && x->has_eal ? &x->eal : ex;
            if (eal_msb) { eal_msb[nout] = ea->msb; eal_lsb[nout] = ea->lsb; eal_node[nout] = ea->node; }
            ready_out[nout++] = g;
            if (rdom && pv_save(s, x)) return -1;
            waiter_free(x);
            continue;
        }
        s->wt[keep++] = *x;
    }
    s->nwt = keep;
    if (s->event_mode && wix_rebuild(s)) return -1;
    /* ascending positions (the executesAtLeast values move with their txns) */
    for (uint32_t a = 1; a < nout; ++a) {
        uint32_t v = ready_out[a], b = a;
        uint64_t m0 = eal_msb ? eal_msb[a] : 0, l0 = eal_msb ? eal_lsb[a] : 0;
        int32_t n0 = eal_msb ? eal_node[a] : 0;
        while (b > 0 && ready_out[b - 1] > v) {
            ready_out[b] = ready_out[b - 1];
            if (eal_msb) { eal_msb[b] = eal_msb[b - 1]; eal_lsb[b] = eal_lsb[b - 1]; eal_node[b] = eal_node[b - 1]; }
            --b;
        }
        ready_out[b] = v;
        if (eal_msb) { eal_msb[b] = m0; eal_lsb[b] = l0; eal_node[b] = n0; }
    }
    *nready = nout;
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * RedundantBefore.collectDeps (local/RedundantBefore.java:418-421) = ReducingRangeMap.foldl
 * (utils/ReducingRangeMap.java:111-194) of Entry.collectDep (:181-190) over the txn's keys or
 * ranges, into a fresh PartialDeps builder (messages/PreAccept.java:251,260-262).  The map is the
 * reference's (starts[], values[]) form with inclusiveEnds = true (intervals (starts[i],
 * starts[i+1]], matching Range.EndInclusive); it is rebuilt here from the entry list the C ABI takes
 * (a gap between two entries is a null value).  Bounds are stream positions (ACCORD_NO_TXN = NONE).
 * ------------------------------------------------------------------------------------------ */
/* SortedArrays.exponentialSearch over u32 (found: index, else -1 - insertion point) */
static long rb_exp_search(const uint32_t *a, long from, long to, uint32_t key)
{
    long lo = from, hi = to;
    while (lo < hi) {
        long m = (lo + hi) >> 1;
        if (a[m] < key) lo = m + 1; else if (a[m] > key) hi = m; else return m;
    }
    return -1 - lo;
}
/* AbstractRanges.findNext(from, key): the range containing key (start < key <= end), else
 * -1 - the first range after it */
static long rb_ranges_find(const uint32_t *rs, const uint32_t *re, long from, long to, uint32_t key)
{
    long lo = from, hi = to;
    while (lo < hi) {
        long m = (lo + hi) >> 1;
        if (re[m] < key) lo = m + 1; else if (rs[m] >= key) hi = m; else return m;
    }
    return -1 - lo;
}

typedef struct {
    uint32_t nstarts;           /* values: nstarts - 1 */
    uint32_t *starts;
    long *value;                /* entry index or -1 (null) */
} rb_map;

static int rb_map_build(rb_map *M, uint32_t m, const uint32_t *es, const uint32_t *ee)
{
    M->starts = (uint32_t *)malloc((2 * (size_t)m + 1) * sizeof(uint32_t));
    M->value = (long *)malloc((2 * (size_t)m + 1) * sizeof(long));
    M->nstarts = 0;
    if (!M->starts || !M->value) return -1;
    for (uint32_t i = 0; i < m; ++i) {
        if (M->nstarts && M->starts[M->nstarts - 1] == es[i]) {
            M->value[M->nstarts - 1] = i;                   /* adjacent: this interval opens here */
        } else {
            if (M->nstarts) M->value[M->nstarts - 1] = -1;  /* gap between entries: null */
            M->starts[M->nstarts] = es[i];
            M->value[M->nstarts] = i;
            ++M->nstarts;
        }
        M->starts[M->nstarts] = ee[i];
        M->value[M->nstarts] = -1;
        ++M->nstarts;
    }
    return 0;
}

typedef struct {
    const uint64_t *sep, *eep;
    const uint32_t *bound;
    uint64_t min_epoch, exec_epoch;
    const uint32_t *es, *ee;
    mm_builder *b;
    int err;
} rb_fold_ctx;

static void rb_collect_dep(rb_fold_ctx *c, long e)      /* Entry.collectDep (:181-190) */
{
    if (e < 0 || c->err) return;
    /* outOfBounds(lb = minEpoch, ub = executeAt): ub.epoch() < startEpoch || lb.epoch() >= endEpoch */
    if (c->exec_epoch < c->sep[e] || c->min_epoch >= c->eep[e]) return;
    if (c->bound[e] == 0xFFFFFFFFu) return;            /* shardAppliedOrInvalidatedBefore == NONE */
    if (mmb_add(c->b, ((uint64_t)c->es[e] << 32) | c->ee[e], c->bound[e])) c->err = 1;
}

static void rb_foldl_keys(const rb_map *M, const uint32_t *keys, long nk, rb_fold_ctx *c)   /* :138-168 */
{
    const long nv = (long)M->nstarts - 1;
    if (nv <= 0) return;
    long i = 0, j = rb_exp_search(keys, 0, nk, M->starts[0]);
    if (j < 0) j = -1 - j; else ++j;                       /* inclusiveEnds */
    while (j < nk) {
        i = rb_exp_search(M->starts, i, M->nstarts, keys[j]);
        if (i < 0) i = -2 - i; else --i;                   /* inclusiveEnds */
        if (i >= nv) return;
        long nextj = rb_exp_search(keys, j, nk, M->starts[i + 1]);
        if (nextj < 0) nextj = -1 - nextj; else ++nextj;   /* inclusiveEnds */
        if (j != nextj && i >= 0) rb_collect_dep(c, M->value[i]);
        ++i;
        j = nextj;
    }
}

static void rb_foldl_ranges(const rb_map *M, const uint32_t *rs, const uint32_t *re, long nr, rb_fold_ctx *c)   /* :170-208 */
{
    const long nv = (long)M->nstarts - 1;
    if (nv <= 0) return;
    long j = rb_ranges_find(rs, re, 0, nr, M->starts[0]);
    if (j < 0) j = -1 - j; else if (re[j] == M->starts[0]) ++j;
    long i = 0;
    while (j < nr) {
        const uint32_t start = rs[j];
        long nexti = rb_exp_search(M->starts, i, M->nstarts, start);
        if (nexti < 0) i = i > -2 - nexti ? i : -2 - nexti;
        else if (nexti > i) i = nexti - 1;                 /* !inclusiveStarts() */
        else i = nexti;
        if (i >= nv) return;
        long toj, nextj = rb_ranges_find(rs, re, j, nr, M->starts[i + 1]);
        if (nextj < 0) toj = nextj = -1 - nextj;
        else {
            toj = nextj + 1;
            if (re[nextj] == M->starts[i + 1]) ++nextj;
        }
        if (toj > j && i >= 0) rb_collect_dep(c, M->value[i]);
        ++i;
        j = nextj;
    }
}

int or_redundant_collect(const or_stream *s, uint32_t m, const uint32_t *es, const uint32_t *ee, const uint64_t *sep,
                         const uint64_t *eep, const uint32_t *bound, uint64_t min_epoch, or_deps *out)
{
    const uint32_t n = s->n;
    ts_t *tbl = (ts_t *)malloc((size_t)(n ? n : 1) * sizeof(ts_t));
    rb_map M = {0, NULL, NULL};
    mm_builder kb, rb;
    mm_out kd, rd;
    int rc = -1;
    if (!tbl) return -1;
    for (uint32_t i = 0; i < n; ++i) { tbl[i].msb = s->msb[i]; tbl[i].lsb = s->lsb[i]; tbl[i].node = s->node[i]; }
    for (uint32_t e = 0; e < m; ++e)
        if (bound[e] != 0xFFFFFFFFu && bound[e] >= n) { free(tbl); return -2; }
    mmb_init(&kb, tbl); mmb_init(&rb, tbl);
    if (mmo_init(&kd) || mmo_init(&rd) || rb_map_build(&M, m, es, ee)) goto done;
    for (uint32_t t = 0; t < n; ++t) {
        const uint64_t em = s->exec_msb ? s->exec_msb[t] : s->msb[t];
        rb_fold_ctx c = {sep, eep, bound, min_epoch, em >> 15, es, ee, &rb, 0};   /* Timestamp.epoch: msb >>> 15 */
        const uint32_t r0 = s->rng_off ? s->rng_off[t] : 0, r1 = s->rng_off ? s->rng_off[t + 1] : 0;
        if (r1 > r0) rb_foldl_ranges(&M, s->rng_start + r0, s->rng_end + r0, (long)(r1 - r0), &c);
        else rb_foldl_keys(&M, s->key_ord + s->key_off[t], (long)(s->key_off[t + 1] - s->key_off[t]), &c);
        if (c.err) goto done;
        if (mmb_build(&kb, &kd, 0) || mmb_build(&rb, &rd, 1)) goto done;
        mmb_reset(&kb); mmb_reset(&rb);
    }
    if (alloc_out(out, &kd, &rd, n)) goto done;
    rc = 0;
done:
    free(M.starts); free(M.value);
    mmb_free(&kb); mmb_free(&rb);
    mmo_free(&kd); mmo_free(&rd);
    free(tbl);
    return rc;
}

/* test aid: the WaitingOn words, pend and until of the waiting txn at position g (-1: not waiting) */
int or_lstore_waiter_debug(const or_lstore *s, uint32_t g, uint64_t *words, uint32_t nwords, uint8_t *pend,
                           uint32_t *until, uint32_t nslots)
{
    for (uint32_t w = 0; w < s->nwt; ++w) {
        const or_waiter *x = &s->wt[w];
        if (x->g != g) continue;
        for (uint32_t a = 0; a < nwords && a < (x->nr + x->nk + 63) / 64; ++a) words[a] = x->words[a];
        for (uint32_t q = 0; q < nslots && q < x->nk; ++q) { pend[q] = x->pend[q]; until[q] = x->until[q]; }
        return (int)(x->nr << 16 | x->nk);
    }
    return -1;
}

/* ------------------------------------------------------------------------------------------
 * Stream segments (multi-GPU ownership by TxnId range)
 *
 * Under the status-at-time model a txn i computing its deps on key k starts at maxCommittedBefore
 * = the last Write j < i - W of the key (local/CommandsForKey.java:620-645): every entry before it
 * is pruned for good for every later txn (the analogue of withRedundantBefore, :1654-1684).  So
 * what a txn at position >= thr + W can still reach of a key's history is the run from the last
 * Write with position < thr on (the whole history when there is none).
 * ------------------------------------------------------------------------------------------ */
#define SEG_ENT(kind, pos) (((uint32_t)(kind) << 29) | (uint32_t)(pos))

int or_cfk_reachable(const or_stream *s, uint32_t lo, uint32_t hi, uint32_t thr, uint32_t *n_out,
                     uint32_t **key_out, uint32_t **ent_out)
{
    *n_out = 0; *key_out = NULL; *ent_out = NULL;
    if (lo > hi || hi > s->n) return -1;
    uint32_t nkeys = 0;
    for (uint32_t i = lo; i < hi; ++i)
        if (domain_of(s->lsb[i]) == 0)
            for (uint32_t p = s->key_off[i]; p < s->key_off[i + 1]; ++p)
                if (s->key_ord[p] + 1 > nkeys) nkeys = s->key_ord[p] + 1;
    uint32_t *hoff = (uint32_t *)calloc((size_t)nkeys + 1, sizeof(uint32_t));
    uint32_t *cur = (uint32_t *)malloc(((size_t)nkeys + 1) * sizeof(uint32_t));
    uint32_t P = s->key_off[hi] - s->key_off[lo];
    uint32_t *hist = (uint32_t *)malloc((size_t)(P ? P : 1) * sizeof(uint32_t));
    uint32_t *ok = NULL, *oe = NULL;
    int rc = -1;
    if (!hoff || !cur || !hist) goto done;
    /* the key's history in TxnId (= position) order: a stable counting sort of the pairs */
    for (uint32_t i = lo; i < hi; ++i)
        if (domain_of(s->lsb[i]) == 0)
            for (uint32_t p = s->key_off[i]; p < s->key_off[i + 1]; ++p) hoff[s->key_ord[p] + 1]++;
    for (uint32_t k = 0; k < nkeys; ++k) hoff[k + 1] += hoff[k];
    memcpy(cur, hoff, ((size_t)nkeys + 1) * sizeof(uint32_t));
    for (uint32_t i = lo; i < hi; ++i)
        if (domain_of(s->lsb[i]) == 0)
            for (uint32_t p = s->key_off[i]; p < s->key_off[i + 1]; ++p) hist[cur[s->key_ord[p]]++] = i;
    /* per key: from the last Write before thr on */
    size_t total = 0;
    for (uint32_t k = 0; k < nkeys; ++k) {
        uint32_t a = hoff[k], b = hoff[k + 1], st = a;
        for (uint32_t e = b; e > a; --e)
            if (hist[e - 1] < thr && kind_of(s->lsb[hist[e - 1]]) == K_WRITE) { st = e - 1; break; }
        cur[k] = st;
        total += b - st;
    }
    ok = (uint32_t *)malloc((total ? total : 1) * sizeof(uint32_t));
    oe = (uint32_t *)malloc((total ? total : 1) * sizeof(uint32_t));
    if (!ok || !oe) goto done;
    size_t w = 0;
    for (uint32_t k = 0; k < nkeys; ++k)
        for (uint32_t e = cur[k]; e < hoff[k + 1]; ++e) {
            ok[w] = k;
            oe[w] = SEG_ENT(kind_of(s->lsb[hist[e]]), hist[e]);
            ++w;
        }
    *n_out = (uint32_t)total; *key_out = ok; *ent_out = oe;
    ok = oe = NULL;
    rc = 0;
done:
    free(hoff); free(cur); free(hist); free(ok); free(oe);
    return rc;
}

/* The reachable entries at the start of segment r (thr = a_r - W) from the reachable summaries of
 * segments 0..r-1 (part q = or_cfk_reachable over [a_q, b_q) with thr b_q - W; any order inside a
 * part).  A later segment's summary keeps every entry a later txn can reach of its own txns; when it
 * holds no Write before thr on a key, the key's run continues into the segments before it -- so the
 * state is, per key, every summary entry at or after the key's last Write before thr over all parts
 * (the walk back from the newest part that stops at that Write).  Output key-major. */
typedef struct { uint32_t key, ent; } seg_ent_t;
static int cmp_seg_ent(const void *a, const void *b)
{
    const seg_ent_t *x = (const seg_ent_t *)a, *y = (const seg_ent_t *)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    const uint32_t px = x->ent & 0x1FFFFFFFu, py = y->ent & 0x1FFFFFFFu;
    return px < py ? -1 : px > py;
}

int or_cfk_fold(uint32_t nparts, const uint32_t *part_n, const uint32_t *const *keys, const uint32_t *const *ents,
                uint32_t thr, uint32_t *n_out, uint32_t **key_out, uint32_t **ent_out)
{
    *n_out = 0; *key_out = NULL; *ent_out = NULL;
    uint32_t nkeys = 0;
    size_t cap = 0;
    for (uint32_t q = 0; q < nparts; ++q) {
        cap += part_n[q];
        for (uint32_t j = 0; j < part_n[q]; ++j) if (keys[q][j] + 1 > nkeys) nkeys = keys[q][j] + 1;
    }
    uint32_t *lw = (uint32_t *)calloc((size_t)nkeys + 1, sizeof(uint32_t));   /* last Write < thr, + 1 */
    seg_ent_t *e = (seg_ent_t *)malloc((cap ? cap : 1) * sizeof(seg_ent_t));
    uint32_t *ok = (uint32_t *)malloc((cap ? cap : 1) * sizeof(uint32_t));
    uint32_t *oe = (uint32_t *)malloc((cap ? cap : 1) * sizeof(uint32_t));
    if (!lw || !e || !ok || !oe) { free(lw); free(e); free(ok); free(oe); return -1; }
    for (uint32_t q = 0; q < nparts; ++q)
        for (uint32_t j = 0; j < part_n[q]; ++j) {
            const uint32_t x = ents[q][j], pos = x & 0x1FFFFFFFu;
            if ((x >> 29) == K_WRITE && pos < thr && pos + 1 > lw[keys[q][j]]) lw[keys[q][j]] = pos + 1;
        }
    size_t m = 0;
    for (uint32_t q = 0; q < nparts; ++q)
        for (uint32_t j = 0; j < part_n[q]; ++j)
            if ((ents[q][j] & 0x1FFFFFFFu) + 1 >= lw[keys[q][j]]) { e[m].key = keys[q][j]; e[m].ent = ents[q][j]; ++m; }
    qsort(e, m, sizeof(seg_ent_t), cmp_seg_ent);
    for (size_t i = 0; i < m; ++i) { ok[i] = e[i].key; oe[i] = e[i].ent; }
    free(lw); free(e);
    *n_out = (uint32_t)m; *key_out = ok; *ent_out = oe;
    return 0;
}

void or_free(void *p) { free(p); }
