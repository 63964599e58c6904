// Execution readiness of a registered-status store (CommandsForKey.notify /
// notifyUnmanaged and Commands.updateWaitingOn on the device).
//
// accord_waiting_on_initialise puts the last computed batch's txns into the store's waiting set: a
// generation holding a copy of their deps (KeyDeps + RangeDeps txnIds, global positions), their
// WaitingOn words and appliedOrInvalidated words, and per (txn, key) the unmanaged pending record.
// accord_ready_update then, against the statuses registered so far:
//   1. summarises every key's CommandsForKey from the resident history (a wave per key): the
//      earliest executeAt among the unapplied committed (COMMITTED / STABLE) txns per kind class
//      (Read, Write, SyncPoints), `next` (the earliest of all of them, nulled when minUncommitted
//      precedes it, local/CommandsForKey.java:432-461) and minUncommitted;
//   2. re-evaluates every waiting txn (a wave per txn, a lane per WaitingOn bit):
//      - range-dep bit: Commands.updateWaitingOn (local/Commands.java:769-830) once the dep
//        hasBeen(PreCommitted): truncated / invalidated -> setAppliedOrInvalidated, executes after
//        us (not awaitsOnlyDeps) -> removeWaitingOn, applied -> setAppliedAndPropagate;
//      - key bit of a managed txn (key domain, globally visible; STABLE): notify's count test
//        (:1512-1635) expectMissingCount == |missing|, which holds iff no unapplied committed txn
//        of a kind it witnesses executes before it (the class minima) and no dep of the key in its
//        deps is still uncommitted (uncommitted non-deps are exactly its missing[] set,
//        computeInfoAndAdditions :1071-1140, committed ones elided :1103-1109);
//      - key bit of an unmanaged txn (range domain, EphemeralRead; hasBeen Stable):
//        registerUnmanaged (:1406-1498) on the first evaluation, a COMMIT record whose waitingUntil
//        precedes minUncommitted re-evaluated as updatePending (:1315-1360), an APPLY record
//        released by notifyUnmanaged(APPLY, next.executeAt) (:1264-1283);
//      - no bit left and STABLE: ReadyToExecute (Commands.maybeExecute, :656-733), reported once.
// The reference evaluates these tests when an event reaches the key (notifyAndUpdatePending,
// :1163-1215); here a txn is re-evaluated at every call at which something its tests read changed,
// so it is released at the first call at which its test holds.  What changed since the last call is
// found from a per-position change epoch (rg_chg, stamped by accord_txn_register and the batch join):
// a key is dirty when a carried entry of it changed (every input of its tests -- the key's summary,
// its deps' statuses and executeAts -- is a carried entry of the key, or a txn the carry dropped for
// good: INVALID / ERASED, whose later events change nothing the tests read, or below the key's
// RedundantBefore bound, which the tests skip); a txn is re-evaluated when it changed itself, a key
// of a set bit is dirty or a range dep of a set bit changed.  A new batch or a truncation (a new carry)
// and a txn's first evaluation evaluate everything.  oracle/oracle.c (or_lstore_ready) restates the same evaluation over
// literal CommandsForKey objects.
// Event-exact mode (accord_ready_set_mode ACCORD_READY_EVENTS): key bits clear only when
// notifyAndUpdatePending's events reach the key, replayed in order by one wave per registration
// (rd_event_kernel below); the calls then evaluate range-dep bits and release.  Equal to the
// event-driven restatement (or_lstore_event_mode) call by call.
#include "store_impl.h"
#include "status_view.h"
#include "redundant_wait.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace accord_status;

#define EV_RC(expr) do { const int32_t rc_ = (expr); if (rc_ != ACCORD_OK) return rc_; } while (0)

namespace {

constexpr uint32_t NONE = 0xFFFFFFFFu;

struct KeySummary {
    uint32_t min_cls[3];              // unapplied committed txn with the earliest executeAt: Read, Write, SyncPoints
    uint32_t next;                    // earliest of them (any kind)
    uint32_t min_unc;                 // first uncommitted txn (TxnId order)
    uint32_t pad[3];
};

__device__ __forceinline__ uint32_t kind_class(uint32_t kind) { return kind == 0u ? 0u : kind == 1u ? 1u : 2u; }

// segment bounds of the carried history (key-major): kseg0[k] .. kseg1[k] (zeroed first); computed
// once per version of the carry (it changes only when a batch is computed or truncated)
__global__ __launch_bounds__(256) void rd_seg_kernel(uint32_t C, const uint32_t *__restrict__ ckey,
                                                     uint32_t *__restrict__ kseg0, uint32_t *__restrict__ kseg1)
{
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
        const uint32_t k = ckey[c];
        if (c == 0 || ckey[c - 1] != k) kseg0[k] = c;
        if (c + 1 == C || ckey[c + 1] != k) kseg1[k] = c + 1;
    }
}

// A candidate txn with its executeAt in registers (g = NONE: none)
struct Cand {
    uint32_t g;
    Ts ex;
};

__device__ __forceinline__ Cand cand_shfl_down(const Cand &c, uint32_t d)
{
    return Cand{(uint32_t)__shfl_down((int)c.g, d, 64),
                Ts{(uint64_t)__shfl_down((long long)c.ex.msb, d, 64), (uint64_t)__shfl_down((long long)c.ex.lsb, d, 64),
                   __shfl_down(c.ex.node, d, 64)}};
}

__device__ __forceinline__ void cand_min(Cand &a, const Cand &b)
{
    if (b.g != NONE && (a.g == NONE || tcmp(b.ex, a.ex) < 0)) a = b;
}

// Per-key summaries in two passes, so a hot key's long history spreads over many waves:
// rd_part_kernel -- a wave per 64 consecutive carried entries (key-major): every key run inside the
//   64 reduced by segmented shuffles (earliest executeAt per kind class among the unapplied
//   committed, first uncommitted), the result stored at the run's first entry (part[]);
// rd_summary_kernel -- a wave per key: its runs' partials (its first entry and every 64-entry
//   boundary inside its history) reduced into the key's summary.
// Managed txns only: EphemeralReads are not inserted into CommandsForKey.
struct KeyPart {
    uint32_t cls[3];
    uint32_t unc;
};

// Incremental calls (dirty != nullptr): a carried entry whose txn changed since epoch `seen` marks
// its key with this call's id and appends it to list[] once (its summary is recomputed); one that
// became committed (or invalid) marks it in eval[] (the "dep uncommitted" tests of its waiters may
// change); only the 64-entry chunks holding a changed entry recompute their partials (part[] keeps
// the others' from earlier calls of the same carry).
struct DirtyMark {
    const uint32_t *chg, *cchg;
    uint32_t seen, call;
    uint32_t *dirty, *list, *cnt, *eval;
};

__global__ __launch_bounds__(256) void rd_part_kernel(uint32_t C, const uint32_t *__restrict__ ckey,
                                                      const uint32_t *__restrict__ cent, StatusView v,
                                                      KeyPart *__restrict__ part, DirtyMark dm)
{
    const uint32_t lane = lane_id(), waves = gridDim.x * (blockDim.x / 64);
    for (uint32_t c0 = (blockIdx.x * (blockDim.x / 64) + wave_id()) * 64u; c0 < C; c0 += waves * 64u) {
        const uint32_t x = c0 + lane;
        uint32_t key = NONE;
        Cand cc[3] = {{NONE, {0, 0, 0}}, {NONE, {0, 0, 0}}, {NONE, {0, 0, 0}}};
        uint32_t mu = NONE;
        const uint32_t e = x < C ? cent[x] : 0u, g = e & ENT_TXN_MASK, kind = e >> ENT_KIND_SHIFT;
        if (x < C) key = ckey[x];
        if (dm.dirty) {
            // incremental call: a chunk none of whose entries changed keeps its partials
            const bool ch = x < C && dm.chg[g] > dm.seen;
            if (__ballot(ch) == 0ull) continue;                  // wave-uniform
            if (ch && dm.dirty[key] != dm.call && atomicExch(&dm.dirty[key], dm.call) != dm.call)
                dm.list[atomicAdd(dm.cnt, 1u)] = key;
            if (ch && dm.cchg[g] > dm.seen) dm.eval[key] = dm.call;
        }
        if (x < C) {
            const uint32_t st = kind == 2u ? ST_INVALID : status_of(v, g);
            if (st < ST_COMMITTED) mu = g;
            else if (st < ST_APPLIED) {
                const Cand me{g, exec_of(v, g)};
                const uint32_t kc = kind_class(kind);
#pragma unroll
                for (uint32_t c = 0; c < 3; ++c)      // static indices: the array stays in registers
                    if (c == kc) cc[c] = me;
            }
        }
        // segmented suffix reduction over the run of equal keys (keys ascend inside the chunk)
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t ok = (uint32_t)__shfl_down((int)key, d, 64);
            const bool take = lane + d < 64 && ok == key;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const Cand o = cand_shfl_down(cc[c], d);
                if (take) cand_min(cc[c], o);
            }
            const uint32_t om = (uint32_t)__shfl_down((int)mu, d, 64);
            if (take) mu = min(mu, om);
        }
        const uint32_t pk = (uint32_t)__shfl_up((int)key, 1, 64);
        if (x < C && (lane == 0 || pk != key)) part[x] = KeyPart{{cc[0].g, cc[1].g, cc[2].g}, mu};
    }
}

// every key (list == nullptr), or the dirty keys list[0 .. *cnt): a key whose summary changed is
// marked in eval[] with this call's id (its waiters' tests read the summary)
__global__ __launch_bounds__(256) void rd_summary_kernel(uint32_t nkeys, const uint32_t *__restrict__ kseg0,
                                                         const uint32_t *__restrict__ kseg1,
                                                         const KeyPart *__restrict__ part, StatusView v,
                                                         KeySummary *__restrict__ sum, const uint32_t *__restrict__ list,
                                                         const uint32_t *__restrict__ cnt, uint32_t *__restrict__ eval,
                                                         uint32_t call)
{
    const uint32_t lane = lane_id(), waves = gridDim.x * (blockDim.x / 64);
    const uint32_t m = list ? *cnt : nkeys;
    for (uint32_t i = blockIdx.x * (blockDim.x / 64) + wave_id(); i < m; i += waves) {
        const uint32_t k = list ? list[i] : i;
        const uint32_t a = kseg0[k], b = kseg1[k];
        Cand cc[3] = {{NONE, {0, 0, 0}}, {NONE, {0, 0, 0}}, {NONE, {0, 0, 0}}};
        uint32_t mu = NONE;
        // the runs: one starting at a, then one at every multiple of 64 inside (a, b)
        const uint32_t nr = a < b ? 1u + ((b - 1) >> 6) - (a >> 6) : 0u;
        constexpr int SB = 4;                        // runs per lane per step: their loads in flight together
        for (uint32_t j0 = lane; j0 < nr; j0 += 64u * SB) {
            KeyPart q[SB];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const uint32_t j = j0 + 64u * u;
                const uint32_t x = j == 0 ? a : ((a >> 6) + j) << 6;
                q[u] = j < nr ? part[x] : KeyPart{{NONE, NONE, NONE}, NONE};
            }
            Cand cq[SB][3];
#pragma unroll
            for (int u = 0; u < SB; ++u)
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    cq[u][c] = q[u].cls[c] != NONE ? Cand{q[u].cls[c], exec_of(v, q[u].cls[c])} : Cand{NONE, {0, 0, 0}};
#pragma unroll
            for (int u = 0; u < SB; ++u) {
#pragma unroll
                for (int c = 0; c < 3; ++c) cand_min(cc[c], cq[u][c]);
                mu = min(mu, q[u].unc);
            }
        }
#pragma unroll
        for (uint32_t d = 32; d >= 1; d >>= 1) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const Cand o{(uint32_t)__shfl_xor((int)cc[c].g, d, 64),
                             Ts{(uint64_t)__shfl_xor((long long)cc[c].ex.msb, d, 64),
                                (uint64_t)__shfl_xor((long long)cc[c].ex.lsb, d, 64), __shfl_xor(cc[c].ex.node, d, 64)}};
                cand_min(cc[c], o);
            }
            mu = min(mu, (uint32_t)__shfl_xor((int)mu, d, 64));
        }
        if (lane == 0) {
            KeySummary s{};
            Cand nx = cc[0];
            cand_min(nx, cc[1]);
            cand_min(nx, cc[2]);
            for (int c = 0; c < 3; ++c) s.min_cls[c] = cc[c].g;
            s.next = nx.g;                           // nulled by the evaluation (TxnId order)
            s.min_unc = mu;
            if (list) {
                const KeySummary o = sum[k];
                if (o.min_cls[0] != s.min_cls[0] || o.min_cls[1] != s.min_cls[1] || o.min_cls[2] != s.min_cls[2] ||
                    o.next != s.next || o.min_unc != s.min_unc)
                    eval[k] = call;
            }
            sum[k] = s;
        }
    }
}

struct ReadyOut {
    uint32_t g;
    int32_t node;                     // Command.executesAtLeast
    uint64_t msb, lsb;
};

struct ReadyParams {
    uint32_t n, key_lo;
    const uint32_t *g;                // [n] global positions
    const uint64_t *lsb;              // [n] TxnId lsb (kind, domain)
    const uint64_t *tmsb, *tlsb;      // the store's TxnIds, ascending, and their global positions (ascending)
    const int32_t *tnode;
    const uint32_t *tg;
    uint32_t tx_n;
    const uint32_t *rd_off, *rd_vals;
    const uint32_t *key_off, *keys, *val_off, *vals, *k2v_off;
    const int32_t *k2v;
    const uint32_t *wo_off;
    unsigned long long *words, *aoi;
    uint8_t *pend;                    // per key slot: 0 unregistered, 1 COMMIT, 2 APPLY, 3 released
    uint32_t *until;                  // unmanaged: the pending record's txn; managed: the committed-deps cursor
    uint8_t *done;
    ReadyOut *out;                    // txns that became ready: position + executesAtLeast
    uint32_t *out_cnt;
    uint32_t *drop, *drop_cnt;        // waiting txns invalidated / truncated: leave the set unreported
    EalRec *eal;                      // [n] WaitingOn.executeAtLeast
    // removeRedundantDependencies (redundant_wait.h; rbx = the map can remove a dep): the txns'
    // participants (keys / ranges) and RangeDeps ranges + rangesToTxnIds
    uint32_t rbx;
    RrMap M;
    const uint32_t *pkoff, *pkeys, *proff, *prs, *pre;
    const uint32_t *rrng_off, *rrs, *rre, *rr2v_off, *rr2v;
    RrSpill spill;                    // txns over the LDS removal scratch (ids: ubase + launch index)
    uint32_t ubase;                   // index of this table's launch's first txn over all launches
    const KeySummary *sum;
    const uint32_t *kb;               // per key: shardRedundantBefore as a position (0: none)
    StatusView v;
    uint32_t full;                    // the generation is new: evaluate every txn of it
    const uint32_t *chg, *dirty;      // by position: change epoch; by key: id of the call it was dirty in
    // setAppliedAndPropagate (local/Command.java:1569-1583): released Range-domain txns' final
    // appliedOrInvalidated (positions), per position pv_at = 1 + pool start (0: none), pv_len
    uint32_t *pv_at, *pv_len, *pv_pool, *pv_cnt;
    uint32_t evmode;                  // event-exact mode: key bits clear on events only (rd_event_kernel)
    uint32_t *inv;                    // 1 + the position of a waiter whose TruncatedApply dep breaks
                                      // updateWaitingOn's checkState (local/Commands.java:789-791); 0 = none
};

// the TxnId of global position g (the store's TxnId table is in stream order)
__device__ __forceinline__ Ts tid_of(const ReadyParams &p, uint32_t g)
{
    uint32_t lo = 0, hi = p.tx_n;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (p.tg[m] < g) lo = m + 1; else hi = m;
    }
    return Ts{p.tmsb[lo], p.tlsb[lo], p.tnode[lo]};
}

// registerUnmanaged (reg) / updatePending over the deps [d0, d1) of one key: 1 = ready, 0 = APPLY
// pending (*until = the relevant dep executing last), -1 = COMMIT pending (*until = the last dep)
__device__ int unmanaged_eval(const ReadyParams &p, uint32_t t, uint32_t d0, uint32_t d1, uint32_t kbound,
                              const Ts &ex, bool only_deps, bool reg, uint32_t &until, uint32_t &executes_at)
{
    executes_at = NONE;
    const uint32_t vb = p.val_off[t], kb0 = p.k2v_off[t];
    uint32_t x = d0;
    while (x < d1 && p.vals[vb + p.k2v[kb0 + x]] < kbound) ++x;    // txnIds.find(shardRedundantBefore)
    if (x >= d1) return 1;
    bool ready = true, to_apply = true;
    uint32_t best = NONE;
    for (; x < d1; ++x) {
        const uint32_t u = p.vals[vb + p.k2v[kb0 + x]], st = status_of(p.v, u);
        if (reg && st < ST_COMMITTED) { ready = to_apply = false; continue; }
        const Ts ue = exec_of(p.v, u);
        if (only_deps || tcmp(ue, ex) < 0) {
            ready &= st >= ST_APPLIED;
            if (best == NONE || tcmp(exec_of(p.v, best), ue) < 0) best = u;
        }
    }
    if (ready) return 1;
    executes_at = best;                                              // the relevant dep executing last
    const uint32_t last = p.vals[vb + p.k2v[kb0 + d1 - 1]];
    if (to_apply) { until = best == NONE ? last : best; return 0; }
    until = last;
    return -1;
}

// a wave per waiting txn, a lane per WaitingOn bit (64 per word); every generation in one launch
// (the waves walk the concatenated txn index space, gbase[] = each generation's first index)
constexpr uint32_t RD_GENS = 32;          // generations evaluated per launch
struct ReadyLaunch {
    uint32_t ngen, total, base;       // base: the launch's first txn over all launches of the call
    uint32_t gbase[RD_GENS + 1];
    uint32_t *work, *wcnt;            // incremental calls: the txns to evaluate (rd_filter_kernel)
    ReadyParams g[RD_GENS];
};

__device__ __forceinline__ void rd_eval_txn(const ReadyParams &p, uint32_t u, uint32_t t, uint32_t lane, const RrBuf &rl,
                                            bool spill);

// Incremental calls: RF_LANES lanes per waiting txn keep those whose inputs changed since the last
// call (the txn itself, the key of a set key bit dirty -- for a managed txn: and no longer blocked by
// the key's class minima --, the txn of a set range-dep bit changed) or that were never evaluated;
// wave-aggregated appends to work[].  The lanes of a txn take its set WaitingOn bits round-robin, so
// a txn's bit tests (each a chain of dependent loads: key, dirty mark, summary, executeAt) run side
// by side (a lane per txn walking its bits in turn took 14.8 us per call, profiles/r05_ready).
// (seen: the change epoch of the last call, call: this call's id, full: evaluate everything)
constexpr uint32_t RF_LANES = 8;
__global__ __launch_bounds__(256) void rd_filter_kernel(const ReadyLaunch *__restrict__ L, uint32_t seen, uint32_t call,
                                                        uint32_t full)
{
    const uint32_t gt = blockIdx.x * blockDim.x + threadIdx.x, lane = lane_id();
    const uint32_t u = gt / RF_LANES, sub = gt % RF_LANES;
    const uint32_t ngen = L->ngen, total = L->total;
    bool need = false;
    if (u < total) {
        uint32_t gi = 0;
        while (gi + 1 < ngen && L->gbase[gi + 1] <= u) ++gi;
        const ReadyParams &p = L->g[gi];
        const uint32_t t = u - L->gbase[gi];
        if (!p.done[t]) {
            const uint32_t g = p.g[t];
            need = full || p.full || p.chg[g] > seen;
            const uint32_t R = p.rd_off[t + 1] - p.rd_off[t], RK = R + p.key_off[t + 1] - p.key_off[t];
            const uint32_t w0 = p.wo_off[t], nw = p.wo_off[t + 1] - w0;
            const uint64_t l = p.lsb[t];
            const uint32_t kind = (uint32_t)(l >> 1) & 7u;
            const bool managed = (l & 1u) == 0 && kind != 2u;
            // a managed txn's key bit clears only when STABLE and no witnessed class minimum of the key
            // executes before it: a dirty key whose minima still block it needs no evaluation
            const bool stable = managed && !need && status_of(p.v, g) == ST_STABLE;
            const uint32_t wmask = witness_mask(kind);
            Ts ex{0, 0, 0};
            if (stable) ex = exec_of(p.v, g);
            uint32_t rank0 = 0;                       // set bits before word q
            for (uint32_t q = 0; q < nw && !need; ++q) {
                const unsigned long long wq = p.words[w0 + q];
                const uint32_t c = (uint32_t)__popcll(wq);
                // this lane's bits of the word: ranks r = sub (mod RF_LANES) among the txn's set bits
                uint32_t r = rank0 + ((sub + RF_LANES - rank0 % RF_LANES) % RF_LANES);
                unsigned long long w = wq;
                for (uint32_t k = rank0; k < r && w; ++k) w &= w - 1ull;   // drop the bits before rank r
                for (; r < rank0 + c && !need; r += RF_LANES) {
                    const uint32_t b = q * 64u + (uint32_t)__ffsll((long long)w) - 1u;
                    for (uint32_t k = 0; k < RF_LANES && w; ++k) w &= w - 1ull;   // next: rank r + RF_LANES
                    if (b >= RK) break;
                    if (b < R) { need = p.chg[p.rd_vals[p.rd_off[t] + b]] > seen; continue; }
                    const uint32_t kk = p.keys[p.key_off[t] + b - R] - p.key_lo;
                    if (p.dirty[kk] != call) continue;
                    if (!managed) { need = true; continue; }
                    if (!stable) continue;                       // not STABLE: its key bits cannot clear
                    const KeySummary sm = p.sum[kk];
                    bool blocked = false;
                    if (((wmask >> 0) & 1u) && sm.min_cls[0] != NONE && tcmp(exec_of(p.v, sm.min_cls[0]), ex) < 0) blocked = true;
                    if (!blocked && ((wmask >> 1) & 1u) && sm.min_cls[1] != NONE && tcmp(exec_of(p.v, sm.min_cls[1]), ex) < 0) blocked = true;
                    if (!blocked && ((wmask >> 3) & 1u) && sm.min_cls[2] != NONE && tcmp(exec_of(p.v, sm.min_cls[2]), ex) < 0) blocked = true;
                    need = !blocked;
                }
                rank0 += c;
            }
        }
    }
    // a txn is kept when any of its lanes needs it; its first lane appends it
    const unsigned long long nb = __ballot(need);
    const uint32_t gbase = lane & ~(RF_LANES - 1u);
    const bool keep = sub == 0 && ((nb >> gbase) & ((1ull << RF_LANES) - 1ull)) != 0ull;
    const unsigned long long m = __ballot(keep);
    if (m) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(L->wcnt, (uint32_t)__popcll(m));
        base = (uint32_t)__shfl((int)base, 0, 64);
        if (keep) L->work[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = u;
    }
}

// The call's result read-back without a copy engine: one block after the evaluation copies the
// header and the first ready records into the page-locked host buffer the host reads once the stream
// has synchronised (a device-to-host copy after the kernels cost ~15 us of a ~60 us call: the hand-off
// to the copy queue and the copy; the kernel boundary orders the evaluation's writes before it).
// It also zeroes the header for the next call (one memset fewer) unless the removal spill pass
// still has to run on it.
__global__ __launch_bounds__(256) void rd_host_out_kernel(uint32_t *__restrict__ cnt, uint32_t *__restrict__ host,
                                                          uint32_t hdr, uint32_t rw, uint32_t peek)
{
    const uint32_t words = hdr + min(cnt[0], peek) * rw;
    const bool spill = cnt[hdr - 2] != 0;
    for (uint32_t x = threadIdx.x; x < words; x += blockDim.x) host[x] = cnt[x];
    __syncthreads();
    if (!spill)
        for (uint32_t x = threadIdx.x; x < hdr; x += blockDim.x) cnt[x] = 0u;
}

// a wave per txn: every txn of the launch (work == nullptr) or the listed ones
__global__ __launch_bounds__(256) void rd_eval_kernel(const ReadyLaunch *__restrict__ L, uint32_t listed)
{
    extern __shared__ RrLds rr_lds[];                // removal scratch, a wave each (when the map can remove)
    const uint32_t lane = lane_id(), waves = gridDim.x * (blockDim.x / 64);
    const uint32_t ngen = L->ngen, m = listed ? *L->wcnt : L->total;
    const RrBuf rl = rr_buf_lds(rr_lds[wave_id()]);
    for (uint32_t i = blockIdx.x * (blockDim.x / 64) + wave_id(); i < m; i += waves) {
        const uint32_t u = listed ? L->work[i] : i;
        uint32_t gi = 0;
        while (gi + 1 < ngen && L->gbase[gi + 1] <= u) ++gi;
        rd_eval_txn(L->g[gi], u, u - L->gbase[gi], lane, rl, false);
    }
}

// The spill pass: the txns rd_eval_kernel left for exceeding its LDS removal scratch, a wave each with
// HBM scratch sized for the largest of them (launch index and txn index packed in the list)
__global__ __launch_bounds__(256) void rd_spill_kernel(const ReadyLaunch *__restrict__ L0, uint32_t nl, RrSpill sp,
                                                       void *base, uint32_t cap_r, uint32_t cap_e)
{
    const uint32_t lane = lane_id(), waves = gridDim.x * (blockDim.x / 64);
    const uint32_t gw = blockIdx.x * (blockDim.x / 64) + wave_id();
    const RrBuf rl = rr_buf_hbm(base, gw, cap_r, cap_e);
    const uint32_t m = *sp.count;
    for (uint32_t i = gw; i < m; i += waves) {
        const uint32_t id = sp.list[i];
        uint32_t k = 0;
        while (k + 1 < nl && L0[k + 1].base <= id) ++k;
        const ReadyLaunch *L = L0 + k;
        const uint32_t u = id - L->base;
        uint32_t gi = 0;
        while (gi + 1 < L->ngen && L->gbase[gi + 1] <= u) ++gi;
        rd_eval_txn(L->g[gi], u, u - L->gbase[gi], lane, rl, true);
    }
}

__device__ __forceinline__ void rd_eval_txn(const ReadyParams &p, uint32_t u, uint32_t t, uint32_t lane, const RrBuf &rl,
                                            bool spill)
{
    {
        if (p.done[t]) return;
        const uint32_t g = p.g[t], st = status_of(p.v, g);
        if (st >= ST_INVALID) {                  // never executes (maybeExecute needs Stable): leaves the set
            if (lane == 0) {
                p.done[t] = 1;
                p.drop[atomicAdd(p.drop_cnt, 1u)] = g;
            }
            return;
        }
        const uint64_t l = p.lsb[t];
        const uint32_t kind = (uint32_t)(l >> 1) & 7u;
        const bool rdom = (l & 1u) != 0;
        const bool only_deps = kind == 4u || kind == 2u;                 // Txn.Kind.awaitsOnlyDeps
        const bool managed = !rdom && kind != 2u;                        // key domain, globally visible
        const Ts ex = exec_of(p.v, g);
        const uint32_t wmask = witness_mask(kind);
        const uint32_t R = p.rd_off[t + 1] - p.rd_off[t], K = p.key_off[t + 1] - p.key_off[t];
        const uint32_t w0 = p.wo_off[t], nw = p.wo_off[t + 1] - w0;
        // removeRedundantDependencies (redundant_wait.h) when minWaitingOnTxnId is a range dep
        bool removal = false;
        RrTxn T{};
        if (p.rbx && R) {
            uint32_t j0 = NONE;
            for (uint32_t q = 0; q < nw && j0 == NONE; ++q) {
                const unsigned long long wq = p.words[w0 + q];
                if (wq) j0 = q * 64u + (uint32_t)__builtin_ctzll(wq);
            }
            if (j0 < R) {
                T.rdom = rdom;
                if (rdom) { T.np = p.proff[t + 1] - p.proff[t]; T.ps = p.prs + p.proff[t]; T.pe = p.pre + p.proff[t]; }
                else { T.np = p.pkoff[t + 1] - p.pkoff[t]; T.pk = p.pkeys + p.pkoff[t]; }
                T.R = R; T.rvals = p.rd_vals + p.rd_off[t];
                T.nrr = p.rrng_off[t + 1] - p.rrng_off[t];
                T.rs = p.rrs + p.rrng_off[t]; T.re = p.rre + p.rrng_off[t];
                T.r2v = p.rr2v + p.rr2v_off[t];
                const uint32_t mpos = T.rvals[j0];
                bool o = false;
                uint32_t ne = 0;
                removal = rr_removal(p.M, T, rl, lane, mpos, tid_of(p, mpos).msb >> 15, ex.msb >> 15, &o, &ne);
                if (o) {                 // over the scratch: nothing decided, the spill pass evaluates it
                    if (lane == 0 && !spill) rr_spill_add(p.spill, p.ubase + u, R, ne);
                    return;
                }
            }
        }
        Ts own{0, 0, 0};                                                // own TxnId (executeAtLeast)
        if (only_deps) own = tid_of(p, g);
        bool eh = false;                                                // this lane's executeAtLeast candidate
        Ts ev{0, 0, 0};
        auto cand = [&](const Ts &x) {
            if (!eh || tcmp(ev, x) < 0) { ev = x; eh = true; }
        };
        // setAppliedAndPropagate: an applied range dep whose own WaitingOn recorded applied /
        // invalidated txnIds clears those bits too, and updateWaitingOn's reverse walk
        // (forEachWaitingOnId) then skips them -- an order the lane-parallel evaluation does not keep.
        // A txn with such a dep walks its range-dep bits in that order on one lane (rare: the dep
        // must be a released Range-domain txn with a set appliedOrInvalidated bit).
        const uint32_t *rv = p.rd_vals + p.rd_off[t];
        bool seqr = false;
        if (R && p.pv_at) {
            for (uint32_t q = 0; q < nw && q * 64u < R && !seqr; ++q) {
                const unsigned long long rclr = removal ? rr_clear(rl, T, q) : 0ull;
                const unsigned long long old = p.words[w0 + q] & ~rclr;
                const uint32_t b = q * 64u + lane;
                bool pr = false;
                if (b < R && ((old >> lane) & 1ull)) {
                    const uint32_t d = rv[b];
                    pr = status_of(p.v, d) == ST_APPLIED && p.pv_at[d] != 0u &&
                         (only_deps || tcmp(exec_of(p.v, d), ex) <= 0);
                }
                seqr = __ballot(pr) != 0ull;
            }
        }
        if (seqr) {
            for (uint32_t q = 0; q < nw && q * 64u < R; ++q) {             // the removal first, as below
                const unsigned long long rclr = removal ? rr_clear(rl, T, q) : 0ull;
                if (rclr && lane == 0) p.words[w0 + q] &= ~rclr;
            }
            if (lane == 0) {
                for (uint32_t j = R; j-- > 0;) {
                    const uint32_t q = j >> 6;
                    const unsigned long long bit = 1ull << (j & 63u), wq = p.words[w0 + q];
                    if (!(wq & bit)) continue;
                    const uint32_t d = rv[j], ds = status_of(p.v, d);
                    if (only_deps && exec_known(ds)) {                           // updateExecuteAtLeast
                        const Ts de = exec_of(p.v, d);
                        if (tcmp(de, own) > 0) cand(de);
                    }
                    if (ds == ST_TRUNC_APPLY && !only_deps && tcmp(exec_of(p.v, d), ex) >= 0) *p.inv = g + 1u;
                    if (ds < ST_COMMITTED) continue;                           // !hasBeen(PreCommitted)
                    bool clr = false, app = false;
                    if (ds >= ST_INVALID) clr = app = true;
                    else if (!only_deps && tcmp(exec_of(p.v, d), ex) > 0) clr = true;
                    else if (ds == ST_APPLIED) clr = app = true;
                    if (!clr) continue;
                    p.words[w0 + q] = wq & ~bit;
                    if (app && rdom) p.aoi[w0 + q] |= bit;
                    if (!(ds == ST_APPLIED && app) || p.pv_at[d] == 0u) continue;
                    // forEachIntersection(propagate.txnIds, txnIds): setAppliedOrInvalidated on ours
                    const uint32_t *L = p.pv_pool + (p.pv_at[d] - 1u);
                    for (uint32_t a = 0, nL = p.pv_len[d]; a < nL; ++a) {
                        uint32_t lo = 0, hi = R;
                        while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (rv[m] < L[a]) lo = m + 1; else hi = m; }
                        if (lo >= R || rv[lo] != L[a]) continue;
                        const uint32_t q2 = lo >> 6;
                        const unsigned long long b2 = 1ull << (lo & 63u), w2 = p.words[w0 + q2];
                        if (!(w2 & b2) || (rdom && (p.aoi[w0 + q2] & b2))) continue;   // :1551-1567
                        p.words[w0 + q2] = w2 & ~b2;
                        if (rdom) p.aoi[w0 + q2] |= b2;
                    }
                }
            }
            __threadfence();              // lane 0's words / aoi before the lanes read them below
        }
        bool waiting = false;
        for (uint32_t q = 0; q < nw; ++q) {
            const unsigned long long rclr = removal ? rr_clear(rl, T, q) : 0ull;
            const unsigned long long old = p.words[w0 + q] & ~rclr;
            const uint32_t b = q * 64u + lane;
            bool clear = false, applied = false;
            // seqr: range bits walked above; event mode: key bits clear on events only
            if (b < R + K && ((old >> lane) & 1ull) && !(seqr && b < R) && !(p.evmode && b >= R)) {
                if (b < R) {                                             // range-dep bit
                    const uint32_t d = p.rd_vals[p.rd_off[t] + b], ds = status_of(p.v, d);
                    if (only_deps && exec_known(ds)) {                           // updateExecuteAtLeast
                        const Ts de = exec_of(p.v, d);
                        if (tcmp(de, own) > 0) cand(de);
                    }
                    // Invariants.checkState(executeAt < waitingExecuteAt || awaitsOnlyDeps) (:789-791)
                    if (ds == ST_TRUNC_APPLY && !only_deps && tcmp(exec_of(p.v, d), ex) >= 0) *p.inv = g + 1u;
                    if (ds >= ST_COMMITTED) {                            // hasBeen(PreCommitted)
                        if (ds >= ST_INVALID) clear = applied = true;
                        else if (!only_deps && tcmp(exec_of(p.v, d), ex) > 0) clear = true;
                        else if (ds == ST_APPLIED) clear = applied = true;
                    }
                } else {                                                 // key bit
                    const uint32_t qs = b - R, slot = p.key_off[t] + qs;
                    const uint32_t kk = p.keys[slot] - p.key_lo;
                    const KeySummary s = p.sum[kk];
                    const uint32_t kbound = p.kb ? p.kb[kk] : 0u;
                    const uint32_t hb = p.k2v_off[t];
                    const uint32_t d0 = qs == 0 ? K : (uint32_t)p.k2v[hb + qs - 1], d1 = (uint32_t)p.k2v[hb + qs];
                    if (managed) {
                        if (st == ST_STABLE) {
                            bool blocked = false;                        // an unapplied committed predecessor
                            if (((wmask >> 0) & 1u) && s.min_cls[0] != NONE && tcmp(exec_of(p.v, s.min_cls[0]), ex) < 0) blocked = true;
                            if (((wmask >> 1) & 1u) && s.min_cls[1] != NONE && tcmp(exec_of(p.v, s.min_cls[1]), ex) < 0) blocked = true;
                            if (((wmask >> 3) & 1u) && s.min_cls[2] != NONE && tcmp(exec_of(p.v, s.min_cls[2]), ex) < 0) blocked = true;
                            // a dep still uncommitted: committed (and below the bound) never reverts, so
                            // the scan resumes where the last one stopped (until[] = its cursor here)
                            // every uncommitted txn of the key is at or after min_unc (positions
                            // ascend with TxnIds): none of the deps when the last one precedes it
                            if (!blocked && d1 > d0 && s.min_unc != NONE &&
                                s.min_unc <= p.vals[p.val_off[t] + p.k2v[hb + d1 - 1]]) {
                                uint32_t x = max(d0, p.until[slot]);
                                for (; x < d1; ++x) {
                                    const uint32_t u = p.vals[p.val_off[t] + p.k2v[hb + x]];
                                    if (u >= kbound && status_of(p.v, u) < ST_COMMITTED) { blocked = true; break; }
                                }
                                p.until[slot] = x;
                            }
                            clear = !blocked;
                        }
                    } else if (st >= ST_STABLE && st < ST_INVALID) {     // hasBeen(Stable), not truncated
                        uint32_t pd = p.pend[slot], un = p.until[slot], ea = NONE;
                        if (pd == 0) {                                   // registerUnmanaged
                            const int r = unmanaged_eval(p, t, d0, d1, kbound, ex, only_deps, true, un, ea);
                            pd = r == 1 ? 3u : r == 0 ? 2u : 1u;
                            if (r == 0 && only_deps && ea != NONE) cand(exec_of(p.v, ea));   // :1470-1478
                        }
                        uint32_t nx = s.next;
                        if (nx != NONE && s.min_unc != NONE && tcmp(tid_of(p, s.min_unc), exec_of(p.v, nx)) < 0)
                            nx = NONE;                                   // nulled by minUncommitted (:454-455)
                        if (pd == 1 && (s.min_unc == NONE || s.min_unc > un)) {   // COMMIT -> updatePending
                            const int r = unmanaged_eval(p, t, d0, d1, kbound, ex, only_deps, false, un, ea);
                            pd = r == 1 ? 3u : 2u;
                            if (r == 0 && only_deps && ea != NONE) cand(exec_of(p.v, ea));   // :1370-1380
                        }
                        if (pd == 2 && (s.min_unc == NONE || nx != NONE)) {       // notifyUnmanaged(APPLY, next)
                            if (nx == NONE || tcmp(exec_of(p.v, un), exec_of(p.v, nx)) < 0) pd = 3;
                        }
                        p.pend[slot] = (uint8_t)pd;
                        p.until[slot] = un;
                        clear = pd == 3;
                    }
                }
            }
            const unsigned long long cm = __ballot(clear);
            const unsigned long long am = __ballot(applied && rdom);   // appliedOrInvalidated: Range-domain txns
            const unsigned long long nwv = old & ~cm;
            if (lane == 0) {
                if (cm || rclr) p.words[w0 + q] = nwv;
                if (am) p.aoi[w0 + q] |= am;
            }
            waiting |= nwv != 0ull;
        }
        EalRec ea{0, 0, 0, 0u};
        if (only_deps) {
            ea = p.eal[t];
            eal_merge(ea, eal_wave_max(eh, ev));
            if (lane == 0 && ea.has) p.eal[t] = ea;
        }
        if (!waiting && st == ST_STABLE && rdom && R && p.pv_pool) {
            // released: its appliedOrInvalidated stays for setAppliedAndPropagate (positions, ascending)
            __threadfence();
            uint32_t cntv = 0;
            for (uint32_t q = 0; q < nw && q * 64u < R; ++q) {
                const unsigned long long m = R - q * 64u >= 64u ? ~0ull : ((1ull << (R - q * 64u)) - 1ull);
                cntv += (uint32_t)__popcll(p.aoi[w0 + q] & m);
            }
            if (cntv) {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(p.pv_cnt, cntv);
                base = (uint32_t)__shfl((int)base, 0, 64);
                uint32_t o = base;
                for (uint32_t q = 0; q < nw && q * 64u < R; ++q) {
                    const unsigned long long m = R - q * 64u >= 64u ? ~0ull : ((1ull << (R - q * 64u)) - 1ull);
                    const unsigned long long a = p.aoi[w0 + q] & m;
                    if ((a >> lane) & 1ull) p.pv_pool[o + (uint32_t)__popcll(a & ((1ull << lane) - 1ull))] = rv[q * 64u + lane];
                    o += (uint32_t)__popcll(a);
                }
                if (lane == 0) { p.pv_len[g] = cntv; p.pv_at[g] = base + 1u; }
            }
        }
        if (!waiting && st == ST_STABLE && lane == 0) {
            p.done[t] = 1;
            const bool use = only_deps && ea.has;                       // Command.executesAtLeast
            p.out[atomicAdd(p.out_cnt, 1u)] = ReadyOut{g, use ? ea.node : ex.node, use ? ea.msb : ex.msb,
                                                       use ? ea.lsb : ex.lsb};
        }
    }
}

inline uint32_t grid_for_waves(uint64_t waves)
{
    uint64_t b = (waves + 3) / 4;
    return (uint32_t)(b < 1 ? 1 : b > 8192 ? 8192 : b);
}


// ---- event-exact readiness (accord_ready_set_mode(ACCORD_READY_EVENTS)) ----
// The reference clears a key bit only when notifyAndUpdatePending's events reach the key
// (local/CommandsForKey.java:1163-1215): a status change of txn X on key k computes k's
// minUncommitted / next / nextWrite (:432-461) and notifies the STABLE waiters of committed[] in an
// executeAt range that depends on the change (notify, :1501-1511, with the count test :1512-1635),
// plus the unmanaged COMMIT / APPLY records of the key (notifyUnmanaged, :1264-1283, 1315-1360).
// One workgroup replays a registration's events in order, each against the state after it: the
// status is applied, then every key of X takes its event; fences and barriers between events make each
// event's writes (statuses, WaitingOn words, pending records) visible to the next.  Orders the
// reference leaves free (keys of one event, waiters of one notify) touch disjoint state.
struct EvCtx {
    const ReadyParams *gens;                 // the live generations (device copies)
    uint32_t ngen;
    const unsigned long long *wmap;          // position -> gi << 32 | t of its waiting txn (~0: none)
    uint32_t wmap_n;
    const uint32_t *ckey, *cent, *kseg0, *kseg1;   // the carried history (CommandsForKey), key-major
    const uint32_t *pk_off, *pk_ent;         // position -> its carried entries
    uint32_t pk_n;
    const uint32_t *uk_off, *uk_slot;        // key -> the unmanaged waiters' key slots on it
    const unsigned long long *uk_w;          //        (gi << 32 | t)
    uint32_t nkeys, key_lo;
    const uint32_t *kb;                      // shardRedundantBefore per key (positions), or null
    StatusView v;
    const uint64_t *tmsb, *tlsb;
    const int32_t *tnode;
    const uint32_t *tg;
    uint32_t tx_n;
    // registration: the events in order (statuses applied here, as reg_apply_kernel does)
    uint32_t n;
    const uint32_t *pos;
    const uint8_t *status;
    const uint64_t *emsb, *elsb;
    const int32_t *enode;
    uint8_t *st;
    uint64_t *xmsb, *xlsb;
    int32_t *xnode;
    uint32_t *chg, *cchg;
    uint32_t epoch;
    uint32_t init_gi;                        // initialisation: the new generation
    const uint32_t *tkeys;                   // truncation: the keys that lost entries
    uint32_t ntkeys;
};

__device__ __forceinline__ Ts ev_tid(const EvCtx &c, uint32_t g)
{
    uint32_t lo = 0, hi = c.tx_n;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (c.tg[m] < g) lo = m + 1; else hi = m;
    }
    return Ts{c.tmsb[lo], c.tlsb[lo], c.tnode[lo]};
}

__device__ __forceinline__ bool ev_waiter(const EvCtx &c, uint32_t g, uint32_t &gi, uint32_t &t)
{
    if (g >= c.wmap_n) return false;
    const unsigned long long w = c.wmap[g];
    if (w == ~0ull) return false;
    gi = (uint32_t)(w >> 32); t = (uint32_t)w;
    return !c.gens[gi].done[t];
}

// KeyDeps key slot of key (absolute ordinal) in waiter t's deps, NONE if absent
__device__ __forceinline__ uint32_t ev_slot(const ReadyParams &p, uint32_t t, uint32_t key)
{
    const uint32_t a = p.key_off[t], b = p.key_off[t + 1];
    uint32_t lo = a, hi = b;
    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (p.keys[m] < key) lo = m + 1; else hi = m; }
    return lo < b && p.keys[lo] == key ? lo - a : NONE;
}

__device__ __forceinline__ bool ev_bit(const ReadyParams &p, uint32_t t, uint32_t b)
{
    return (p.words[p.wo_off[t] + (b >> 6)] >> (b & 63u)) & 1ull;
}

// a key bit cleared by an event; in a registration the waiter is stamped changed at its epoch, so
// the next accord_ready_update's filter lists it (its release is the update's) without a full pass
__device__ __forceinline__ void ev_stamp(const EvCtx &c, const ReadyParams &p, uint32_t t)
{
    if (c.chg) c.chg[p.g[t]] = c.epoch;
}
__device__ __forceinline__ void ev_clear(const EvCtx &c, const ReadyParams &p, uint32_t t, uint32_t b)
{
    p.words[p.wo_off[t] + (b >> 6)] &= ~(1ull << (b & 63u));
    ev_stamp(c, p, t);
}

__device__ __forceinline__ Cand cand_xor(const Cand &c, uint32_t d)
{
    return Cand{(uint32_t)__shfl_xor((int)c.g, d, 64),
                Ts{(uint64_t)__shfl_xor((long long)c.ex.msb, d, 64), (uint64_t)__shfl_xor((long long)c.ex.lsb, d, 64),
                   __shfl_xor(c.ex.node, d, 64)}};
}

// The replay runs on one workgroup of EV_T threads (round 6; it was one wave): events stay in order,
// and every scan inside an event -- a key's carried entries (next / nextWrite / minUncommitted,
// notify's candidates and count tests), its unmanaged records, a waiter's key slots -- is spread over
// the workgroup, with barriers between the dependent steps (a status write before the reads of the
// next step, a key's event before the next key's).
constexpr uint32_t EV_T = 1024, EV_W = EV_T / 64;
struct EvSh {
    uint32_t mu[EV_W];
    Cand nx[EV_W], nw[EV_W], cm[3][EV_W], cmf[3];
    EalRec eal[EV_W];
    uint32_t ncand;
    uint32_t cgi[EV_T], ct[EV_T], cq[EV_T];
};

// the CommandsForKey constructor's minUncommitted, next, nextWrite of key kk (:432-461), next and
// nextWrite nulled when minUncommitted's TxnId precedes their executeAt (uniform results)
__device__ void ev_nexts(const EvCtx &c, EvSh &S, uint32_t kk, uint32_t &mu, Cand &nx, Cand &nw)
{
    const uint32_t tid = threadIdx.x, w = tid >> 6;
    mu = NONE;
    nx = Cand{NONE, {0, 0, 0}};
    nw = Cand{NONE, {0, 0, 0}};
#pragma unroll 4
    for (uint32_t x = c.kseg0[kk] + tid; x < c.kseg1[kk]; x += EV_T) {
        const uint32_t e = c.cent[x], g = e & ENT_TXN_MASK, kind = e >> ENT_KIND_SHIFT;
        const uint32_t st = kind == 2u ? ST_INVALID : status_of(c.v, g);
        if (st < ST_COMMITTED) mu = min(mu, g);
        else if (st < ST_APPLIED) {
            const Cand me{g, exec_of(c.v, g)};
            cand_min(nx, me);
            if (kind == 1u) cand_min(nw, me);
        }
    }
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1) {
        mu = min(mu, (uint32_t)__shfl_xor((int)mu, d, 64));
        cand_min(nx, cand_xor(nx, d));
        cand_min(nw, cand_xor(nw, d));
    }
    if ((tid & 63u) == 0) { S.mu[w] = mu; S.nx[w] = nx; S.nw[w] = nw; }
    __syncthreads();
    mu = NONE;
    nx = Cand{NONE, {0, 0, 0}};
    nw = Cand{NONE, {0, 0, 0}};
    for (uint32_t j = 0; j < EV_W; ++j) {
        mu = min(mu, S.mu[j]);
        cand_min(nx, S.nx[j]);
        cand_min(nw, S.nw[j]);
    }
    __syncthreads();                              // (S reused by the next step)
    if (mu != NONE) {
        const Ts tm = ev_tid(c, mu);
        if (nx.g != NONE && tcmp(tm, nx.ex) < 0) nx.g = NONE;
        if (nw.g != NONE && tcmp(tm, nw.ex) < 0) nw.g = NONE;
    }
}

// the unapplied committed txn with the earliest executeAt per kind class (Read, Write, SyncPoints)
// on key kk, into S.cmf: notify's count tests read these minima (statuses do not change inside an
// event), so the key is scanned once per notify that has candidates, not once per candidate (the
// minima stay in LDS: held in registers across the candidate loop they spilled)
__device__ void ev_class_minima(const EvCtx &c, EvSh &S, uint32_t kk)
{
    const uint32_t tid = threadIdx.x, w = tid >> 6;
    Cand cm[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) cm[k] = Cand{NONE, {0, 0, 0}};
    for (uint32_t x = c.kseg0[kk] + tid; x < c.kseg1[kk]; x += EV_T) {
        const uint32_t e = c.cent[x], u = e & ENT_TXN_MASK, uk = e >> ENT_KIND_SHIFT;
        if (uk == 2u) continue;
        const uint32_t st = status_of(c.v, u);
        if (st < ST_COMMITTED || st >= ST_APPLIED) continue;
        const Cand me{u, exec_of(c.v, u)};
        const uint32_t kc = kind_class(uk);
#pragma unroll
        for (uint32_t k = 0; k < 3; ++k)                // static indices: the array stays in registers
            if (k == kc) cand_min(cm[k], me);
    }
#pragma unroll
    for (uint32_t d = 32; d >= 1; d >>= 1)
#pragma unroll
        for (int k = 0; k < 3; ++k) cand_min(cm[k], cand_xor(cm[k], d));
    if ((tid & 63u) == 0)
#pragma unroll
        for (int k = 0; k < 3; ++k) S.cm[k][w] = cm[k];
    __syncthreads();
    if (tid < 3) {
        Cand m{NONE, {0, 0, 0}};
        for (uint32_t j = 0; j < EV_W; ++j) cand_min(m, S.cm[tid][j]);
        S.cmf[tid] = m;
    }
    __syncthreads();
}

// notify's count test for waiter (gi, t) on key slot q of key kk (expectMissingCount == |missing|):
// no unapplied committed txn of a witnessed kind executes before it on the key -- the key's class
// minima cm[] (ev_class_minima; the waiter itself, at its own executeAt, never blocks) -- and none of
// its deps on the key is uncommitted (a registered-status waiter can hold thousands on a hot key:
// the whole workgroup scans them; uniform result)
__device__ bool ev_managed_ok(const EvCtx &c, const EvSh &S, const ReadyParams &p, uint32_t t, uint32_t q, uint32_t kk,
                              bool use_cm)
{
    const uint32_t tid = threadIdx.x;
    const uint32_t g = p.g[t], kind = (uint32_t)(p.lsb[t] >> 1) & 7u, wmask = witness_mask(kind);
    const Ts ex = exec_of(c.v, g);
#pragma unroll
    for (uint32_t cls = 0; cls < 3; ++cls) {
        const uint32_t gate = cls == 0u ? 0u : cls == 1u ? 1u : 3u;
        if (use_cm && ((wmask >> gate) & 1u) && S.cmf[cls].g != NONE && tcmp(S.cmf[cls].ex, ex) < 0) return false;
    }
    bool blocked = false;
    if (!use_cm) {                                       // a lone candidate: its own scan of the key
        for (uint32_t x = c.kseg0[kk] + tid; x < c.kseg1[kk]; x += EV_T) {
            const uint32_t e = c.cent[x], u = e & ENT_TXN_MASK, uk = e >> ENT_KIND_SHIFT;
            if (uk == 2u) continue;
            const uint32_t st = status_of(c.v, u);
            if (st < ST_COMMITTED || st >= ST_APPLIED) continue;
            const uint32_t cls = kind_class(uk), gate = cls == 0u ? 0u : cls == 1u ? 1u : 3u;
            if (((wmask >> gate) & 1u) && tcmp(exec_of(c.v, u), ex) < 0) blocked = true;
        }
    }
    const uint32_t kbound = c.kb ? c.kb[kk] : 0u;
    const uint32_t K = p.key_off[t + 1] - p.key_off[t], hb = p.k2v_off[t];
    const uint32_t d0 = q == 0 ? K : (uint32_t)p.k2v[hb + q - 1], d1 = (uint32_t)p.k2v[hb + q];
    for (uint32_t x = d0 + tid; x < d1; x += EV_T) {
        const uint32_t u = p.vals[p.val_off[t] + p.k2v[hb + x]];
        if (u >= kbound && status_of(c.v, u) < ST_COMMITTED) blocked = true;
    }
    return __syncthreads_or(blocked ? 1 : 0) == 0;
}

// notify(from, to) (:1501-1511): the STABLE waiters of committed[] executing in [from, to] on kk.
// A chunk's candidates are listed, then tested one by one (the tests read statuses only, and each
// candidate is a different waiter, so their order does not matter)
__device__ void ev_notify(const EvCtx &c, EvSh &S, uint32_t kk, bool has_from, const Ts &from, bool has_to,
                          const Ts &to)
{
    const uint32_t tid = threadIdx.x, key = c.key_lo + kk;
    bool have_cm = false;
    for (uint32_t x0 = c.kseg0[kk]; x0 < c.kseg1[kk]; x0 += EV_T) {
        const uint32_t x = x0 + tid;
        bool cand = false;
        uint32_t gi = 0, t = 0, q = NONE;
        if (x < c.kseg1[kk]) {
            const uint32_t e = c.cent[x], u = e & ENT_TXN_MASK;
            if ((e >> ENT_KIND_SHIFT) != 2u && status_of(c.v, u) == ST_STABLE) {
                const Ts ue = exec_of(c.v, u);
                if ((!has_from || tcmp(ue, from) >= 0) && (!has_to || tcmp(ue, to) <= 0) && ev_waiter(c, u, gi, t)) {
                    const ReadyParams &p = c.gens[gi];
                    const uint32_t kind = (uint32_t)(p.lsb[t] >> 1) & 7u;
                    if ((p.lsb[t] & 1u) == 0 && kind != 2u) {                  // managed
                        q = ev_slot(p, t, key);
                        const uint32_t R = p.rd_off[t + 1] - p.rd_off[t];
                        cand = q != NONE && ev_bit(p, t, R + q);
                    }
                }
            }
        }
        if (tid == 0) S.ncand = 0;
        __syncthreads();
        if (cand) {
            const uint32_t j = atomicAdd(&S.ncand, 1u);
            S.cgi[j] = gi; S.ct[j] = t; S.cq[j] = q;
        }
        __syncthreads();
        const uint32_t nc = S.ncand;
        if (nc > 1 && !have_cm) {                        // uniform: nc was read after the barrier
            __syncthreads();                             // every thread has read S.ncand
            ev_class_minima(c, S, kk);
            have_cm = true;
        }
        for (uint32_t j = 0; j < nc; ++j) {
            const uint32_t lgi = S.cgi[j], lt = S.ct[j], lq = S.cq[j];
            const ReadyParams &p = c.gens[lgi];
            if (ev_managed_ok(c, S, p, lt, lq, kk, have_cm) && tid == 0) {
                const uint32_t R = p.rd_off[lt + 1] - p.rd_off[lt];
                ev_clear(c, p, lt, R + lq);
            }
        }
        __syncthreads();
    }
}

__device__ __forceinline__ void ev_eal(const ReadyParams &p, uint32_t t, const Ts &x)
{
    EalRec a = p.eal[t];
    eal_merge(a, EalRec{x.msb, x.lsb, x.node, 1u});
    p.eal[t] = a;
}

// notifyUnmanaged(COMMIT, minUncommitted) / (APPLY, next) over the unmanaged records of kk (a thread
// per record: each is a different waiter's slot on kk)
__device__ void ev_unmanaged(const EvCtx &c, uint32_t kk, bool commit, uint32_t mu, const Cand &nx)
{
    const uint32_t kbound = c.kb ? c.kb[kk] : 0u;
    for (uint32_t j = c.uk_off[kk] + threadIdx.x; j < c.uk_off[kk + 1]; j += EV_T) {
        const unsigned long long w = c.uk_w[j];
        const uint32_t gi = (uint32_t)(w >> 32), t = (uint32_t)w, q = c.uk_slot[j];
        const ReadyParams &p = c.gens[gi];
        if (p.done[t]) continue;
        const uint32_t R = p.rd_off[t + 1] - p.rd_off[t], slot = p.key_off[t] + q;
        if (!ev_bit(p, t, R + q)) continue;
        uint32_t pd = p.pend[slot], un = p.until[slot];
        if (commit) {
            if (pd != 1u || !(mu == NONE || mu > un)) continue;
            const uint32_t kind = (uint32_t)(p.lsb[t] >> 1) & 7u, g = p.g[t];
            const bool only_deps = kind == 4u || kind == 2u;
            const uint32_t K = p.key_off[t + 1] - p.key_off[t], hb = p.k2v_off[t];
            const uint32_t d0 = q == 0 ? K : (uint32_t)p.k2v[hb + q - 1], d1 = (uint32_t)p.k2v[hb + q];
            uint32_t ea = NONE;
            const int r = unmanaged_eval(p, t, d0, d1, kbound, exec_of(c.v, g), only_deps, false, un, ea);
            if (r == 1) { pd = 3; ev_clear(c, p, t, R + q); }
            else {
                pd = 2;
                if (only_deps && ea != NONE) ev_eal(p, t, exec_of(c.v, ea));   // :1370-1380
            }
            p.pend[slot] = (uint8_t)pd;
            p.until[slot] = un;
        } else if (pd == 2u && (nx.g == NONE || tcmp(exec_of(c.v, un), nx.ex) < 0)) {
            p.pend[slot] = 3;
            ev_clear(c, p, t, R + q);
        }
    }
}

// registerUnmanaged (:1406-1498) on every key slot of an unmanaged waiter that now hasBeen(Stable)
__device__ void ev_register_unmanaged(const EvCtx &c, EvSh &S, uint32_t gi, uint32_t t)
{
    const uint32_t tid = threadIdx.x, w = tid >> 6;
    const ReadyParams &p = c.gens[gi];
    const uint32_t g = p.g[t], kind = (uint32_t)(p.lsb[t] >> 1) & 7u;
    const bool only_deps = kind == 4u || kind == 2u;
    const uint32_t R = p.rd_off[t + 1] - p.rd_off[t], K = p.key_off[t + 1] - p.key_off[t], hb = p.k2v_off[t];
    const Ts ex = exec_of(c.v, g);
    for (uint32_t q0 = 0; q0 < K; q0 += EV_T) {
        const uint32_t q = q0 + tid;
        bool has = false;
        Ts cand{0, 0, 0};
        if (q < K) {
            const uint32_t slot = p.key_off[t] + q;
            if (ev_bit(p, t, R + q) && p.pend[slot] == 0u) {
                const uint32_t kk = p.keys[slot] - c.key_lo, kbound = c.kb ? c.kb[kk] : 0u;
                const uint32_t d0 = q == 0 ? K : (uint32_t)p.k2v[hb + q - 1], d1 = (uint32_t)p.k2v[hb + q];
                uint32_t un = p.until[slot], ea = NONE;
                const int r = unmanaged_eval(p, t, d0, d1, kbound, ex, only_deps, true, un, ea);
                p.pend[slot] = (uint8_t)(r == 1 ? 3u : r == 0 ? 2u : 1u);
                p.until[slot] = un;
                if (r == 1) {
                    atomicAnd(&p.words[p.wo_off[t] + ((R + q) >> 6)], ~(1ull << ((R + q) & 63u)));
                    ev_stamp(c, p, t);
                }
                if (r == 0 && only_deps && ea != NONE) { has = true; cand = exec_of(c.v, ea); }   // :1470-1478
            }
        }
        const EalRec m = eal_wave_max(has, cand);
        if ((tid & 63u) == 0) S.eal[w] = m;
        __syncthreads();
        if (tid == 0) {
            EalRec a = p.eal[t];
            for (uint32_t j = 0; j < EV_W; ++j) eal_merge(a, S.eal[j]);
            p.eal[t] = a;
        }
        __syncthreads();
    }
}

// notifyAndUpdatePending(safeStore, X, nw, exec, prev) on key kk (:1163-1215), after X's update
__device__ void ev_key_event(const EvCtx &c, EvSh &S, uint32_t kk, uint32_t X, uint32_t prev, uint32_t nw,
                             const Ts &exec)
{
    uint32_t mu;
    Cand nx, nwr;
    ev_nexts(c, S, kk, mu, nx, nwr);
    // the notify range of the event (one call site: the notify is inlined once)
    bool doit = false, hf = false, ht = false;
    Ts from{0, 0, 0}, to{0, 0, 0};
    if (nw == ST_STABLE || nw == ST_COMMITTED) {
        const int cmp = nwr.g == NONE ? -1 : tcmp(exec, nwr.ex);
        if (cmp <= 0) {
            if (nw == ST_STABLE) { doit = true; hf = nx.g != NONE; from = nx.ex; ht = true; to = exec; }   // we may execute
        } else {
            const Ts tx = ev_tid(c, X);
            // waiters on us may be ready, if we execute after them, were known and not committed
            if (!(prev == ST_COMMITTED || tcmp(nwr.ex, tx) < 0 || tcmp(exec, tx) == 0)) {
                doit = true; hf = true; from = nx.ex; ht = true; to = nwr.ex;
            }
        }
    } else if ((nw == ST_APPLIED || nw == ST_INVALID) && nx.g != NONE) {
        doit = true; hf = true; from = nx.ex; ht = nwr.g != NONE; to = nwr.ex;
    }
    if (doit) ev_notify(c, S, kk, hf, from, ht, to);
    if (nw >= ST_COMMITTED && prev < ST_COMMITTED) {
        ev_unmanaged(c, kk, true, mu, nx);
        __threadfence();
        __syncthreads();
    }
    if (mu == NONE || nx.g != NONE) ev_unmanaged(c, kk, false, mu, nx);
}

// every key event of txn g (its carried entries; truncated keys excluded)
__device__ void ev_txn_keys(const EvCtx &c, EvSh &S, uint32_t g, uint32_t prev, uint32_t nw, const Ts &exec)
{
    if (g >= c.pk_n) return;
    for (uint32_t j = c.pk_off[g]; j < c.pk_off[g + 1]; ++j) {
        const uint32_t kk = c.ckey[c.pk_ent[j]];
        if (c.kb && g < c.kb[kk]) continue;
        ev_key_event(c, S, kk, g, prev, nw, exec);
        __threadfence();
        __syncthreads();
    }
}

// MODE 0: a registration's events; 1: a generation's initialisation; 2: truncated keys
template <int MODE>
__global__ __launch_bounds__(EV_T) void rd_event_kernel(EvCtx c)
{
    __shared__ EvSh S;
    const uint32_t tid = threadIdx.x;
    if (MODE == 0) {
        for (uint32_t r = 0; r < c.n; ++r) {
            const uint32_t g = c.pos[r], nw = c.status[r], cur = c.st[g];
            __syncthreads();                                 // every thread has read the old status
            if (tid == 0) {                                  // the status first (reg_apply_kernel's update)
                c.st[g] = (uint8_t)nw;
                c.chg[g] = c.epoch;
                if (cur < ST_COMMITTED && nw >= ST_COMMITTED) c.cchg[g] = c.epoch;
                if ((nw >= ST_ACCEPTED && nw <= ST_APPLIED) || nw == ST_TRUNC_APPLY) {
                    c.xmsb[g] = c.emsb[r]; c.xlsb[g] = c.elsb[r]; c.xnode[g] = c.enode[r];
                }
            }
            __threadfence();
            __syncthreads();
            uint32_t gi, t;
            const bool w = ev_waiter(c, g, gi, t);
            if (w && nw >= ST_STABLE && nw < ST_INVALID && cur < ST_STABLE) {
                const ReadyParams &p = c.gens[gi];
                const uint32_t kind = (uint32_t)(p.lsb[t] >> 1) & 7u;
                if ((p.lsb[t] & 1u) != 0 || kind == 2u) ev_register_unmanaged(c, S, gi, t);   // unmanaged
                __threadfence();
                __syncthreads();
            }
            // CommandsForKey.update on every key (TruncatedApply and Erased leave it as INVALID_OR_TRUNCATED)
            const uint32_t cs = nw >= ST_INVALID ? ST_INVALID : nw, ps = cur >= ST_INVALID ? ST_INVALID : cur;
            ev_txn_keys(c, S, g, ps, cs, exec_of(c.v, g));
        }
    } else if (MODE == 1) {
        const ReadyParams &p = c.gens[c.init_gi];
        for (uint32_t t = 0; t < p.n; ++t) {
            const uint32_t g = p.g[t], st = status_of(c.v, g);
            if (st < ST_STABLE || st >= ST_INVALID) continue;
            const uint32_t kind = (uint32_t)(p.lsb[t] >> 1) & 7u;
            if ((p.lsb[t] & 1u) != 0 || kind == 2u) {
                ev_register_unmanaged(c, S, c.init_gi, t);
                __threadfence();
                __syncthreads();
                continue;
            }
            if (st != ST_STABLE) continue;
            ev_txn_keys(c, S, g, ST_STABLE, ST_STABLE, exec_of(c.v, g));
        }
    } else {
        for (uint32_t j = 0; j < c.ntkeys; ++j) {        // notifyAndUpdatePending(safeStore, prevCfk)
            const uint32_t kk = c.tkeys[j];
            uint32_t mu;
            Cand nx, nwr;
            ev_nexts(c, S, kk, mu, nx, nwr);
            if (mu == NONE || nx.g != NONE) ev_unmanaged(c, kk, false, mu, nx);
            __threadfence();
            __syncthreads();
        }
    }
}

// index builders: position -> waiting txn, key -> unmanaged slots, position -> carried entries
__global__ __launch_bounds__(256) void ev_wmap_kernel(ReadyParams p, uint32_t gi, unsigned long long *wmap, uint32_t wn)
{
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < p.n; t += gridDim.x * blockDim.x)
        if (!p.done[t] && p.g[t] < wn) wmap[p.g[t]] = (unsigned long long)gi << 32 | t;
}

template <bool FILL>
__global__ __launch_bounds__(256) void ev_uk_kernel(ReadyParams p, uint32_t gi, uint32_t *cnt, const uint32_t *off,
                                                    uint32_t *cur, unsigned long long *uw, uint32_t *us)
{
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < p.n; t += gridDim.x * blockDim.x) {
        const uint32_t kind = (uint32_t)(p.lsb[t] >> 1) & 7u;
        if (p.done[t] || ((p.lsb[t] & 1u) == 0 && kind != 2u)) continue;     // unmanaged waiting txns
        for (uint32_t q = 0, K = p.key_off[t + 1] - p.key_off[t]; q < K; ++q) {
            const uint32_t kk = p.keys[p.key_off[t] + q] - p.key_lo;
            if (!FILL) { atomicAdd(&cnt[kk], 1u); continue; }
            const uint32_t j = off[kk] + atomicAdd(&cur[kk], 1u);
            uw[j] = (unsigned long long)gi << 32 | t;
            us[j] = q;
        }
    }
}

template <bool FILL>
__global__ __launch_bounds__(256) void ev_pk_kernel(uint32_t C, const uint32_t *__restrict__ cent, uint32_t pn,
                                                    uint32_t *cnt, const uint32_t *off, uint32_t *cur, uint32_t *ent)
{
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < C; x += gridDim.x * blockDim.x) {
        const uint32_t e = cent[x], g = e & ENT_TXN_MASK;
        if ((e >> ENT_KIND_SHIFT) == 2u || g >= pn) continue;             // not in CommandsForKey
        if (!FILL) atomicAdd(&cnt[g], 1u);
        else ent[off[g] + atomicAdd(&cur[g], 1u)] = x;
    }
}

// truncation: keys whose carried history starts below their new bound (entries leave the CFK)
__global__ __launch_bounds__(256) void ev_tkeys_kernel(uint32_t nkeys, const uint32_t *__restrict__ kseg0,
                                                       const uint32_t *__restrict__ kseg1, const uint32_t *__restrict__ cent,
                                                       const uint32_t *__restrict__ kb, uint32_t *list, uint32_t *cnt)
{
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nkeys; k += gridDim.x * blockDim.x) {
        bool any = false;
        for (uint32_t x = kseg0[k]; x < kseg1[k] && !any; ++x) any = (cent[x] & ENT_TXN_MASK) < kb[k];
        if (any) list[atomicAdd(cnt, 1u)] = k;
    }
}

} // namespace

namespace accord_impl {

struct ReadyGen {
    uint32_t n = 0, left = 0, glo = 0, ghi = 0;   // txns, not yet ready, first / last global position
    uint64_t rvals = 0;                           // RangeDeps txnIds of its txns (setAppliedAndPropagate's pool bound)
    bool fresh = true;                            // not evaluated yet
    uint64_t words = 0;
    DevBuf g, lsb, rd_off, rd_vals, key_off, keys, val_off, vals, k2v_off, k2v, wo_off, wo, aoi, pend, until, done;
    DevBuf eal, pkoff, pkeys, proff, prs, pre, rrng_off, rrs, rre, rr2v_off, rr2v;
    void release()
    {
        DevBuf *b[] = {&g, &lsb, &rd_off, &rd_vals, &key_off, &keys, &val_off, &vals, &k2v_off, &k2v, &wo_off, &wo, &aoi,
                       &pend, &until, &done, &eal, &pkoff, &pkeys, &proff, &prs, &pre, &rrng_off, &rrs, &rre,
                       &rr2v_off, &rr2v};
        for (DevBuf *x : b) x->release();
    }
};

void ready_destroy(accord_store *s)
{
    if (s->rdy_stats && s->rdy_stats[0])
        fprintf(stderr, "ready stats: calls %llu dirty keys %llu waiting-set scans %llu evaluated %llu\n",
                (unsigned long long)s->rdy_stats[0], (unsigned long long)s->rdy_stats[1],
                (unsigned long long)s->rdy_stats[2], (unsigned long long)s->rdy_stats[3]);
    delete[] s->rdy_stats;
    s->rdy_stats = nullptr;
    for (ReadyGen *r : s->rdy_gens) { r->release(); delete r; }
    s->rdy_gens.clear();
    s->rdy_batch_gen = nullptr;
    s->rdy_waiting = 0;
    if (s->rdy_host) { (void)hipHostFree(s->rdy_host); s->rdy_host = nullptr; }
    if (s->rdy_tab_host) { (void)hipHostFree(s->rdy_tab_host); s->rdy_tab_host = nullptr; s->rdy_tab_cap = 0; }
    s->rdy_pv_at.release(); s->rdy_pv_len.release(); s->rdy_pv_pool.release();
    s->rdy_pv_n = 0;
    s->rdy_pv_pos = 0;
}

// A batch's WaitingOn may be initialised again (a retry, or before and after its RedundantBefore
// union) only while its generation has not been evaluated: the new generation then replaces it.
// After an accord_ready_update has seen it, its released txns were reported and a second
// generation would report them again -- refused.
int32_t ready_batch_check(accord_store *s)
{
    if (s->rdy_batch_gen && !s->rdy_batch_gen->fresh)
        return fail(s, ACCORD_ERR_STATE, "the batch's WaitingOn is already in the waiting set and was evaluated "
                                         "by accord_ready_update; compute the next batch first");
    return ACCORD_OK;
}

namespace {
// a larger buffer keeping the first `used` bytes, the rest zeroed
hipError_t grow_keep(DevBuf &b, size_t used, size_t want, hipStream_t st)
{
    if (want <= b.cap && b.p) return hipSuccess;
    DevBuf nb;
    hipError_t e = nb.ensure(std::max(want, b.cap * 2));
    if (e == hipSuccess) e = hipMemsetAsync(nb.p, 0, nb.cap, st);
    if (e == hipSuccess && used && b.p) e = hipMemcpyAsync(nb.p, b.p, std::min(used, b.cap), hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) { nb.release(); return e; }
    b.release();
    b = nb;
    return hipSuccess;
}

StatusView store_view(accord_store *s)
{
    StatusView v;
    v.status = s->rg_status.as<uint8_t>();
    v.emsb = s->rg_emsb.as<uint64_t>(); v.elsb = s->rg_elsb.as<uint64_t>(); v.enode = s->rg_enode.as<int32_t>();
    v.known = s->rg_known;
    return v;
}

// the per-key shardRedundantBefore bounds on the device (null when none was set)
int32_t store_kb(accord_store *s, bool force, const uint32_t **kb)
{
    const uint32_t nkeys = s->cfg.key_hi - s->cfg.key_lo;
    const bool has_kb = s->rdy_kb_host.size() == nkeys;     // a shardRedundantBefore bound was set
    if ((s->rdy_kb_dirty || force) && has_kb) {
        HIPCHECK(s, s->rdy_kb.ensure((size_t)nkeys * 4 + 4));
        HIPCHECK(s, hipMemcpyAsync(s->rdy_kb.p, s->rdy_kb_host.data(), (size_t)nkeys * 4, hipMemcpyHostToDevice, s->stream));
        HIPCHECK(s, hipStreamSynchronize(s->stream));
        s->rdy_kb_dirty = false;
    }
    *kb = has_kb && s->rdy_kb.p ? s->rdy_kb.as<uint32_t>() : nullptr;
    return ACCORD_OK;
}

// segment bounds of the carried history per key, once per carry version
int32_t store_kseg(accord_store *s, bool force)
{
    const uint32_t nkeys = s->cfg.key_hi - s->cfg.key_lo, C = s->carry_n;
    hipStream_t st = s->stream;
    if (s->rdy_kseg_version != s->carry_version || !s->rdy_kseg0.p || force) {
        HIPCHECK(s, s->rdy_kseg0.ensure((size_t)nkeys * 4 + 4));
        HIPCHECK(s, s->rdy_kseg1.ensure((size_t)nkeys * 4 + 4));
        HIPCHECK(s, hipMemsetAsync(s->rdy_kseg0.p, 0, (size_t)nkeys * 4, st));
        HIPCHECK(s, hipMemsetAsync(s->rdy_kseg1.p, 0, (size_t)nkeys * 4, st));
        if (C) hipLaunchKernelGGL(rd_seg_kernel, dim3(std::min<uint32_t>((C + 255) / 256, 8192u)), dim3(256), 0, st, C,
                                  s->cy_key.as<uint32_t>(), s->rdy_kseg0.as<uint32_t>(), s->rdy_kseg1.as<uint32_t>());
        s->rdy_kseg_version = s->carry_version;
    }
    return ACCORD_OK;
}

// a generation's table entry: its deps, WaitingOn and the store's shared tables
ReadyParams gen_params(accord_store *s, ReadyGen *r, const StatusView &v, const uint32_t *kb)
{
    ReadyParams p{};
    p.n = r->n; p.key_lo = s->cfg.key_lo;
    p.g = r->g.as<uint32_t>(); p.lsb = r->lsb.as<uint64_t>();
    p.tmsb = s->rg_tmsb.as<uint64_t>(); p.tlsb = s->rg_tlsb.as<uint64_t>(); p.tnode = s->rg_tnode.as<int32_t>();
    p.tg = s->rg_tg.as<uint32_t>(); p.tx_n = s->rg_tx_n;
    p.rd_off = r->rd_off.as<uint32_t>(); p.rd_vals = r->rd_vals.as<uint32_t>();
    p.key_off = r->key_off.as<uint32_t>(); p.keys = r->keys.as<uint32_t>();
    p.val_off = r->val_off.as<uint32_t>(); p.vals = r->vals.as<uint32_t>();
    p.k2v_off = r->k2v_off.as<uint32_t>(); p.k2v = r->k2v.as<int32_t>();
    p.wo_off = r->wo_off.as<uint32_t>(); p.words = r->wo.as<unsigned long long>(); p.aoi = r->aoi.as<unsigned long long>();
    p.pend = r->pend.as<uint8_t>(); p.until = r->until.as<uint32_t>(); p.done = r->done.as<uint8_t>();
    p.eal = r->eal.as<EalRec>();
    p.kb = kb;
    p.v = v;
    return p;
}

// event-exact readiness: the generations' table, position -> waiting txn, key -> unmanaged slots,
// position -> carried entries (rebuilt with the carry), the kernel's context
int32_t ev_prepare(accord_store *s, EvCtx &c, ReadyGen *want, uint32_t *want_gi)
{
    hipStream_t st = s->stream;
    const uint32_t nkeys = s->cfg.key_hi - s->cfg.key_lo, C = s->carry_n, pn = s->next_global;
    const StatusView v = store_view(s);
    const uint32_t *kb = nullptr;
    EV_RC(store_kb(s, false, &kb));
    EV_RC(store_kseg(s, false));
    std::vector<ReadyParams> P;
    size_t ukcap = 1;
    for (ReadyGen *r : s->rdy_gens) {
        if (r->left == 0) continue;
        if (r == want && want_gi) *want_gi = (uint32_t)P.size();
        P.push_back(gen_params(s, r, v, kb));
        ukcap += r->keys.cap / 4;
    }
    HIPCHECK(s, s->ev_gens.ensure(P.size() * sizeof(ReadyParams) + 64));
    if (!P.empty())
        HIPCHECK(s, hipMemcpyAsync(s->ev_gens.p, P.data(), P.size() * sizeof(ReadyParams), hipMemcpyHostToDevice, st));
    HIPCHECK(s, s->ev_tot.ensure(64));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(std::max({nkeys, pn, 1u})), st));
    // position -> waiting txn
    HIPCHECK(s, s->ev_wmap.ensure((size_t)pn * 8 + 8));
    HIPCHECK(s, hipMemsetAsync(s->ev_wmap.p, 0xFF, (size_t)pn * 8 + 8, st));
    for (size_t i = 0; i < P.size(); ++i)
        hipLaunchKernelGGL(ev_wmap_kernel, dim3(grid_for_waves((P[i].n + 63) / 64)), dim3(256), 0, st, P[i], (uint32_t)i,
                           s->ev_wmap.as<unsigned long long>(), pn);
    // key -> unmanaged slots (CSR)
    HIPCHECK(s, s->ev_ukcnt.ensure((size_t)nkeys * 4 + 8));
    HIPCHECK(s, s->ev_ukoff.ensure((size_t)nkeys * 4 + 8));
    HIPCHECK(s, s->ev_ukw.ensure(ukcap * 8));
    HIPCHECK(s, s->ev_uks.ensure(ukcap * 4));
    HIPCHECK(s, hipMemsetAsync(s->ev_ukcnt.p, 0, (size_t)nkeys * 4 + 8, st));
    for (size_t i = 0; i < P.size(); ++i)
        hipLaunchKernelGGL(ev_uk_kernel<false>, dim3(grid_for_waves((P[i].n + 63) / 64)), dim3(256), 0, st, P[i],
                           (uint32_t)i, s->ev_ukcnt.as<uint32_t>(), nullptr, nullptr, nullptr, nullptr);
    if (nkeys) accord::exclusive_scan_u32(s->ev_ukcnt.as<uint32_t>(), s->ev_ukoff.as<uint32_t>(), nkeys,
                                          s->ev_tot.as<unsigned long long>(), s->scan_tmp.p, st);
    HIPCHECK(s, hipMemsetAsync(s->ev_ukcnt.p, 0, (size_t)nkeys * 4 + 8, st));
    for (size_t i = 0; i < P.size(); ++i)
        hipLaunchKernelGGL(ev_uk_kernel<true>, dim3(grid_for_waves((P[i].n + 63) / 64)), dim3(256), 0, st, P[i],
                           (uint32_t)i, nullptr, s->ev_ukoff.as<uint32_t>(), s->ev_ukcnt.as<uint32_t>(),
                           s->ev_ukw.as<unsigned long long>(), s->ev_uks.as<uint32_t>());
    // position -> carried entries (CommandsForKey membership), per carry version
    if (s->ev_pk_version != s->carry_version || !s->ev_pkoff.p || s->ev_pk_n != pn) {
        HIPCHECK(s, s->ev_pkcnt.ensure((size_t)pn * 4 + 8));
        HIPCHECK(s, s->ev_pkoff.ensure((size_t)pn * 4 + 8));
        HIPCHECK(s, s->ev_pkent.ensure((size_t)C * 4 + 8));
        HIPCHECK(s, hipMemsetAsync(s->ev_pkcnt.p, 0, (size_t)pn * 4 + 8, st));
        if (C) hipLaunchKernelGGL(ev_pk_kernel<false>, dim3(std::min<uint32_t>((C + 255) / 256, 8192u)), dim3(256), 0, st,
                                  C, s->cy_ent.as<uint32_t>(), pn, s->ev_pkcnt.as<uint32_t>(), nullptr, nullptr, nullptr);
        if (pn) accord::exclusive_scan_u32(s->ev_pkcnt.as<uint32_t>(), s->ev_pkoff.as<uint32_t>(), pn,
                                           s->ev_tot.as<unsigned long long>(), s->scan_tmp.p, st);
        else HIPCHECK(s, hipMemsetAsync(s->ev_pkoff.p, 0, 4, st));
        HIPCHECK(s, hipMemsetAsync(s->ev_pkcnt.p, 0, (size_t)pn * 4 + 8, st));
        if (C) hipLaunchKernelGGL(ev_pk_kernel<true>, dim3(std::min<uint32_t>((C + 255) / 256, 8192u)), dim3(256), 0, st,
                                  C, s->cy_ent.as<uint32_t>(), pn, nullptr, s->ev_pkoff.as<uint32_t>(),
                                  s->ev_pkcnt.as<uint32_t>(), s->ev_pkent.as<uint32_t>());
        s->ev_pk_version = s->carry_version;
        s->ev_pk_n = pn;
    }
    c = EvCtx{};
    c.gens = s->ev_gens.as<ReadyParams>(); c.ngen = (uint32_t)P.size();
    c.wmap = s->ev_wmap.as<unsigned long long>(); c.wmap_n = pn;
    c.ckey = s->cy_key.as<uint32_t>(); c.cent = s->cy_ent.as<uint32_t>();
    c.kseg0 = s->rdy_kseg0.as<uint32_t>(); c.kseg1 = s->rdy_kseg1.as<uint32_t>();
    c.pk_off = s->ev_pkoff.as<uint32_t>(); c.pk_ent = s->ev_pkent.as<uint32_t>(); c.pk_n = s->ev_pk_n;
    c.uk_off = s->ev_ukoff.as<uint32_t>(); c.uk_slot = s->ev_uks.as<uint32_t>(); c.uk_w = s->ev_ukw.as<unsigned long long>();
    c.nkeys = nkeys; c.key_lo = s->cfg.key_lo;
    c.kb = kb;
    c.v = v;
    c.tmsb = s->rg_tmsb.as<uint64_t>(); c.tlsb = s->rg_tlsb.as<uint64_t>(); c.tnode = s->rg_tnode.as<int32_t>();
    c.tg = s->rg_tg.as<uint32_t>(); c.tx_n = s->rg_tx_n;
    HIPCHECK(s, hipStreamSynchronize(st));          // the table copy's host source
    return ACCORD_OK;
}

// the generation's device copies of the batch's deps and WaitingOn; no state of the store changes
int32_t ready_gen_fill(accord_store *s, ReadyGen *r)
{
    const uint32_t n = s->n;
    hipStream_t st = s->stream;
    r->n = r->left = n;
    r->words = s->wo_words_total;
    const size_t n1 = (size_t)n + 1;
    auto copy = [&](DevBuf &dst, const void *src, size_t bytes) -> hipError_t {
        hipError_t e = dst.ensure(bytes + 8);
        if (e == hipSuccess && bytes) e = hipMemcpyAsync(dst.p, src, bytes, hipMemcpyDeviceToDevice, st);
        return e;
    };
    const CurDeps cd = cur_deps(s);                           // the batch's deps (with RedundantBefore's)
    HIPCHECK(s, copy(r->g, s->txn_index.p, (size_t)n * 4));  // resident stores: global positions
    HIPCHECK(s, hipMemcpyAsync(&r->glo, s->txn_index.p, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipMemcpyAsync(&r->ghi, s->txn_index.as<uint32_t>() + n - 1, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(s, copy(r->lsb, s->lsb.p, (size_t)n * 8));
    HIPCHECK(s, copy(r->rd_off, cd.rd_val_off, n1 * 4));
    HIPCHECK(s, copy(r->rd_vals, cd.rd_vals, cd.tot_rvals * 4));
    r->rvals = cd.tot_rvals;
    HIPCHECK(s, copy(r->key_off, cd.kd_key_off, n1 * 4));
    HIPCHECK(s, copy(r->keys, cd.kd_keys, cd.tot_keys * 4));
    HIPCHECK(s, copy(r->val_off, cd.kd_val_off, n1 * 4));
    HIPCHECK(s, copy(r->vals, cd.kd_vals, cd.tot_vals * 4));
    HIPCHECK(s, copy(r->k2v_off, cd.kd_k2v_off, n1 * 4));
    HIPCHECK(s, copy(r->k2v, cd.kd_k2v, cd.tot_k2v * 4));
    HIPCHECK(s, copy(r->wo_off, s->wo_off.p, n1 * 4));
    HIPCHECK(s, copy(r->wo, s->wo_words.p, s->wo_words_total * 8));
    HIPCHECK(s, copy(r->aoi, s->wo_aoi.p, s->wo_words_total * 8));
    HIPCHECK(s, copy(r->eal, s->wo_eal.p, (size_t)n * sizeof(EalRec)));
    if (const char *f = getenv("ACCORD_INJECT_FAIL"); f && std::strcmp(f, "ready_gen") == 0)   // test hook
        return fail(s, ACCORD_ERR_OOM, "injected failure (ACCORD_INJECT_FAIL=ready_gen) with the generation half built");
    // the participants (the batch's keys / ranges) and RangeDeps ranges: removeRedundantDependencies
    HIPCHECK(s, copy(r->pkoff, s->key_off.p, n1 * 4));
    HIPCHECK(s, copy(r->pkeys, s->key_ord.p, (size_t)s->P * 4));
    if (s->R) {
        HIPCHECK(s, copy(r->proff, s->rng_off.p, n1 * 4));
        HIPCHECK(s, copy(r->prs, s->rng_start.p, (size_t)s->R * 4));
        HIPCHECK(s, copy(r->pre, s->rng_end.p, (size_t)s->R * 4));
    } else {
        HIPCHECK(s, r->proff.ensure(n1 * 4 + 8));
        HIPCHECK(s, hipMemsetAsync(r->proff.p, 0, n1 * 4, st));
    }
    HIPCHECK(s, copy(r->rrng_off, cd.rd_rng_off, n1 * 4));
    HIPCHECK(s, copy(r->rrs, cd.rd_rng_start, cd.tot_rngs * 4));
    HIPCHECK(s, copy(r->rre, cd.rd_rng_end, cd.tot_rngs * 4));
    HIPCHECK(s, copy(r->rr2v_off, cd.rd_r2v_off, n1 * 4));
    HIPCHECK(s, copy(r->rr2v, cd.rd_r2v, cd.tot_r2v * 4));
    HIPCHECK(s, r->pend.ensure(cd.tot_keys + 8));
    HIPCHECK(s, r->until.ensure(cd.tot_keys * 4 + 8));
    HIPCHECK(s, r->done.ensure((size_t)n + 8));
    HIPCHECK(s, hipMemsetAsync(r->pend.p, 0, cd.tot_keys + 8, st));
    HIPCHECK(s, hipMemsetAsync(r->until.p, 0, cd.tot_keys * 4 + 8, st));
    HIPCHECK(s, hipMemsetAsync(r->done.p, 0, (size_t)n + 8, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    return ACCORD_OK;
}
} // namespace

// the last computed batch (its WaitingOn just initialised) joins the waiting set.  The generation is
// built completely before it joins (a failed copy or allocation leaves the set as it was), and it
// replaces an unevaluated generation of the same batch (ready_batch_check)
int32_t ready_track_batch(accord_store *s)
{
    if (s->n == 0) return ACCORD_OK;
    int32_t rc = ready_batch_check(s);
    if (rc != ACCORD_OK) return rc;
    ReadyGen *r = new (std::nothrow) ReadyGen();
    if (!r) return fail(s, ACCORD_ERR_OOM, "out of host memory");
    rc = ready_gen_fill(s, r);
    if (rc == ACCORD_OK) {
        try { s->rdy_gens.reserve(s->rdy_gens.size() + 1); }
        catch (...) { rc = fail(s, ACCORD_ERR_OOM, "out of host memory"); }
    }
    if (rc != ACCORD_OK) { r->release(); delete r; return rc; }
    if (ReadyGen *old = s->rdy_batch_gen) {                    // an unevaluated generation of this batch
        for (size_t i = 0; i < s->rdy_gens.size(); ++i)
            if (s->rdy_gens[i] == old) { s->rdy_gens.erase(s->rdy_gens.begin() + i); break; }
        s->rdy_waiting -= old->left;
        old->release();
        delete old;
    }
    s->rdy_gens.push_back(r);
    s->rdy_batch_gen = r;
    s->rdy_waiting += r->n;
    return ACCORD_OK;
}

int32_t ready_register_events(accord_store *s, uint32_t n, const uint32_t *pos, const uint8_t *status,
                              const uint64_t *emsb, const uint64_t *elsb, const int32_t *enode, uint32_t epoch)
{
    EvCtx c;
    EV_RC(ev_prepare(s, c, nullptr, nullptr));
    c.n = n; c.pos = pos; c.status = status; c.emsb = emsb; c.elsb = elsb; c.enode = enode;
    c.st = s->rg_status.as<uint8_t>();
    c.xmsb = s->rg_emsb.as<uint64_t>(); c.xlsb = s->rg_elsb.as<uint64_t>(); c.xnode = s->rg_enode.as<int32_t>();
    c.chg = s->rg_chg.as<uint32_t>(); c.cchg = s->rg_cchg.as<uint32_t>(); c.epoch = epoch;
    hipLaunchKernelGGL(rd_event_kernel<0>, dim3(1), dim3(EV_T), 0, s->stream, c);
    HIPCHECK(s, hipGetLastError());
    return ACCORD_OK;
}

int32_t ready_init_events(accord_store *s)
{
    ReadyGen *r = s->rdy_batch_gen;
    if (!r || r->n == 0) return ACCORD_OK;
    EvCtx c;
    uint32_t gi = ~0u;
    EV_RC(ev_prepare(s, c, r, &gi));
    if (gi == ~0u) return ACCORD_OK;
    c.init_gi = gi;
    hipLaunchKernelGGL(rd_event_kernel<1>, dim3(1), dim3(EV_T), 0, s->stream, c);
    HIPCHECK(s, hipGetLastError());
    return ACCORD_OK;
}

// before a truncation: the keys whose carried history has an entry below the key's new bound
int32_t ready_truncate_keys(accord_store *s, const std::vector<uint32_t> &kb, std::vector<uint32_t> &keys)
{
    keys.clear();
    const uint32_t nkeys = s->cfg.key_hi - s->cfg.key_lo;
    if (!nkeys || !s->carry_n) return ACCORD_OK;
    hipStream_t st = s->stream;
    EV_RC(store_kseg(s, false));
    HIPCHECK(s, s->ev_tk.ensure((size_t)nkeys * 8 + 16));
    uint32_t *kbd = s->ev_tk.as<uint32_t>(), *list = kbd + nkeys, *cnt = list + nkeys;
    HIPCHECK(s, hipMemcpyAsync(kbd, kb.data(), (size_t)nkeys * 4, hipMemcpyHostToDevice, st));
    HIPCHECK(s, hipMemsetAsync(cnt, 0, 4, st));
    hipLaunchKernelGGL(ev_tkeys_kernel, dim3(grid_for_waves((nkeys + 63) / 64)), dim3(256), 0, st, nkeys,
                       s->rdy_kseg0.as<uint32_t>(), s->rdy_kseg1.as<uint32_t>(), s->cy_ent.as<uint32_t>(), kbd, list, cnt);
    uint32_t m = 0;
    HIPCHECK(s, hipMemcpyAsync(&m, cnt, 4, hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    keys.resize(m);
    if (m) {
        HIPCHECK(s, hipMemcpyAsync(keys.data(), list, (size_t)m * 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(s, hipStreamSynchronize(st));
    }
    return ACCORD_OK;
}

// after it: notifyAndUpdatePending(safeStore, prevCfk) on those keys (the unmanaged APPLY records)
int32_t ready_truncate_events(accord_store *s, const std::vector<uint32_t> &keys)
{
    if (keys.empty()) return ACCORD_OK;
    EvCtx c;
    EV_RC(ev_prepare(s, c, nullptr, nullptr));
    if (c.ngen == 0) return ACCORD_OK;
    HIPCHECK(s, s->ev_tk.ensure(keys.size() * 4 + 16));
    HIPCHECK(s, hipMemcpyAsync(s->ev_tk.p, keys.data(), keys.size() * 4, hipMemcpyHostToDevice, s->stream));
    HIPCHECK(s, hipStreamSynchronize(s->stream));
    c.tkeys = s->ev_tk.as<uint32_t>(); c.ntkeys = (uint32_t)keys.size();
    hipLaunchKernelGGL(rd_event_kernel<2>, dim3(1), dim3(EV_T), 0, s->stream, c);
    HIPCHECK(s, hipGetLastError());
    return ACCORD_OK;
}

} // namespace accord_impl

extern "C" int32_t accord_ready_set_mode(accord_store *s, uint32_t mode)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (mode > ACCORD_READY_EVENTS) return fail(s, ACCORD_ERR_ARG, "unknown readiness mode %u", mode);
    if (!accord_impl::registered_mode(s))
        return fail(s, ACCORD_ERR_STATE, "accord_ready_set_mode needs a registered-status store (resident, ACCORD_WINDOW_NONE)");
    if (s->rdy_waiting) return fail(s, ACCORD_ERR_STATE, "accord_ready_set_mode with txns in the waiting set");
    s->rdy_event_mode = mode == ACCORD_READY_EVENTS;
    return ACCORD_OK;
}

extern "C" int32_t accord_ready_update(accord_store *s, accord_ready *out)
{
    if (!s || !out) return fail(s, ACCORD_ERR_ARG, "null argument");
    if (!accord_impl::registered_mode(s))
        return fail(s, ACCORD_ERR_STATE, "accord_ready_update needs a registered-status store (resident, ACCORD_WINDOW_NONE)");
    out->n = 0;
    out->txn = nullptr;
    out->eal_msb = out->eal_lsb = nullptr;
    out->eal_node = nullptr;
    out->waiting = s->rdy_waiting;
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    hipStream_t st = s->stream;
    const uint32_t nkeys = s->cfg.key_hi - s->cfg.key_lo, C = s->carry_n;
    uint64_t cap = 0;
    for (accord_impl::ReadyGen *r : s->rdy_gens) cap += r->left ? r->n : 0;
    s->rdy_list.clear();
    if (cap == 0) return ACCORD_OK;
    constexpr uint32_t PEEK = 1024;            // ready records read back with the count in one copy
    constexpr uint32_t RW = sizeof(ReadyOut) / 4;
    HIPCHECK(s, s->rdy_sum.ensure((size_t)nkeys * sizeof(KeySummary) + 64));
    {   // header, ready records [cap], dropped [cap]; a reallocation (even at the same address) holds
        // no zeroed header, so the skip below must not trust the cached pointer after one
        const size_t out_cap = s->rdy_out.cap;
        const void *out_p = s->rdy_out.p;
        HIPCHECK(s, s->rdy_out.ensure(cap * (4 * RW + 4) + 512));
        if (s->rdy_out.cap != out_cap || s->rdy_out.p != out_p) s->rdy_hdr_zero = nullptr;
    }
    HIPCHECK(s, s->rdy_spill.ensure(cap * 4 + 64));              // txns left to the removal spill pass
    const uint32_t ngens = (uint32_t)s->rdy_gens.size();
    const uint32_t nl = (ngens + RD_GENS - 1) / RD_GENS;
    HIPCHECK(s, s->rdy_launch.ensure((size_t)std::max(1u, nl) * sizeof(ReadyLaunch)));
    if (!s->rdy_host) {
        HIPCHECK(s, hipHostMalloc(&s->rdy_host, (PEEK * RW + 64) * 4, hipHostMallocDefault));
    }
    constexpr uint32_t HDR = 64;               // rdy_out header words: ready count, dirty keys, work counts
    if (s->rdy_hdr_zero != s->rdy_out.p) HIPCHECK(s, hipMemsetAsync(s->rdy_out.p, 0, HDR * 4, st));
    s->rdy_hdr_zero = nullptr;                 // until this call has read its header back
    // setAppliedAndPropagate's tables: every position of the store, and a pool for the
    // appliedOrInvalidated of every waiting txn (bounded by its RangeDeps txnIds); the pool's fill
    // count rides in the header (cnt[HDR - 5]) and comes back with it
    uint64_t rv_live = 0;                      // no range deps waiting: nothing to save or propagate
    for (accord_impl::ReadyGen *r : s->rdy_gens) rv_live += r->left ? r->rvals : 0;
    const bool pv_on = rv_live > 0;
    if (pv_on) {
        const uint64_t pool_need = s->rdy_pv_n + rv_live;
        const size_t pos_need = (size_t)s->next_global + s->n + 1;
        HIPCHECK(s, accord_impl::grow_keep(s->rdy_pv_at, s->rdy_pv_pos * 4, pos_need * 4, st));
        HIPCHECK(s, accord_impl::grow_keep(s->rdy_pv_len, s->rdy_pv_pos * 4, pos_need * 4, st));
        s->rdy_pv_pos = std::min(s->rdy_pv_at.cap, s->rdy_pv_len.cap) / 4;
        HIPCHECK(s, accord_impl::grow_keep(s->rdy_pv_pool, (size_t)s->rdy_pv_n * 4, pool_need * 4 + 4, st));
        if (pool_need >= (1ull << 32)) return fail(s, ACCORD_ERR_CAPACITY, "appliedOrInvalidated pool exceeds 2^32 entries");
        HIPCHECK(s, hipMemsetD32Async((hipDeviceptr_t)(s->rdy_out.as<uint32_t>() + (HDR - 5)), (int)s->rdy_pv_n, 1, st));
    }
    // everything is re-evaluated after a new carry (batch, truncation) or RedundantBefore bound
    // (and after a call that failed part-way: its bookkeeping below may be ahead of the device)
    const bool force = s->rdy_force_full;
    // (event-exact mode too: a key bit its events cleared stamps the waiter changed, ev_clear)
    const bool full = force || s->rdy_kb_dirty || s->rdy_sum_version != s->carry_version;
    const uint32_t seen = s->rdy_seen, call = ++s->rdy_call;
    s->rdy_force_full = true;                  // cleared once this call has synchronised
    s->rdy_seen = s->rg_epoch;
    s->rdy_sum_version = s->carry_version;
    const uint32_t *kbp = nullptr;
    EV_RC(accord_impl::store_kb(s, force, &kbp));
    const StatusView v = accord_impl::store_view(s);
    HIPCHECK(s, s->rdy_part.ensure((size_t)C * sizeof(KeyPart) + 64));
    HIPCHECK(s, s->rdy_dirty.ensure_zeroed((size_t)nkeys * 4 + 4, st));
    HIPCHECK(s, s->rdy_dirty2.ensure_zeroed((size_t)nkeys * 4 + 4, st));
    HIPCHECK(s, s->rdy_dlist.ensure((size_t)nkeys * 4 + 4));
    // cnt[0]: ready txns, cnt[1]: dirty keys, cnt[2 ..]: work counts, cnt[HDR - 5]: pool fill,
    // cnt[HDR - 4 .. HDR - 2]: spill, cnt[HDR - 1]: dropped txns
    uint32_t *cnt = s->rdy_out.as<uint32_t>();
    ReadyOut *list = (ReadyOut *)(cnt + HDR);
    uint32_t *drop = (uint32_t *)(list + cap);
    DirtyMark dm{};
    if (!full) {
        dm.chg = s->rg_chg.as<uint32_t>(); dm.cchg = s->rg_cchg.as<uint32_t>(); dm.seen = seen; dm.call = call;
        dm.dirty = s->rdy_dirty.as<uint32_t>(); dm.list = s->rdy_dlist.as<uint32_t>(); dm.cnt = cnt + 1;
        dm.eval = s->rdy_dirty2.as<uint32_t>();
    }
    if (C) hipLaunchKernelGGL(rd_part_kernel, dim3(grid_for_waves((C + 63) / 64)), dim3(256), 0, st, C,
                              s->cy_key.as<uint32_t>(), s->cy_ent.as<uint32_t>(), v, s->rdy_part.as<KeyPart>(), dm);
    EV_RC(accord_impl::store_kseg(s, force));
    if (nkeys) hipLaunchKernelGGL(rd_summary_kernel, dim3(full ? grid_for_waves(nkeys) : std::min(grid_for_waves(nkeys), 256u)),
                                  dim3(256), 0, st, nkeys, s->rdy_kseg0.as<uint32_t>(), s->rdy_kseg1.as<uint32_t>(),
                                  s->rdy_part.as<KeyPart>(), v, s->rdy_sum.as<KeySummary>(),
                                  full ? nullptr : s->rdy_dlist.as<uint32_t>(), cnt + 1, s->rdy_dirty2.as<uint32_t>(), call);
    // the generations with txns left, RD_GENS per launch (their parameter table copied to the device)
    std::vector<ReadyLaunch> tabs;
    bool any_inc = false;
    for (accord_impl::ReadyGen *r : s->rdy_gens) {
        if (r->left == 0) continue;
        if (tabs.empty() || tabs.back().ngen == RD_GENS) {
            const uint32_t b = tabs.empty() ? 0u : tabs.back().base + tabs.back().total;
            tabs.emplace_back();
            tabs.back().ngen = 0; tabs.back().total = 0; tabs.back().base = b;
        }
        ReadyLaunch &L = tabs.back();
        ReadyParams &p = L.g[L.ngen];
        p = accord_impl::gen_params(s, r, v, kbp);
        p.evmode = s->rdy_event_mode ? 1u : 0u;
        p.out = list; p.out_cnt = cnt;
        p.drop = drop; p.drop_cnt = cnt + (HDR - 1);
        p.inv = cnt + (HDR - 6);
        p.rbx = s->rb_ext && s->rb_m ? 1u : 0u;
        p.M = rr_map_of(s);
        p.pkoff = r->pkoff.as<uint32_t>(); p.pkeys = r->pkeys.as<uint32_t>();
        p.proff = r->proff.as<uint32_t>(); p.prs = r->prs.as<uint32_t>(); p.pre = r->pre.as<uint32_t>();
        p.rrng_off = r->rrng_off.as<uint32_t>(); p.rrs = r->rrs.as<uint32_t>(); p.rre = r->rre.as<uint32_t>();
        p.rr2v_off = r->rr2v_off.as<uint32_t>(); p.rr2v = r->rr2v.as<uint32_t>();
        p.spill = RrSpill{cnt + (HDR - 2), cnt + (HDR - 3), cnt + (HDR - 4), s->rdy_spill.as<uint32_t>()};
        p.ubase = L.base;
        p.sum = s->rdy_sum.as<KeySummary>();
        p.full = r->fresh ? 1u : 0u;
        any_inc |= !full && !r->fresh;
        p.chg = s->rg_chg.as<uint32_t>(); p.dirty = s->rdy_dirty2.as<uint32_t>();
        if (pv_on) {
            p.pv_at = s->rdy_pv_at.as<uint32_t>(); p.pv_len = s->rdy_pv_len.as<uint32_t>();
            p.pv_pool = s->rdy_pv_pool.as<uint32_t>(); p.pv_cnt = cnt + (HDR - 5);
        }
        r->fresh = false;
        L.gbase[L.ngen] = L.total;
        L.total += r->n;
        L.gbase[++L.ngen] = L.total;
    }
    if (any_inc) {          // a work list per launch: cap entries, counts in rdy_wcnt
        HIPCHECK(s, s->rdy_work.ensure(cap * 4 + 64));
        uint32_t *wc = cnt + 2;                // in the header (cleared above) unless too many launches
        if (tabs.size() > HDR - 8) {
            HIPCHECK(s, s->rdy_wcnt.ensure(tabs.size() * 4 + 64));
            HIPCHECK(s, hipMemsetAsync(s->rdy_wcnt.p, 0, tabs.size() * 4, st));
            wc = s->rdy_wcnt.as<uint32_t>();
        }
        uint64_t off = 0;
        for (size_t i = 0; i < tabs.size(); ++i) {
            tabs[i].work = s->rdy_work.as<uint32_t>() + off;
            tabs[i].wcnt = wc + i;
            off += tabs[i].total;
        }
    }
    HIPCHECK(s, s->rdy_launch.ensure(tabs.size() * sizeof(ReadyLaunch)));
    const size_t tab_bytes = tabs.size() * sizeof(ReadyLaunch);
    if (s->rdy_tab_cap < tab_bytes) {          // pinned staging for the tables (the call ends synchronised)
        if (s->rdy_tab_host) (void)hipHostFree(s->rdy_tab_host);
        s->rdy_tab_host = nullptr; s->rdy_tab_cap = 0;
        HIPCHECK(s, hipHostMalloc(&s->rdy_tab_host, tab_bytes * 2, hipHostMallocDefault));
        s->rdy_tab_cap = tab_bytes * 2;
    }
    // the tables change only when the generations or the buffers they point at do (the per-call
    // epoch and id go to the filter as arguments): re-sent only then
    // (and after a call that failed part-way: force)
    if (force || s->rdy_tab_last.size() != tab_bytes || s->rdy_tab_dev != s->rdy_launch.p ||
        std::memcmp(s->rdy_tab_last.data(), tabs.data(), tab_bytes) != 0) {
        std::memcpy(s->rdy_tab_host, tabs.data(), tab_bytes);
        HIPCHECK(s, hipMemcpyAsync(s->rdy_launch.p, s->rdy_tab_host, tab_bytes, hipMemcpyHostToDevice, st));
        s->rdy_tab_last.assign((const uint8_t *)tabs.data(), (const uint8_t *)tabs.data() + tab_bytes);
        s->rdy_tab_dev = s->rdy_launch.p;
    }
    const size_t rr_lds = s->rb_ext && s->rb_m ? 4 * sizeof(RrLds) : 0;   // removal scratch, a wave each
    // (evaluating every txn of an incremental call instead of the filtered ones measured slower even
    // at 8 k waiting txns: 23-42 us against 13 + 6 us, profiles/r05_ready)
    for (size_t i = 0; i < tabs.size(); ++i) {
        const ReadyLaunch *L = s->rdy_launch.as<ReadyLaunch>() + i;
        if (any_inc) {
            hipLaunchKernelGGL(rd_filter_kernel, dim3(((uint64_t)tabs[i].total * RF_LANES + 255) / 256), dim3(256), 0, st, L,
                               seen, call, full ? 1u : 0u);
            hipLaunchKernelGGL(rd_eval_kernel, dim3(std::min(grid_for_waves(tabs[i].total), 1024u)), dim3(256), rr_lds, st, L, 1u);
        } else {
            hipLaunchKernelGGL(rd_eval_kernel, dim3(grid_for_waves(tabs[i].total)), dim3(256), rr_lds, st, L, 0u);
        }
    }
    uint32_t *peek = (uint32_t *)s->rdy_host;
    {
        void *peek_dev = nullptr;
        HIPCHECK(s, hipHostGetDevicePointer(&peek_dev, peek, 0));
        hipLaunchKernelGGL(rd_host_out_kernel, dim3(1), dim3(256), 0, st, cnt, (uint32_t *)peek_dev, HDR, RW,
                           (uint32_t)std::min<uint64_t>(cap, PEEK));
    }
    HIPCHECK(s, hipGetLastError());
    if (!s->rdy_stats && getenv("ACCORD_READY_STATS")) s->rdy_stats = new uint64_t[4]{0, 0, 0, 0};
    HIPCHECK(s, hipStreamSynchronize(st));       // the header is in peek; the parameter tables were consumed
    if (!peek[HDR - 2]) s->rdy_hdr_zero = s->rdy_out.p;   // rd_host_out_kernel zeroed it
    if (peek[HDR - 2]) {    // txns over the LDS removal scratch: the spill pass, then the header again
        const uint32_t nsp = peek[HDR - 2], blocks = std::min<uint32_t>((nsp + 3) / 4, 64u);
        HIPCHECK(s, s->rdy_spill_mem.ensure((size_t)blocks * 4 * rr_spill_wave_bytes(peek[HDR - 3], peek[HDR - 4])));
        const RrSpill sp{cnt + (HDR - 2), cnt + (HDR - 3), cnt + (HDR - 4), s->rdy_spill.as<uint32_t>()};
        hipLaunchKernelGGL(rd_spill_kernel, dim3(blocks), dim3(256), 0, st, s->rdy_launch.as<ReadyLaunch>(),
                           (uint32_t)tabs.size(), sp, s->rdy_spill_mem.p, peek[HDR - 3], peek[HDR - 4]);
        HIPCHECK(s, hipGetLastError());
        HIPCHECK(s, hipMemcpyAsync(peek, cnt, (HDR + std::min<uint64_t>(cap, PEEK) * RW) * 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(s, hipStreamSynchronize(st));
    }
    const uint32_t nr = peek[0], nd = peek[HDR - 1];
    if (pv_on) s->rdy_pv_n = peek[HDR - 5];
    if (peek[HDR - 6])
        return fail(s, ACCORD_ERR_STATE, "Invariants.checkState: txn %u waits on a TruncatedApply dep executing at or "
                    "after it (local/Commands.java:789-791)", peek[HDR - 6] - 1u);
    if (s->rdy_stats) {                          // ACCORD_READY_STATS: diagnostic totals (ready_destroy prints)
        s->rdy_stats[0] += 1; s->rdy_stats[1] += peek[1]; s->rdy_stats[2] += cap;
        if (any_inc && tabs.size() <= HDR - 8)
            for (size_t i = 0; i < tabs.size(); ++i) s->rdy_stats[3] += peek[2 + i];
        else s->rdy_stats[3] += cap;
    }
    s->rdy_list.resize(nr);
    s->rdy_eal_msb.resize(nr); s->rdy_eal_lsb.resize(nr); s->rdy_eal_node.resize(nr);
    if (nr) {
        std::vector<ReadyOut> recs(nr);
        if (nr <= PEEK) {
            std::memcpy(recs.data(), peek + HDR, (size_t)nr * sizeof(ReadyOut));
        } else {
            HIPCHECK(s, hipMemcpyAsync(recs.data(), list, (size_t)nr * sizeof(ReadyOut), hipMemcpyDeviceToHost, st));
            HIPCHECK(s, hipStreamSynchronize(st));
        }
        std::sort(recs.begin(), recs.end(), [](const ReadyOut &a, const ReadyOut &b) { return a.g < b.g; });
        for (uint32_t i = 0; i < nr; ++i) {
            s->rdy_list[i] = recs[i].g;
            s->rdy_eal_msb[i] = recs[i].msb; s->rdy_eal_lsb[i] = recs[i].lsb; s->rdy_eal_node[i] = recs[i].node;
        }
    }
    std::vector<uint32_t> dropped(nd);
    if (nd) {
        HIPCHECK(s, hipMemcpyAsync(dropped.data(), drop, (size_t)nd * 4, hipMemcpyDeviceToHost, st));
        HIPCHECK(s, hipStreamSynchronize(st));
        std::sort(dropped.begin(), dropped.end());
    }
    s->rdy_force_full = false;                 // the device and the bookkeeping below agree again
    // generations drain in stream order: count each one's released (or dropped) txns, free the empty ones
    auto settle = [&](const std::vector<uint32_t> &l) {
        size_t a = 0;
        for (accord_impl::ReadyGen *r : s->rdy_gens) {
            uint32_t c = 0;
            while (a < l.size() && l[a] <= r->ghi) { c += l[a] >= r->glo; ++a; }
            r->left -= c;
        }
    };
    settle(s->rdy_list);
    settle(dropped);
    std::vector<accord_impl::ReadyGen *> keep;
    for (accord_impl::ReadyGen *r : s->rdy_gens) {
        if (r->left == 0) {
            if (r == s->rdy_batch_gen) s->rdy_batch_gen = nullptr;
            r->release();
            delete r;
        }
        else keep.push_back(r);
    }
    s->rdy_gens.swap(keep);
    s->rdy_waiting -= (uint64_t)nr + nd;
    out->n = nr;
    out->txn = s->rdy_list.data();
    out->eal_msb = s->rdy_eal_msb.data(); out->eal_lsb = s->rdy_eal_lsb.data(); out->eal_node = s->rdy_eal_node.data();
    out->waiting = s->rdy_waiting;
    return ACCORD_OK;
}
