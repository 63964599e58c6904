// Real status events for a resident store (SURVEY.md §8a a4, §8b accord_txn_register, §8f row 1).
//
// A store created with ACCORD_STORE_RESIDENT and window ACCORD_WINDOW_NONE has no status-at-time
// model: a txn enters its keys' CommandsForKey PREACCEPTED when its batch is computed and keeps that
// status until accord_txn_register reports another (CommandsForKey.update, local/CommandsForKey.java:
// 652-706).  The store holds, per global position, the txn's InternalStatus and executeAt, and a
// TxnId-sorted table to find a txn by TxnId.
//
// Deps of a (txn, key) pair whose key history holds an entry with a registered status follow the
// general mapReduceActive (:614-650) instead of the contiguous-slice fast path:
//   maxCommittedBefore = max executeAt over COMMITTED/STABLE/APPLIED Writes with executeAt <
//                        startedBefore (the committed[] search of :620-624; executeAt >= TxnId, so
//                        only entries before the pair's bound can qualify)
//   emitted            = entries before the bound whose kind is witnessed, not TRANSITIVELY_KNOWN /
//                        INVALID_OR_TRUNCATED, and (if committed) executeAt >= maxCommittedBefore
// The emitted entries of every such pair are written to an extension of the history array and the
// pair's slice is pointed at them, so the fill kernels are unchanged.
// Between batches an entry leaves the resident state when its txn is INVALID_OR_TRUNCATED (a
// truncated committed Write no longer bounds maxCommittedBefore, so nothing else can be dropped
// without knowing the future events).
#include "store_impl.h"
#include "status_view.h"
#include "redundant_wait.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

using namespace accord_status;

using accord::RC_KIND_ERASED;

__device__ __forceinline__ void record_error(accord::DevStatus *st, uint32_t i, int32_t code)
{
    unsigned long long v = ((unsigned long long)i << 32) | (uint32_t)(-code);
    atomicMin(&st->first, v);
}

// keys whose carried history holds a txn with a registered status
struct GenParams {
    uint32_t n, key_lo;
    const uint64_t *msb, *lsb;
    const int32_t *node;
    const uint64_t *xmsb, *xlsb;      // Accept batch executeAt (nullptr: startedBefore = TxnId)
    const int32_t *xnode;
    const uint32_t *key_off, *key_ord, *txn_index, *flag, *hist;
    accord::PairSlice *slice;
    uint32_t *gcnt;
    const uint32_t *goff;
    uint32_t *hist2;
    uint32_t ext_base;                // first extension position of hist2
    StatusView v;
    // committed[] index of the Writes (cw_*): cw_off[x] = committed Writes before history position x,
    // cw_pos[j] = the j-th one's position, cw_pm[j] = the one with the latest executeAt among its key's
    // up to j (CommandsForKey.committed, local/CommandsForKey.java:462-469)
    const uint32_t *cw_off, *cw_pos, *cw_pm;
    // per history position (hx_*): hx = the committed entry of [key's first entry, x] executing last
    // (NONE: none), hu = the uncommitted entries there; skey = each position's key
    const uint32_t *hx, *hu, *skey;
    const uint32_t *abort;            // speculative fill (store.cpp): the extension would not fit
};

// One pair, one wave (lanes stride over the pair's slice [lo, pos) of the key's history):
//   maxCommittedBefore = max executeAt over committed Writes with executeAt < startedBefore (:620-624)
//   emitted            = witnessed entries, not TRANSITIVELY_KNOWN / INVALID_OR_TRUNCATED, committed
//                        ones only with executeAt >= maxCommittedBefore (:634-645); p1 excluded
// Count pass: when the emitted entries are exactly the witnessed entries of [first emitted, pos) --
// the common case once the carried history is pruned -- the pair's slice is narrowed to that range of
// the history itself (the fill kernels filter by kind and drop the txn itself); otherwise its count
// reserves an extension run that the fill pass writes.
template <bool FILL>
__device__ void general_pair(const GenParams &p, uint32_t t, uint32_t q, uint32_t lane)
{
    const accord::PairSlice sl = p.slice[q];
    const uint64_t l = p.lsb[t];
    const uint32_t wmask = witness_mask((uint32_t)(l >> 1) & 7);
    Ts sb{p.msb[t], l, p.node[t]};
    bool p1 = false;    // p1 = executeAt.equals(txnId) ? null : txnId (messages/PreAccept.java:259)
    if (p.xmsb) {
        const Ts x{p.xmsb[t], p.xlsb[t], p.xnode[t]};
        p1 = !(x.msb == sb.msb && ((x.lsb ^ sb.lsb) & 0xFFFFFFFFFFFF001Eull) == 0 && x.node == sb.node);
        sb = x;
    }
    const uint32_t self = p.txn_index[t];
    const uint32_t lo = sl.lo, hi = sl.pos;
    // maxCommittedBefore (:620-624): the latest executeAt before startedBefore among the key's committed
    // Writes before the bound, walked back from the last one; the running argmax (cw_pm) ends the walk
    // as soon as no earlier Write can beat the best found (usually the first step: executeAts follow
    // TxnId order but for the few still executing after startedBefore)
    bool has_mcb = false;
    Ts mcb{0, 0, 0};
    for (uint32_t j = p.cw_off[hi], j0 = p.cw_off[lo]; j > j0; --j) {   // wave-uniform
        const Ts best = exec_of(p.v, p.hist[p.cw_pos[p.cw_pm[j - 1]]] & ENT_TXN_MASK);
        if (has_mcb && tcmp(best, mcb) <= 0) break;
        if (tcmp(best, sb) < 0) { mcb = best; has_mcb = true; break; }
        const Ts ex = exec_of(p.v, p.hist[p.cw_pos[j - 1]] & ENT_TXN_MASK);
        if (tcmp(ex, sb) < 0 && (!has_mcb || tcmp(ex, mcb) > 0)) { mcb = ex; has_mcb = true; }
    }
    // what the fill kernels keep of a history entry (kind witnessed, not the txn itself)
    auto witnessed = [&](uint32_t e) { return ((wmask >> (e >> ENT_KIND_SHIFT)) & 1u) && (e & ENT_TXN_MASK) != self; };
    auto emitted = [&](uint32_t e) -> bool {
        if (!((wmask >> (e >> ENT_KIND_SHIFT)) & 1u)) return false;
        const uint32_t g = e & ENT_TXN_MASK;
        if (p1 && g == self) return false;
        const uint32_t st = status_of(p.v, g);
        if (st == ST_TK || st >= ST_INVALID) return false;
        return !(committed(st) && has_mcb && tcmp(exec_of(p.v, g), mcb) < 0);
    };
    if (!FILL) {
        // skip the prefix [lo, F) of the slice whose committed entries all execute before
        // maxCommittedBefore and that holds no uncommitted entry: nothing in it is emitted.  F = the
        // first position whose running latest-executing committed entry reaches maxCommittedBefore
        // (monotone), found by a 64-way search.
        uint32_t start = lo;
        if (has_mcb && p.hx && hi > lo) {
            uint32_t L = lo, H = hi;
            while (L < H) {                                            // wave-uniform
                const uint32_t step = (H - L + 63u) / 64u, y = L + lane * step;
                bool reach = false;
                if (y < H) {
                    const uint32_t m = p.hx[y];
                    reach = m != 0xFFFFFFFFu && tcmp(exec_of(p.v, p.hist[m] & ENT_TXN_MASK), mcb) >= 0;
                }
                const uint64_t bm = __ballot(reach);
                if (bm == 0ull) {
                    const uint64_t live = __ballot(y < H);
                    L = L + (63u - (uint32_t)__builtin_clzll(live)) * step + 1u;
                } else {
                    const uint32_t f = (uint32_t)__builtin_ctzll(bm);
                    H = L + f * step;
                    if (f) L = L + (f - 1u) * step + 1u;
                }
            }
            if (L > lo) {
                const uint32_t u = p.hu[L - 1] - ((lo > 0 && p.skey[lo - 1] == p.skey[lo]) ? p.hu[lo - 1] : 0u);
                if (u == 0) start = L;
            }
        }
        // emitted count, first emitted position, last witnessed-but-not-emitted position
        uint32_t c = 0, first = hi, last_rej = 0;
        bool any_rej = false;
        for (uint32_t x = start + lane; x < hi; x += 64) {
            const uint32_t e = p.hist[x];
            if (emitted(e)) { ++c; first = min(first, x); }
            else if (witnessed(e)) { any_rej = true; last_rej = max(last_rej, x); }
        }
        c = wave_sum(c);
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) first = min(first, (uint32_t)__shfl_xor((int)first, d, 64));
        const bool rej = __any(any_rej && last_rej > first);      // first is wave-uniform here
        if (lane == 0) {
            if (!rej) {   // contiguous: the fill reads the history range itself
                p.slice[q] = accord::PairSlice{c ? first : hi, hi, c, sl.key};
                p.gcnt[q] = 0;
            } else {      // the count now (the sizes pass reads it), the range until the emit pass
                p.slice[q] = accord::PairSlice{lo, hi, c, sl.key};
                p.gcnt[q] = c;
            }
        }
        return;
    }
    // fill (pairs with an extension run only): the emitted entries, in order
    const uint64_t lt = lanemask_lt();
    const uint32_t out = p.ext_base + p.goff[q];
    uint32_t c = 0;
    for (uint32_t x0 = lo; x0 < hi; x0 += 64) {
        const uint32_t x = x0 + lane;
        const bool em = x < hi && emitted(p.hist[x]);
        const uint64_t b = __ballot(em);
        if (em) p.hist2[out + c + (uint32_t)__popcll(b & lt)] = p.hist[x];
        c += (uint32_t)__popcll(b);
    }
    if (lane == 0) p.slice[q] = accord::PairSlice{out, out + c, c, sl.key};
}

// committed[] index of the Writes (see GenParams): flags and positions (gen_pre_kernel / gen_mid_kernel),
// running argmax by executeAt
// cw_pm[j] = the argmax by executeAt over the key's committed Writes up to j (ties: the later one;
// executeAts are unique), as a segmented scan over the index in two passes so a hot key's long run
// spreads over many waves:
// cw_local_kernel -- a wave per 64 index entries: the running argmax inside the chunk, restarting at
//   key changes (keys ascend along the index); per chunk {first key, last key, argmax of its
//   trailing run};
// cw_carry_kernel -- a wave per chunk whose first run continues the previous chunk's last one: the
//   argmax over the run's earlier chunks (their trailing-run argmaxes, 64 chunks per step) merged
//   into the chunk's first run.
__device__ __forceinline__ uint32_t cw_total(uint32_t PH, const uint32_t *flag, const uint32_t *off)
{
    return PH ? off[PH - 1] + flag[PH - 1] : 0u;
}

__device__ __forceinline__ bool cw_better(uint32_t a, const Ts &ea, uint32_t b, const Ts &eb)
{
    if (a == 0xFFFFFFFFu) return false;
    if (b == 0xFFFFFFFFu) return true;
    const int c = tcmp(ea, eb);
    return c > 0 || (c == 0 && a > b);
}

__global__ __launch_bounds__(256) void cw_local_kernel(uint32_t PH, const uint32_t *__restrict__ flag,
                                                       const uint32_t *__restrict__ off, const uint32_t *__restrict__ pos,
                                                       const uint32_t *__restrict__ hist, const uint32_t *__restrict__ skey,
                                                       StatusView v, uint32_t *__restrict__ pm, uint4 *__restrict__ chunk)
{
    const uint32_t J = cw_total(PH, flag, off);
    const uint32_t lane = lane_id(), waves = gridDim.x * (blockDim.x / 64);
    for (uint32_t c0 = (blockIdx.x * (blockDim.x / 64) + wave_id()) * 64u; c0 < J; c0 += waves * 64u) {
        const uint32_t j = c0 + lane;
        const bool valid = j < J;
        const uint32_t x = valid ? pos[j] : 0u;
        const uint32_t key = valid ? skey[x] : 0xFFFFFFFFu;
        uint32_t m = valid ? j : 0xFFFFFFFFu;
        Ts ex = valid ? exec_of(v, hist[x] & ENT_TXN_MASK) : Ts{0, 0, 0};
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t om = (uint32_t)__shfl_up((int)m, d, 64), ok = (uint32_t)__shfl_up((int)key, d, 64);
            const Ts oe{(uint64_t)__shfl_up((long long)ex.msb, d, 64), (uint64_t)__shfl_up((long long)ex.lsb, d, 64),
                        __shfl_up(ex.node, d, 64)};
            if (lane >= (uint32_t)d && ok == key && cw_better(om, oe, m, ex)) { m = om; ex = oe; }
        }
        if (valid) pm[j] = m;
        const int last = (int)min(63u, J - 1u - c0);
        const uint32_t kl = readlane(key, last), ml = readlane(m, last), kf = readlane(key, 0);
        if (lane == 0) chunk[c0 >> 6] = make_uint4(kf, kl, ml, 0u);
    }
}

__global__ __launch_bounds__(256) void cw_carry_kernel(uint32_t PH, const uint32_t *__restrict__ flag,
                                                       const uint32_t *__restrict__ off, const uint32_t *__restrict__ pos,
                                                       const uint32_t *__restrict__ hist, const uint32_t *__restrict__ skey,
                                                       StatusView v, const uint4 *__restrict__ chunk,
                                                       uint32_t *__restrict__ pm)
{
    const uint32_t J = cw_total(PH, flag, off), nch = (J + 63u) / 64u;
    const uint32_t lane = lane_id(), waves = gridDim.x * (blockDim.x / 64);
    for (uint32_t c = blockIdx.x * (blockDim.x / 64) + wave_id(); c < nch; c += waves) {
        const uint32_t kf = chunk[c].x;
        if (c == 0 || chunk[c - 1].y != kf) continue;             // wave-uniform: the run starts here
        uint32_t best = 0xFFFFFFFFu;
        Ts bex{0, 0, 0};
        for (uint32_t top = c; top > 0; top = top > 64u ? top - 64u : 0u) {   // chunks top-1 .. top-64
            const bool in = lane < top;
            const uint4 q = in ? chunk[top - 1 - lane] : make_uint4(0u, 0u, 0u, 0u);
            const bool same = in && q.y == kf;                       // its trailing run is this key's
            const bool stop = !same || q.x != kf;                    // ... and the run starts inside it
            const unsigned long long sm = __ballot(stop);
            const uint32_t first = sm ? (uint32_t)__builtin_ctzll(sm) : 64u;
            if ((lane < first || lane == first) && same) {
                const Ts e = exec_of(v, hist[pos[q.z]] & ENT_TXN_MASK);
                if (cw_better(q.z, e, best, bex)) { best = q.z; bex = e; }
            }
            if (sm) break;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t ob = (uint32_t)__shfl_xor((int)best, d, 64);
            const Ts oe{(uint64_t)__shfl_xor((long long)bex.msb, d, 64), (uint64_t)__shfl_xor((long long)bex.lsb, d, 64),
                        __shfl_xor(bex.node, d, 64)};
            if (cw_better(ob, oe, best, bex)) { best = ob; bex = oe; }
        }
        const uint32_t j = c * 64u + lane;
        if (best != 0xFFFFFFFFu && j < J && skey[pos[j]] == kf) {    // the chunk's first run
            const uint32_t m = pm[j];
            if (cw_better(best, bex, m, exec_of(v, hist[pos[m]] & ENT_TXN_MASK))) pm[j] = best;
        }
    }
}

// hx / hu (GenParams) in the same two passes as cw_pm: chunk-local segmented scans, then the
// carries of runs crossing chunks.  chunk = {first key, last key, hx of the trailing run, hu of it}.
__device__ __forceinline__ void hx_local_chunk(uint32_t PH, const uint32_t *__restrict__ hist,
                                               const uint32_t *__restrict__ skey, const StatusView &v,
                                               uint32_t *__restrict__ hx, uint32_t *__restrict__ hu,
                                               uint4 *__restrict__ chunk, uint32_t c0, uint32_t lane)
{
    {
        const uint32_t x = c0 + lane;
        const bool valid = x < PH;
        const uint32_t key = valid ? skey[x] : 0xFFFFFFFFu;
        const uint32_t g = valid ? hist[x] & ENT_TXN_MASK : 0u, st = valid ? status_of(v, g) : ST_INVALID;
        uint32_t m = valid && committed(st) ? x : 0xFFFFFFFFu;
        uint32_t u = valid && st < ST_COMMITTED ? 1u : 0u;
        Ts ex = m != 0xFFFFFFFFu ? exec_of(v, g) : Ts{0, 0, 0};
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t om = (uint32_t)__shfl_up((int)m, d, 64), ok = (uint32_t)__shfl_up((int)key, d, 64);
            const uint32_t ou = (uint32_t)__shfl_up((int)u, d, 64);
            const Ts oe{(uint64_t)__shfl_up((long long)ex.msb, d, 64), (uint64_t)__shfl_up((long long)ex.lsb, d, 64),
                        __shfl_up(ex.node, d, 64)};
            if (lane >= (uint32_t)d && ok == key) {
                u += ou;
                if (cw_better(om, oe, m, ex)) { m = om; ex = oe; }
            }
        }
        if (valid) { hx[x] = m; hu[x] = u; }
        const int last = (int)min(63u, PH - 1u - c0);
        const uint32_t kl = readlane(key, last), ml = readlane(m, last), ul = readlane(u, last), kf = readlane(key, 0);
        if (lane == 0) chunk[c0 >> 6] = make_uint4(kf, kl, ml, ul);
    }
}

__device__ __forceinline__ void hx_carry_chunk(uint32_t PH, const uint32_t *__restrict__ hist,
                                               const uint32_t *__restrict__ skey, const StatusView &v,
                                               const uint4 *__restrict__ chunk, uint32_t *__restrict__ hx,
                                               uint32_t *__restrict__ hu, uint32_t c, uint32_t lane)
{
    {
        const uint32_t kf = chunk[c].x;
        if (c == 0 || chunk[c - 1].y != kf) return;               // wave-uniform: the run starts here
        uint32_t best = 0xFFFFFFFFu, cnt = 0;
        Ts bex{0, 0, 0};
        for (uint32_t top = c; top > 0; top = top > 64u ? top - 64u : 0u) {
            const bool in = lane < top;
            const uint4 q = in ? chunk[top - 1 - lane] : make_uint4(0u, 0u, 0u, 0u);
            const bool same = in && q.y == kf;
            const bool stop = !same || q.x != kf;
            const unsigned long long sm = __ballot(stop);
            const uint32_t first = sm ? (uint32_t)__builtin_ctzll(sm) : 64u;
            if (lane <= first && same) {
                cnt += q.w;
                if (q.z != 0xFFFFFFFFu) {
                    const Ts e = exec_of(v, hist[q.z] & ENT_TXN_MASK);
                    if (cw_better(q.z, e, best, bex)) { best = q.z; bex = e; }
                }
            }
            if (sm) break;
        }
        cnt = wave_sum(cnt);
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t ob = (uint32_t)__shfl_xor((int)best, d, 64);
            const Ts oe{(uint64_t)__shfl_xor((long long)bex.msb, d, 64), (uint64_t)__shfl_xor((long long)bex.lsb, d, 64),
                        __shfl_xor(bex.node, d, 64)};
            if (cw_better(ob, oe, best, bex)) { best = ob; bex = oe; }
        }
        const uint32_t x = c * 64u + lane;
        if (x < PH && skey[x] == kf) {                                // the chunk's first run
            hu[x] += cnt;
            const uint32_t m = hx[x];
            if (best != 0xFFFFFFFFu &&
                cw_better(best, bex, m, m != 0xFFFFFFFFu ? exec_of(v, hist[m] & ENT_TXN_MASK) : Ts{0, 0, 0}))
                hx[x] = best;
        }
    }
}

// The committed[] index and hx / hu in three launches instead of eight: a wave per 64 items of
// each independent pass, the passes' wave ranges laid end to end in one grid.
//   gen_pre_kernel : carried keys' flags (flag_keys), the committed-Write flags (cw_flag), hx / hu
//                    chunk-local scans (hx_local)
//   (scan of the committed-Write flags)
//   gen_mid_kernel : the committed-Writes' positions (cw_scatter), hx / hu carries (hx_carry)
//   cw_local_kernel, cw_carry_kernel as before
__global__ __launch_bounds__(256) void gen_pre_kernel(uint32_t C, const uint32_t *__restrict__ ckey,
                                                      const uint32_t *__restrict__ cent, uint32_t PH,
                                                      const uint32_t *__restrict__ hist, const uint32_t *__restrict__ skey,
                                                      StatusView v, uint32_t *__restrict__ kflag, uint32_t *__restrict__ cwflag,
                                                      uint32_t *__restrict__ hx, uint32_t *__restrict__ hu,
                                                      uint4 *__restrict__ hxchunk)
{
    const uint32_t lane = lane_id(), waves = gridDim.x * (blockDim.x / 64);
    const uint32_t nC = (C + 63u) / 64u, nP = (PH + 63u) / 64u;
    for (uint32_t w = blockIdx.x * (blockDim.x / 64) + wave_id(); w < nC + 2u * nP; w += waves) {
        if (w < nC) {
            const uint32_t c = w * 64u + lane;
            if (c < C && status_of(v, cent[c] & ENT_TXN_MASK) != ST_PREACCEPTED) kflag[ckey[c]] = 1u;
        } else if (w < nC + nP) {
            const uint32_t x = (w - nC) * 64u + lane;
            if (x < PH) {
                const uint32_t e = hist[x];
                cwflag[x] = (e >> ENT_KIND_SHIFT) == 1u && committed(status_of(v, e & ENT_TXN_MASK)) ? 1u : 0u;
            }
        } else {
            hx_local_chunk(PH, hist, skey, v, hx, hu, hxchunk, (w - nC - nP) * 64u, lane);
        }
    }
}

__global__ __launch_bounds__(256) void gen_mid_kernel(uint32_t PH, const uint32_t *__restrict__ cwflag,
                                                      const uint32_t *__restrict__ cwoff, uint32_t *__restrict__ cwpos,
                                                      const uint32_t *__restrict__ hist, const uint32_t *__restrict__ skey,
                                                      StatusView v, const uint4 *__restrict__ hxchunk,
                                                      uint32_t *__restrict__ hx, uint32_t *__restrict__ hu)
{
    const uint32_t lane = lane_id(), waves = gridDim.x * (blockDim.x / 64);
    const uint32_t nP = (PH + 63u) / 64u;
    for (uint32_t w = blockIdx.x * (blockDim.x / 64) + wave_id(); w < 2u * nP; w += waves) {
        if (w < nP) {
            const uint32_t x = w * 64u + lane;
            if (x < PH && cwflag[x]) cwpos[cwoff[x]] = x;
        } else {
            hx_carry_chunk(PH, hist, skey, v, hxchunk, hx, hu, w - nP, lane);
        }
    }
}

// GEN_SPLIT waves per txn, each over every GEN_SPLIT-th of its keys that hold a registered status
// (a pair's walk is a chain of dependent loads: a small batch's txns run their pairs side by side --
// one wave per txn had taken 37 us per 1024-txn batch): the count pass narrows contiguous pairs'
// slices itself and counts the others, the fill pass writes the counted ones.
constexpr uint32_t GEN_SPLIT = 8;
template <bool FILL>
__global__ __launch_bounds__(256) void general_kernel(GenParams p)
{
    if (FILL && p.abort && *p.abort) return;
    if (FILL)       // the extended history starts as the batch history (a copy launch fewer)
        for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < p.ext_base; x += gridDim.x * blockDim.x)
            p.hist2[x] = p.hist[x];
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x / 64);
    const uint64_t total = (uint64_t)p.n * GEN_SPLIT;
    for (uint64_t w = blockIdx.x * (blockDim.x / 64) + wave_id(); w < total; w += waves) {
        const uint32_t t = (uint32_t)(w / GEN_SPLIT), k0 = (uint32_t)(w % GEN_SPLIT);
        for (uint32_t q = p.key_off[t] + k0; q < p.key_off[t + 1]; q += GEN_SPLIT) {
            if (!p.flag[p.key_ord[q] - p.key_lo]) { if (!FILL && lane == 0) p.gcnt[q] = 0; continue; }
            if (FILL && p.gcnt[q] == 0) continue;          // contiguous pair: slice already set
            general_pair<FILL>(p, t, q, lane);
        }
    }
}

// carry flags of a registered-status store: an entry stays until its txn is INVALID_OR_TRUNCATED
// (CommandsForKey skips those for good, local/CommandsForKey.java:436,643) or the store's
// RedundantBefore truncates it (status_truncate_carry); every other entry can still be emitted, or
// bound maxCommittedBefore, after later events
__global__ __launch_bounds__(256) void prune_mark_kernel(uint32_t P, const uint32_t *__restrict__ hist, StatusView v,
                                                         uint32_t *__restrict__ keep_flag)
{
    for (uint32_t x = blockIdx.x * blockDim.x + threadIdx.x; x < P; x += gridDim.x * blockDim.x)
        keep_flag[x] = status_of(v, hist[x] & ENT_TXN_MASK) < ST_INVALID ? 1u : 0u;
}

// CommandsForKey.withRedundantBefore (:1654-1684) on the carried history: entries below their key's
// shardRedundantBefore leave
// each carried entry's key bound from the store's RedundantBefore entries themselves (m ascending,
// disjoint (start, end] ranges; a binary search per entry instead of a per-key table uploaded from
// the host -- 400 KB per call at 100 k keys)
__global__ __launch_bounds__(256) void truncate_mark_kernel(uint32_t C, const uint32_t *__restrict__ ckey,
                                                            const uint32_t *__restrict__ cent, uint32_t key_lo,
                                                            uint32_t m, const uint32_t *__restrict__ rs,
                                                            const uint32_t *__restrict__ re,
                                                            const uint32_t *__restrict__ rbound,
                                                            uint32_t *__restrict__ keep_flag)
{
    for (uint32_t c = blockIdx.x * blockDim.x + threadIdx.x; c < C; c += gridDim.x * blockDim.x) {
        const uint32_t k = ckey[c] + key_lo;
        uint32_t lo = 0, hi = m;                       // first entry with end >= k
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (re[mid] < k) lo = mid + 1; else hi = mid;
        }
        uint32_t kb = 0;
        if (lo < m && rs[lo] < k && rbound[lo] != ACCORD_NO_TXN) kb = rbound[lo];
        keep_flag[c] = (cent[c] & ENT_TXN_MASK) >= kb ? 1u : 0u;
    }
}

// ---- registration ----
struct RegParams {
    uint32_t n, tx_n;
    const uint64_t *msb, *lsb;
    const int32_t *node;
    const uint8_t *status;
    const uint64_t *emsb, *elsb;
    const int32_t *enode;
    const uint64_t *tmsb, *tlsb;       // the store's TxnIds, ascending
    const int32_t *tnode;
    const uint32_t *tg;                // their global positions
    uint8_t *st;                       // by global position
    uint64_t *xmsb, *xlsb;
    int32_t *xnode;
    uint32_t *pos;                     // out: global position of every event
    accord::DevStatus *err;
    uint32_t *chg;                     // by global position: the registration epoch of its last change
    uint32_t *cchg;                    // ... of its last change from uncommitted to committed / invalid
    uint32_t epoch;
};

// The TxnId lookup in two levels: every stride-th TxnId of the store's table sampled into LDS by
// each workgroup (<= REG_SAMPLES of them), a search there, then one inside a stride of the table --
// log2(stride) dependent global loads instead of log2(tx_n) (a registration's check was 13 us on a
// 65 k-txn table)
constexpr uint32_t REG_SAMPLES = 2048;
__global__ __launch_bounds__(256) void reg_check_kernel(RegParams p, uint32_t stride_log)
{
    __shared__ uint64_t smsb[REG_SAMPLES], slsb[REG_SAMPLES];
    __shared__ int32_t snode[REG_SAMPLES];
    const uint32_t stride = 1u << stride_log, ns = (p.tx_n + stride - 1) >> stride_log;
    for (uint32_t j = threadIdx.x; j < ns; j += blockDim.x) {
        const uint32_t t = j << stride_log;
        smsb[j] = p.tmsb[t]; slsb[j] = p.tlsb[t]; snode[j] = p.tnode[t];
    }
    __syncthreads();
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < p.n; r += gridDim.x * blockDim.x) {
        const Ts id{p.msb[r], p.lsb[r], p.node[r]};
        if (r > 0 && ts_cmp(p.msb[r - 1], p.lsb[r - 1], p.node[r - 1], id.msb, id.lsb, id.node) >= 0)
            record_error(p.err, r, ACCORD_ERR_UNSORTED);
        const uint32_t nw = p.status[r];
        if (nw > ST_TRUNC_APPLY) { record_error(p.err, r, ACCORD_ERR_ARG); continue; }
        uint32_t J = 0, jh = ns;                      // samples below id
        while (J < jh) {
            const uint32_t m = (J + jh) >> 1;
            if (ts_cmp(smsb[m], slsb[m], snode[m], id.msb, id.lsb, id.node) < 0) J = m + 1; else jh = m;
        }
        // the first table entry >= id lies in ((J - 1) * stride, J * stride]
        uint32_t lo = J ? ((J - 1) << stride_log) + 1 : 0u, hi = min(J << stride_log, p.tx_n);
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (ts_cmp(p.tmsb[m], p.tlsb[m], p.tnode[m], id.msb, id.lsb, id.node) < 0) lo = m + 1; else hi = m;
        }
        if (lo >= p.tx_n || ts_cmp(p.tmsb[lo], p.tlsb[lo], p.tnode[lo], id.msb, id.lsb, id.node) != 0) {
            record_error(p.err, r, ACCORD_ERR_ARG);       // not a txn of this store
            continue;
        }
        const uint32_t g = p.tg[lo];
        p.pos[r] = g;
        const uint32_t cur = p.st[g];
        if (status_rank(nw) < status_rank(cur)) { record_error(p.err, r, ACCORD_ERR_STATE); continue; }   // never back
        if ((nw >= ST_ACCEPTED && nw <= ST_APPLIED) || nw == ST_TRUNC_APPLY) {
            const Ts ex{p.emsb[r], p.elsb[r], p.enode[r]};
            if (ts_cmp(ex.msb, ex.lsb, ex.node, id.msb, id.lsb, id.node) < 0) record_error(p.err, r, ACCORD_ERR_ARG);
            if (committed(cur) && (ex.msb != p.xmsb[g] || ex.lsb != p.xlsb[g] || ex.node != p.xnode[g]))
                record_error(p.err, r, ACCORD_ERR_STATE);  // a committed executeAt never changes
        }
    }
}

// An Erased / Invalidated range command leaves the range scan (impl/InMemoryCommandStore.java:891,
// SaveStatus >= Erased): its carried entries (owners ascending, one per range) get a kind no txn
// witnesses.
__global__ __launch_bounds__(256) void reg_erase_ranges_kernel(RegParams p, uint32_t rc_n, const uint32_t *__restrict__ rc_owner,
                                                               uint32_t *__restrict__ rc_kind)
{
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < p.n; r += gridDim.x * blockDim.x) {
        if (p.status[r] != ST_ERASED || !(p.lsb[r] & 1ull)) continue;
        const uint32_t g = p.pos[r];
        uint32_t lo = 0, hi = rc_n;
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (rc_owner[m] < g) lo = m + 1; else hi = m;
        }
        for (; lo < rc_n && rc_owner[lo] == g; ++lo) rc_kind[lo] = RC_KIND_ERASED;
    }
}

__global__ __launch_bounds__(256) void reg_apply_kernel(RegParams p)
{
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < p.n; r += gridDim.x * blockDim.x) {
        const uint32_t g = p.pos[r], nw = p.status[r], cur = p.st[g];
        p.st[g] = (uint8_t)nw;
        p.chg[g] = p.epoch;                 // readiness re-evaluates the keys of changed txns
        if (cur < ST_COMMITTED && nw >= ST_COMMITTED) p.cchg[g] = p.epoch;
        if ((nw >= ST_ACCEPTED && nw <= ST_APPLIED) || nw == ST_TRUNC_APPLY) { p.xmsb[g] = p.emsb[r]; p.xlsb[g] = p.elsb[r]; p.xnode[g] = p.enode[r]; }
    }
}

// a computed batch joins the store: TxnId table (ascending) + PREACCEPTED at executeAt = TxnId
__global__ __launch_bounds__(256) void join_kernel(uint32_t n, uint32_t tx_n, const uint64_t *__restrict__ msb,
                                                   const uint64_t *__restrict__ lsb, const int32_t *__restrict__ node,
                                                   const uint32_t *__restrict__ gidx, uint64_t *__restrict__ tmsb,
                                                   uint64_t *__restrict__ tlsb, int32_t *__restrict__ tnode,
                                                   uint32_t *__restrict__ tg, uint8_t *__restrict__ st,
                                                   uint64_t *__restrict__ xmsb, uint64_t *__restrict__ xlsb,
                                                   int32_t *__restrict__ xnode, uint32_t *__restrict__ chg, uint32_t epoch,
                                                   uint32_t *__restrict__ cchg, uint32_t known, uint32_t G,
                                                   const accord::DevStatus *__restrict__ guard)
{
    // queued before the compute's final host read: a batch the compute rejected joins nothing
    if (guard->first != ~0ull || guard->overflow) return;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        const uint32_t g = gidx[t];
        // the store's new positions [known, G): those no txn of this store holds (txn_index gaps, never
        // looked at) before g -- and after the last txn -- start PREACCEPTED and unchanged
        const uint32_t to = t + 1 == n ? G : g;
        for (uint32_t q = t ? gidx[t - 1] + 1u : known; q < to; ++q) {
            if (q == g) continue;
            chg[q] = 0u; cchg[q] = 0u; st[q] = ST_PREACCEPTED;
        }
        chg[g] = epoch;
        cchg[g] = 0u;
        tmsb[tx_n + t] = msb[t]; tlsb[tx_n + t] = lsb[t]; tnode[tx_n + t] = node[t]; tg[tx_n + t] = g;
        st[g] = ST_PREACCEPTED;
        xmsb[g] = msb[t]; xlsb[g] = lsb[t]; xnode[g] = node[t];
    }
}

inline uint32_t grid_for(uint64_t n)
{
    uint64_t b = (n + 255) / 256;
    return (uint32_t)(b < 1 ? 1 : b > 8192 ? 8192 : b);
}

// grow a buffer keeping its first `keep` bytes (the store's tables)
hipError_t grow_keep(DevBuf &b, size_t bytes, size_t keep, hipStream_t s)
{
    if (bytes <= b.cap && b.p) return hipSuccess;
    size_t want = std::max(bytes, b.cap * 2);
    void *np = nullptr;
    hipError_t e = hipMalloc(&np, want);
    if (e != hipSuccess) return e;
    if (keep && b.p) {
        e = hipMemcpyAsync(np, b.p, keep, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) { (void)hipFree(np); return e; }
    }
    if (b.p) (void)hipFree(b.p);
    b.p = np;
    b.cap = want;
    return hipSuccess;
}

StatusView view_of(accord_store *s)
{
    StatusView v;
    v.status = s->rg_status.as<uint8_t>();
    v.emsb = s->rg_emsb.as<uint64_t>(); v.elsb = s->rg_elsb.as<uint64_t>(); v.enode = s->rg_enode.as<int32_t>();
    v.known = s->next_global;
    return v;
}

// ---- range txns in a registered-status store ----
// KeyDeps of a range txn (mapReduceForKey over every CFK key of its ranges, impl/InMemoryCommandStore.
// java:274-289) without a window: per key the entries before the bound (first entry >= the txn /
// its executeAt's registered prefix), through the full mapReduceActive filter on keys that hold a
// registered status (maxCommittedBefore, committed pruning, TK / INVALID skipped) and the witness
// filter elsewhere.  One wave per range txn, a lane per key; count (FILL = false) or fill the
// keys, header and body (dep txn positions; the union pass turns them into ranks).
struct RkGenParams {
    accord::RangeDepsParams p;
    StatusView v;
    const uint32_t *flag;              // keys holding a registered status (nullptr: none)
    const uint64_t *msb, *xmsb, *xlsb;
    const int32_t *node, *xnode;
};

template <bool FILL>
__global__ __launch_bounds__(256) void rk_general_kernel(RkGenParams q)
{
    const accord::RangeDepsParams &p = q.p;
    const uint32_t lane = lane_id();
    const uint64_t lt = lanemask_lt();
    const uint32_t waves = gridDim.x * (blockDim.x / 64);
    for (uint32_t li = blockIdx.x * (blockDim.x / 64) + wave_id(); li < p.n_range_txns; li += waves) {
        const uint32_t i = p.range_txns[li];
        const uint64_t l = p.lsb[i];
        const uint32_t wmask = witness_mask((uint32_t)(l >> 1) & 7);
        const Ts sb = q.xmsb ? Ts{q.xmsb[i], q.xlsb[i], q.xnode[i]} : Ts{q.msb[i], l, q.node[i]};
        const uint32_t eb = p.g0 + (p.bound_l ? p.bound_l[i] : i);   // entries before it are registered
        uint32_t key_base = 0, kc_total = 0, k2v_base = 0;
        if (FILL) {
            key_base = p.kd_key_off[i];
            kc_total = p.kd_key_off[i + 1] - key_base;
            k2v_base = p.kd_k2v_off[i];
        }
        uint32_t kc = 0, body = 0;
        for (uint32_t r = p.rng_off[i]; r < p.rng_off[i + 1]; ++r) {
            const uint32_t ks = max(p.rng_start[r] + 1, p.key_lo), ke = min(p.rng_end[r], p.key_hi - 1);
            if (ks > ke) continue;
            for (uint32_t c0 = ks; c0 <= ke && c0 >= ks; c0 += 64) {
                const uint32_t key = c0 + lane;
                const bool valid = key <= ke && key >= ks;
                uint32_t a = 0, pos = 0, cnt = 0;
                bool flagged = false, has_mcb = false;
                Ts mcb{0, 0, 0};
                if (valid) {
                    const uint32_t kk = key - p.key_lo;
                    a = p.seg_start[kk];
                    const uint32_t c = p.seg_end[kk];
                    uint32_t lo = a, hi = c;                // first entry with txn >= eb
                    while (lo < hi) {
                        const uint32_t m = (lo + hi) >> 1;
                        if ((p.hist[m] & ENT_TXN_MASK) < eb) lo = m + 1; else hi = m;
                    }
                    pos = a < c ? lo : a;
                    flagged = q.flag && q.flag[kk];
                    if (flagged)
                        for (uint32_t x = a; x < pos; ++x) {  // maxCommittedBefore (:620-624)
                            const uint32_t e = p.hist[x], gg = e & ENT_TXN_MASK;
                            if ((e >> ENT_KIND_SHIFT) != 1u || !committed(status_of(q.v, gg))) continue;
                            const Ts ex = exec_of(q.v, gg);
                            if (tcmp(ex, sb) >= 0) continue;
                            if (!has_mcb || tcmp(ex, mcb) > 0) { mcb = ex; has_mcb = true; }
                        }
                }
                // emitted entries of [a, pos): counted, then (fill) written at the key's body offset
                auto emitted = [&](uint32_t e) -> bool {
                    if (!((wmask >> (e >> ENT_KIND_SHIFT)) & 1u)) return false;
                    if (!flagged) return true;
                    const uint32_t gg = e & ENT_TXN_MASK, st = status_of(q.v, gg);
                    if (st == ST_TK || st >= ST_INVALID) return false;
                    return !(committed(st) && has_mcb && tcmp(exec_of(q.v, gg), mcb) < 0);
                };
                for (uint32_t x = a; x < pos; ++x) cnt += emitted(p.hist[x]) ? 1u : 0u;
                const uint64_t hb = __ballot(cnt > 0);
                const uint32_t wincl = wave_incl_scan(cnt);
                if (FILL && cnt) {
                    const uint32_t ns = kc + (uint32_t)__popcll(hb & lt);
                    p.kd_keys[key_base + ns] = key;
                    p.kd_k2v[k2v_base + ns] = (int32_t)(kc_total + body + wincl);
                    uint32_t o = k2v_base + kc_total + body + wincl - cnt;
                    for (uint32_t x = a; x < pos; ++x) {
                        const uint32_t e = p.hist[x];
                        if (emitted(e)) p.kd_k2v[o++] = (int32_t)(e & ENT_TXN_MASK);
                    }
                }
                kc += (uint32_t)__popcll(hb);
                body += readlane(wincl, 63);
            }
        }
        if (!FILL && lane == 0) {
            p.cnt_keys[i] = kc;
            p.cnt_vals_k[i] = body;          // txnIds upper bound (exact count: the union pass)
            p.cnt_k2v[i] = kc + body;
        }
    }
}

} // namespace

namespace {

// ---- WaitingOn of a registered-status store's batch ----
// Commands.initialiseWaitingOn (local/Commands.java:735-753) and its initial updateWaitingOn
// (:755-830; WaitingOn.Update, local/Command.java:1403-1600) against the registered statuses: the
// RangeDeps txnId bits start set and each dep that hasBeen(PreCommitted) is resolved -- truncated /
// invalidated: setAppliedOrInvalidated; executing after us (own kind not awaitsOnlyDeps):
// removeWaitingOn; APPLIED: setAppliedAndPropagate (the dep's own appliedOrInvalidated taken as
// empty) -- the KeyDeps key bits stay set (CommandsForKey.notify clears them later).  The
// appliedOrInvalidated set exists for Range-domain txns only (Update(TxnId, Keys, ...) :1431-1437).
// A thread per txn builds its words one at a time.
// With a RedundantBefore map that can remove deps (pre != nullptr), rr_init_kernel ran first and left
// in words[] the range deps removeRedundantDependencies keeps: the others are not visited.
// executeAtLeast (awaitsOnlyDeps kinds): every visited range dep committed with an executeAt after the
// txn's TxnId (local/Commands.java:782-783) -> eal[t].
__global__ __launch_bounds__(256) void wo_init_kernel(uint32_t n, const uint64_t *__restrict__ msb,
                                                      const uint64_t *__restrict__ lsb, const int32_t *__restrict__ node,
                                                      const uint32_t *__restrict__ txn_index,
                                                      const uint32_t *__restrict__ kd_key_off,
                                                      const uint32_t *__restrict__ rd_val_off,
                                                      const uint32_t *__restrict__ rd_vals,
                                                      const uint32_t *__restrict__ wo_off, StatusView v,
                                                      unsigned long long *__restrict__ words,
                                                      unsigned long long *__restrict__ aoi, bool pre, EalRec *__restrict__ eal,
                                                      const uint32_t *__restrict__ pv_at, const uint32_t *__restrict__ pv_len,
                                                      const uint32_t *__restrict__ pv_pool, uint32_t pv_pos,
                                                      accord::DevStatus *__restrict__ err)
{
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        const uint32_t g = txn_index[t], ost = status_of(v, g);
        const uint64_t l = lsb[t];
        // own executeAt: the registered one once it has one, else the TxnId
        const Ts own = ost >= ST_ACCEPTED && ost <= ST_APPLIED ? exec_of(v, g) : Ts{msb[t], l, node[t]};
        const uint32_t kind = (uint32_t)(l >> 1) & 7u;
        const bool only_deps = kind == 4u || kind == 2u;      // Txn.Kind.awaitsOnlyDeps (Txn.java:211-214)
        const bool range_domain = (l & 1u) != 0;
        const uint32_t r0 = rd_val_off[t], R = rd_val_off[t + 1] - r0;
        const uint32_t bits = R + (kd_key_off[t + 1] - kd_key_off[t]);
        const uint32_t w0 = wo_off[t], nw = wo_off[t + 1] - w0;
        EalRec ea{0, 0, 0, 0u};                            // Timestamp.nonNullOrMax over the candidates
        // setAppliedAndPropagate: with an applied range dep whose own (released) WaitingOn recorded
        // applied / invalidated txnIds, the visit order matters -- updateWaitingOn walks the bits in
        // reverse (forEachWaitingOnId) and a propagated bit is never visited itself (ready.hip)
        bool prop = false;
        if (pv_at) {
            for (uint32_t b = 0; b < R && !prop; ++b) {
                if (pre && !((words[w0 + (b >> 6)] >> (b & 63u)) & 1ull)) continue;
                const uint32_t d = rd_vals[r0 + b];
                prop = d < pv_pos && pv_at[d] != 0u && status_of(v, d) == ST_APPLIED &&
                       (only_deps || tcmp(exec_of(v, d), own) <= 0);
            }
        }
        if (prop) {
            for (uint32_t q = 0; q < nw; ++q) {
                const uint32_t b0 = q * 64u;
                const unsigned long long all = b0 + 64u <= bits ? ~0ull : ((1ull << (bits - b0)) - 1ull);
                const unsigned long long rng = b0 >= R ? 0ull : b0 + 64u <= R ? ~0ull : ((1ull << (R - b0)) - 1ull);
                const unsigned long long kept = pre ? words[w0 + q] : ~0ull;
                words[w0 + q] = (all & ~rng) | (all & rng & kept);
                aoi[w0 + q] = 0ull;
            }
            for (uint32_t j = R; j-- > 0;) {
                const uint32_t q = j >> 6;
                const unsigned long long bit = 1ull << (j & 63u), wq = words[w0 + q];
                if (!(wq & bit)) continue;
                const uint32_t d = rd_vals[r0 + j], st = status_of(v, d);
                if (only_deps && exec_known(st)) {                            // updateExecuteAtLeast
                    const Ts de = exec_of(v, d);
                    if (ts_cmp(de.msb, de.lsb, de.node, msb[t], l, node[t]) > 0) eal_merge(ea, EalRec{de.msb, de.lsb, de.node, 1u});
                }
                if (st == ST_TRUNC_APPLY && !only_deps && tcmp(exec_of(v, d), own) >= 0) trunc_check_fail(err, t);
                if (st < ST_COMMITTED) continue;
                bool clr = false, app = false;
                if (st >= ST_INVALID) clr = app = true;
                else if (!only_deps && tcmp(exec_of(v, d), own) > 0) clr = true;
                else if (st == ST_APPLIED) clr = app = true;
                if (!clr) continue;
                words[w0 + q] = wq & ~bit;
                if (app && range_domain) aoi[w0 + q] |= bit;
                if (!(st == ST_APPLIED && app) || d >= pv_pos || pv_at[d] == 0u) continue;
                const uint32_t *Lp = pv_pool + (pv_at[d] - 1u);
                for (uint32_t a = 0, nL = pv_len[d]; a < nL; ++a) {
                    uint32_t lo = 0, hi = R;
                    while (lo < hi) { const uint32_t m = (lo + hi) >> 1; if (rd_vals[r0 + m] < Lp[a]) lo = m + 1; else hi = m; }
                    if (lo >= R || rd_vals[r0 + lo] != Lp[a]) continue;
                    const uint32_t q2 = lo >> 6;
                    const unsigned long long b2 = 1ull << (lo & 63u), w2 = words[w0 + q2];
                    if (!(w2 & b2) || (range_domain && (aoi[w0 + q2] & b2))) continue;
                    words[w0 + q2] = w2 & ~b2;
                    if (range_domain) aoi[w0 + q2] |= b2;
                }
            }
            eal[t] = ea;
            continue;
        }
        for (uint32_t q = 0; q < nw; ++q) {
            unsigned long long wv = 0, av = 0;
            const unsigned long long kept = pre ? words[w0 + q] : ~0ull;   // removeRedundantDependencies
            const uint32_t b0 = q * 64u, b1 = min(bits, b0 + 64u);
            for (uint32_t b = b0; b < b1; ++b) {
                const unsigned long long bit = 1ull << (b & 63u);
                if (b >= R) { wv |= bit; continue; }            // key bits
                if (!(kept & bit)) continue;                    // removed: not waited on, not visited
                const uint32_t d = rd_vals[r0 + b], st = status_of(v, d);
                bool wait = true, applied = false;
                if (only_deps && exec_known(st)) {                            // updateExecuteAtLeast
                    const Ts de = exec_of(v, d);
                    if (ts_cmp(de.msb, de.lsb, de.node, msb[t], l, node[t]) > 0) eal_merge(ea, EalRec{de.msb, de.lsb, de.node, 1u});
                }
                // Invariants.checkState(executeAt < waitingExecuteAt || awaitsOnlyDeps) (:789-791)
                if (st == ST_TRUNC_APPLY && !only_deps && tcmp(exec_of(v, d), own) >= 0) trunc_check_fail(err, t);
                if (st >= ST_COMMITTED) {                       // hasBeen(PreCommitted)
                    if (st >= ST_INVALID) { wait = false; applied = true; }                 // truncated / invalidated
                    else if (!only_deps && tcmp(exec_of(v, d), own) > 0) wait = false;     // executes after us
                    else if (st == ST_APPLIED) { wait = false; applied = true; }
                }
                if (wait) wv |= bit;
                if (applied && range_domain) av |= bit;
            }
            words[w0 + q] = wv;
            aoi[w0 + q] = av;
        }
        eal[t] = ea;
    }
}

// removeRedundantDependencies at initialiseWaitingOn (every bit set: minWaitingOnTxnId = the first
// range dep), a wave per txn: words[] = the range deps it keeps, key bits set.  SPILL = false: every
// txn, scratch in LDS; a txn over its caps is listed in sp and left alone.  SPILL = true: the listed
// txns, scratch in HBM (spill_base, sized for the largest of them).
template <bool SPILL>
__global__ __launch_bounds__(256) void rr_init_kernel(uint32_t n, const uint64_t *__restrict__ msb,
                                                      const uint64_t *__restrict__ lsb, const uint32_t *__restrict__ txn_index,
                                                      const uint32_t *__restrict__ key_off, const uint32_t *__restrict__ key_ord,
                                                      const uint32_t *__restrict__ rng_off, const uint32_t *__restrict__ rng_start,
                                                      const uint32_t *__restrict__ rng_end, accord_impl::CurDeps cd,
                                                      const uint64_t *__restrict__ tmsb, const uint32_t *__restrict__ tg,
                                                      uint32_t tx_n, RrMap M, const uint32_t *__restrict__ wo_off,
                                                      StatusView v, unsigned long long *__restrict__ words,
                                                      RrSpill sp, void *spill_base, uint32_t cap_r, uint32_t cap_e)
{
    __shared__ RrLds lds[4];
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    const uint32_t gw = blockIdx.x * 4u + w;
    RrBuf L;
    if constexpr (SPILL) L = rr_buf_hbm(spill_base, gw, cap_r, cap_e);
    else L = rr_buf_lds(lds[w]);
    const uint32_t m = SPILL ? *sp.count : n;
    for (uint32_t i = gw; i < m; i += gridDim.x * 4u) {
        const uint32_t t = SPILL ? sp.list[i] : i;
        const uint32_t r0 = cd.rd_val_off[t], R = cd.rd_val_off[t + 1] - r0;
        const uint32_t bits = R + (cd.kd_key_off[t + 1] - cd.kd_key_off[t]);
        const uint32_t w0 = wo_off[t], nw = wo_off[t + 1] - w0;
        bool removal = false, o = false;
        uint32_t ne = 0;
        RrTxn T{};
        if (R) {
            const uint64_t l = lsb[t];
            T.rdom = (l & 1u) != 0;
            if (T.rdom) { T.np = rng_off[t + 1] - rng_off[t]; T.ps = rng_start + rng_off[t]; T.pe = rng_end + rng_off[t]; }
            else { T.np = key_off[t + 1] - key_off[t]; T.pk = key_ord + key_off[t]; }
            T.R = R; T.rvals = cd.rd_vals + r0;
            T.nrr = cd.rd_rng_off[t + 1] - cd.rd_rng_off[t];
            T.rs = cd.rd_rng_start + cd.rd_rng_off[t]; T.re = cd.rd_rng_end + cd.rd_rng_off[t];
            T.r2v = cd.rd_r2v + cd.rd_r2v_off[t];
            const uint32_t g = txn_index[t], ost = status_of(v, g);
            const uint64_t em = ost >= ST_ACCEPTED && ost <= ST_APPLIED ? v.emsb[g] : msb[t];
            const uint32_t mpos = T.rvals[0];
            uint32_t lo = 0, hi = tx_n;                          // TxnId of the dep at mpos (epoch)
            while (lo < hi) { const uint32_t mm = (lo + hi) >> 1; if (tg[mm] < mpos) lo = mm + 1; else hi = mm; }
            removal = rr_removal(M, T, L, lane, mpos, tmsb[lo] >> 15, em >> 15, &o, &ne);
        }
        if (o) {                                                 // over the LDS caps: the spill pass
            if (lane == 0) rr_spill_add(sp, t, R, ne);
            continue;
        }
        for (uint32_t q = lane; q < nw; q += 64) {
            const uint32_t b0 = q * 64u;
            unsigned long long wv = b0 + 64u <= bits ? ~0ull : ((1ull << (bits - b0)) - 1ull);
            if (removal) wv &= ~rr_clear(L, T, q);
            words[w0 + q] = wv;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

} // namespace

namespace accord_impl {

bool registered_mode(const accord_store *s) { return s->resident && s->cfg.window == ACCORD_WINDOW_NONE; }

// WaitingOn words + appliedOrInvalidated of the last computed batch (wo_off already scanned)
int32_t status_waiting_on_init(accord_store *s, const uint32_t *wo_off, unsigned long long *words,
                               unsigned long long *aoi)
{
    const CurDeps cd = cur_deps(s);
    const uint32_t n = s->n;
    HIPCHECK(s, s->wo_eal.ensure((size_t)n * sizeof(EalRec) + 64));
    if (!n) return ACCORD_OK;
    const bool pre = s->rb_ext && s->rb_m && cd.tot_rvals;
    if (pre) {                     // removeRedundantDependencies first (redundant_wait.h)
        HIPCHECK(s, s->rr_ovf.ensure((size_t)n * 4 + 64));
        uint32_t *hdr = s->rr_ovf.as<uint32_t>();
        HIPCHECK(s, hipMemsetAsync(hdr, 0, 16, s->stream));
        const RrSpill sp{hdr, hdr + 1, hdr + 2, hdr + 16};
        auto launch = [&](bool spill, uint32_t grid, void *base, uint32_t cr, uint32_t ce) {
            auto k = spill ? rr_init_kernel<true> : rr_init_kernel<false>;
            hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, s->stream, n,
                               s->msb.as<uint64_t>(), s->lsb.as<uint64_t>(), s->txn_index.as<uint32_t>(),
                               s->key_off.as<uint32_t>(), s->key_ord.as<uint32_t>(), s->R ? s->rng_off.as<uint32_t>() : nullptr,
                               s->R ? s->rng_start.as<uint32_t>() : nullptr, s->R ? s->rng_end.as<uint32_t>() : nullptr, cd,
                               s->rg_tmsb.as<uint64_t>(), s->rg_tg.as<uint32_t>(), s->rg_tx_n, rr_map_of(s), wo_off, view_of(s),
                               words, sp, base, cr, ce);
        };
        launch(false, std::min<uint32_t>((n + 3) / 4, 8192u), nullptr, 0, 0);
        uint32_t h[3] = {0, 0, 0};
        HIPCHECK(s, hipMemcpyAsync(h, hdr, 12, hipMemcpyDeviceToHost, s->stream));
        HIPCHECK(s, hipStreamSynchronize(s->stream));
        if (h[0]) {                // txns over the LDS caps: again, with HBM scratch sized for the largest
            const uint32_t blocks = std::min<uint32_t>((h[0] + 3) / 4, 64u);
            HIPCHECK(s, s->rr_spill.ensure((size_t)blocks * 4 * rr_spill_wave_bytes(h[1], h[2])));
            launch(true, blocks, s->rr_spill.p, h[1], h[2]);
        }
    }
    HIPCHECK(s, s->wo_err.ensure(sizeof(HostTotals)));
    HostTotals *err = s->wo_err.as<HostTotals>();
    HIPCHECK(s, hipMemsetAsync(&err->status, 0xFF, sizeof(unsigned long long), s->stream));
    hipLaunchKernelGGL(wo_init_kernel, dim3(grid_for(n)), dim3(256), 0, s->stream, n, s->msb.as<uint64_t>(),
                       s->lsb.as<uint64_t>(), s->node.as<int32_t>(), s->txn_index.as<uint32_t>(),
                       cd.kd_key_off, cd.rd_val_off, cd.rd_vals, wo_off, view_of(s), words, aoi, pre,
                       s->wo_eal.as<EalRec>(), s->rdy_pv_at.as<uint32_t>(), s->rdy_pv_len.as<uint32_t>(),
                       s->rdy_pv_pool.as<uint32_t>(),
                       (uint32_t)std::min<size_t>(s->rdy_pv_pos, std::min(s->rdy_pv_at.cap, s->rdy_pv_len.cap) / 4),
                       &err->status);
    HIPCHECK(s, hipMemcpyAsync(&s->pinned->reg_status, &err->status, sizeof(accord::DevStatus), hipMemcpyDeviceToHost,
                               s->stream));
    HIPCHECK(s, hipStreamSynchronize(s->stream));
    if (s->pinned->reg_status.first != ~0ull)
        return fail(s, ACCORD_ERR_STATE, "Invariants.checkState: txn %u waits on a TruncatedApply dep executing at or "
                    "after it (local/Commands.java:789-791)", (uint32_t)(s->pinned->reg_status.first >> 32));
    return ACCORD_OK;
}


// After the segment stage of a registered-status store: pairs on keys with registered entries get
// their emitted entries materialised in two steps, so the compute needs no host read of its own:
//   status_general_count -- key flags, the committed-Write index, the per-pair counts and their
//     scan (the total lands in the store's totals[9], read back with the output sizes);
//   status_general_emit  -- once the total is known: the extended history (the batch history +
//     the emitted entries) the fill must read.
// Only the fill passes read the extension; the count passes read positions < PH, equal in both.
static GenParams general_params(accord_store *s)
{
    GenParams g{};
    g.n = s->n; g.key_lo = s->cfg.key_lo;
    g.msb = s->msb.as<uint64_t>(); g.lsb = s->lsb.as<uint64_t>(); g.node = s->node.as<int32_t>();
    if (s->has_exec) { g.xmsb = s->exec_msb.as<uint64_t>(); g.xlsb = s->exec_lsb.as<uint64_t>(); g.xnode = s->exec_node.as<int32_t>(); }
    g.key_off = s->key_off.as<uint32_t>(); g.key_ord = s->key_ord.as<uint32_t>();
    g.txn_index = s->txn_index.as<uint32_t>(); g.flag = s->rg_flag.as<uint32_t>(); g.hist = s->hist.as<uint32_t>();
    g.slice = s->slice.as<accord::PairSlice>();
    g.gcnt = s->rg_gcnt.as<uint32_t>(); g.goff = s->rg_goff.as<uint32_t>();
    g.v = view_of(s);
    g.cw_off = s->rg_cwoff.as<uint32_t>(); g.cw_pos = s->rg_cwpos.as<uint32_t>(); g.cw_pm = s->rg_cwpm.as<uint32_t>();
    g.hx = s->rg_hx.as<uint32_t>(); g.hu = s->rg_hu.as<uint32_t>(); g.skey = s->sort_key.as<uint32_t>();
    return g;
}

int32_t status_general_count(accord_store *s, uint32_t C, uint32_t PH, bool *pending)
{
    const uint32_t n = s->n, P = s->P, nkeys = s->cfg.key_hi - s->cfg.key_lo;
    hipStream_t st = s->stream;
    *pending = false;
    s->rg_flag_ok = false;
    if (C == 0 || s->next_global == 0) return ACCORD_OK;       // nothing registered can be on a key yet
    HIPCHECK(s, s->rg_flag.ensure((size_t)nkeys * 4 + 4));
    HIPCHECK(s, s->rg_gcnt.ensure((size_t)P * 4 + 4));
    HIPCHECK(s, s->rg_goff.ensure(((size_t)P + 1) * 4));
    if (!s->rg_flag_zeroed) HIPCHECK(s, hipMemsetAsync(s->rg_flag.p, 0, (size_t)nkeys * 4, st));
    s->rg_flag_zeroed = false;
    const StatusView v = view_of(s);
    s->rg_flag_ok = true;
    {   // the committed[] index of the Writes over the combined history, hx / hu
        HIPCHECK(s, s->rg_cwflag.ensure(((size_t)PH + 1) * 4));
        HIPCHECK(s, s->rg_cwoff.ensure(((size_t)PH + 1) * 4));
        HIPCHECK(s, s->rg_cwpos.ensure((size_t)PH * 4 + 4));
        HIPCHECK(s, s->rg_cwpm.ensure((size_t)PH * 4 + 4));
        HIPCHECK(s, s->rg_cwchunk.ensure(((size_t)PH / 64 + 2) * sizeof(uint4)));
        HIPCHECK(s, s->rg_hxchunk.ensure(((size_t)PH / 64 + 2) * sizeof(uint4)));
        HIPCHECK(s, s->rg_hx.ensure((size_t)PH * 4 + 4));
        HIPCHECK(s, s->rg_hu.ensure((size_t)PH * 4 + 4));
        uint32_t *flag = s->rg_cwflag.as<uint32_t>(), *off = s->rg_cwoff.as<uint32_t>();
        const uint64_t w1 = (uint64_t)(C + 63) / 64 + 2ull * ((PH + 63) / 64);
        hipLaunchKernelGGL(gen_pre_kernel, dim3((uint32_t)std::min<uint64_t>((w1 + 3) / 4, 8192u)), dim3(256), 0, st, C,
                           s->cy_key.as<uint32_t>(), s->cy_ent.as<uint32_t>(), PH, s->hist.as<uint32_t>(),
                           s->sort_key.as<uint32_t>(), v, s->rg_flag.as<uint32_t>(), flag, s->rg_hx.as<uint32_t>(),
                           s->rg_hu.as<uint32_t>(), s->rg_hxchunk.as<uint4>());
        HostTotals *dv = s->status_totals.as<HostTotals>();
        accord::exclusive_scan_u32(flag, off, PH, &dv->totals[9], s->scan_tmp.p, st);
        const uint64_t w2 = 2ull * ((PH + 63) / 64);
        hipLaunchKernelGGL(gen_mid_kernel, dim3((uint32_t)std::min<uint64_t>((w2 + 3) / 4, 8192u)), dim3(256), 0, st, PH,
                           flag, off, s->rg_cwpos.as<uint32_t>(), s->hist.as<uint32_t>(), s->sort_key.as<uint32_t>(), v,
                           s->rg_hxchunk.as<uint4>(), s->rg_hx.as<uint32_t>(), s->rg_hu.as<uint32_t>());
        const uint32_t cwb = std::min<uint32_t>((PH / 64 + 4) / 4, 8192u);
        hipLaunchKernelGGL(cw_local_kernel, dim3(cwb), dim3(256), 0, st, PH, flag, off, s->rg_cwpos.as<uint32_t>(),
                           s->hist.as<uint32_t>(), s->sort_key.as<uint32_t>(), v, s->rg_cwpm.as<uint32_t>(),
                           s->rg_cwchunk.as<uint4>());
        hipLaunchKernelGGL(cw_carry_kernel, dim3(cwb), dim3(256), 0, st, PH, flag, off, s->rg_cwpos.as<uint32_t>(),
                           s->hist.as<uint32_t>(), s->sort_key.as<uint32_t>(), v, s->rg_cwchunk.as<uint4>(),
                           s->rg_cwpm.as<uint32_t>());
    }
    const GenParams g = general_params(s);
    const uint32_t gw = (uint32_t)std::min<uint64_t>(((uint64_t)n * GEN_SPLIT + 3) / 4, 8192u);
    if (n) hipLaunchKernelGGL(general_kernel<false>, dim3(gw), dim3(256), 0, st, g);
    HostTotals *dev = s->status_totals.as<HostTotals>();
    accord::exclusive_scan_u32(g.gcnt, s->rg_goff.as<uint32_t>(), P, &dev->totals[9], s->scan_tmp.p, st);
    *pending = true;
    return ACCORD_OK;
}

// abort != nullptr (speculative fill): X is not known on the host yet -- the extension goes into
// rg_hist2 as sized (the caller ensured PH + 1 entries), and the device check aborts the pass when
// it does not fit
int32_t status_general_emit(accord_store *s, uint32_t PH, uint64_t X, const uint32_t *abort,
                            const uint32_t **hist_for_fill)
{
    const uint32_t n = s->n;
    hipStream_t st = s->stream;
    *hist_for_fill = s->hist.as<uint32_t>();
    if (X == 0 && !abort) return ACCORD_OK;
    if ((uint64_t)PH + X >= (1ull << 31)) return fail(s, ACCORD_ERR_CAPACITY, "general deps of %llu entries", (unsigned long long)X);
    HIPCHECK(s, s->rg_hist2.ensure(((size_t)PH + (abort ? 1 : X)) * 4));
    GenParams g = general_params(s);
    g.hist2 = s->rg_hist2.as<uint32_t>();
    g.ext_base = PH;
    g.abort = abort;
    const uint32_t gw = (uint32_t)std::min<uint64_t>(((uint64_t)n * GEN_SPLIT + 3) / 4, 8192u);
    if (n) hipLaunchKernelGGL(general_kernel<true>, dim3(gw), dim3(256), 0, st, g);
    *hist_for_fill = s->rg_hist2.as<uint32_t>();
    return ACCORD_OK;
}

// KeyDeps of the batch's range txns in a registered-status store (count or fill pass); the flags of
// status_general_pairs (keys holding a registered status) must be current.
int32_t status_range_keys(accord_store *s, const accord::RangeDepsParams &rp, bool fill)
{
    if (rp.n_range_txns == 0) return ACCORD_OK;
    RkGenParams q{};
    q.p = rp;
    q.v = view_of(s);
    q.flag = s->rg_flag_ok ? s->rg_flag.as<uint32_t>() : nullptr;
    q.msb = s->msb.as<uint64_t>(); q.node = s->node.as<int32_t>();
    if (s->has_exec) { q.xmsb = s->exec_msb.as<uint64_t>(); q.xlsb = s->exec_lsb.as<uint64_t>(); q.xnode = s->exec_node.as<int32_t>(); }
    const uint32_t blocks = std::min<uint32_t>((rp.n_range_txns + 3) / 4, 4096u);
    if (fill) hipLaunchKernelGGL(rk_general_kernel<true>, dim3(blocks), dim3(256), 0, s->stream, q);
    else hipLaunchKernelGGL(rk_general_kernel<false>, dim3(blocks), dim3(256), 0, s->stream, q);
    HIPCHECK(s, hipGetLastError());
    return ACCORD_OK;
}

// Carry flags of a registered-status store (the keep flags launch_carry scans), per history entry.
int32_t status_prune_flags(accord_store *s, uint32_t PH, uint32_t *keep_flag)
{
    if (PH)
        hipLaunchKernelGGL(prune_mark_kernel, dim3(grid_for(PH)), dim3(256), 0, s->stream, PH, s->hist.as<uint32_t>(),
                           view_of(s), keep_flag);
    return ACCORD_OK;
}

// CommandsForKey.withRedundantBefore (local/CommandsForKey.java:1654-1684) on a registered-status
// store's carried history, for a new RedundantBefore map (m entries (start, end], bound =
// shardAppliedOrInvalidatedBefore as a position, ACCORD_NO_TXN = none): every key's entries below its
// entry's bound leave the resident state, so the next batches no longer see them.  A bound never
// goes back in the reference (:1656); a lower one here truncates nothing more.
int32_t status_truncate_carry(accord_store *s, uint32_t m, const uint32_t *start, const uint32_t *end,
                              const uint32_t *bound)
{
    const uint32_t C = s->carry_n, key_lo = s->cfg.key_lo, nkeys = s->cfg.key_hi - key_lo;
    if (C == 0 || m == 0) return ACCORD_OK;
    // entry e covers the keys (start[e], end[e]] of the store's [key_lo, key_hi): per entry, its
    // clipped key range (store-relative, inclusive) -- no per-key table built on the host unless the
    // event-exact readiness needs one (a 100 k-key table and its walk had cost ~90 us per call)
    auto clip = [&](uint32_t e, uint32_t &lo, uint32_t &hi) {
        if (bound[e] == ACCORD_NO_TXN || bound[e] == 0) return false;
        const uint64_t a = std::max<uint64_t>((uint64_t)start[e] + 1, key_lo), b = std::min<uint64_t>(end[e], (uint64_t)key_lo + nkeys - 1);
        if (a > b) return false;
        lo = (uint32_t)(a - key_lo); hi = (uint32_t)(b - key_lo);
        return true;
    };
    bool any = false;
    for (uint32_t e = 0; e < m && !any; ++e) {
        uint32_t lo, hi;
        any = clip(e, lo, hi);
    }
    if (!any) return ACCORD_OK;
    // the readiness evaluation skips deps below each key's bound (ready.hip): a cumulative max
    std::vector<uint32_t> tkeys;          // event-exact readiness: the keys that lose entries
    if (s->rdy_event_mode) {
        std::vector<uint32_t> kb(nkeys, 0u);
        for (uint32_t e = 0; e < m; ++e) {
            uint32_t lo, hi;
            if (clip(e, lo, hi)) std::fill(kb.begin() + lo, kb.begin() + hi + 1, bound[e]);
        }
        const int32_t rc = accord_impl::ready_truncate_keys(s, kb, tkeys);
        if (rc != ACCORD_OK) return rc;
    }
    if (s->rdy_kb_host.size() != nkeys) s->rdy_kb_host.assign(nkeys, 0u);
    for (uint32_t e = 0; e < m; ++e) {
        uint32_t lo, hi;
        if (!clip(e, lo, hi)) continue;
        uint32_t *kh = s->rdy_kb_host.data();
        const uint32_t bv = bound[e];
        for (uint32_t r = lo; r <= hi; ++r) kh[r] = kh[r] > bv ? kh[r] : bv;
    }
    s->rdy_kb_dirty = true;
    hipStream_t st = s->stream;
    HIPCHECK(s, s->carry_tmp.ensure(accord::carry_temp_bytes(C, nkeys)));
    HIPCHECK(s, s->cy_key2.ensure((size_t)C * 4 + 4));
    HIPCHECK(s, s->cy_ent2.ensure((size_t)C * 4 + 4));
    HIPCHECK(s, s->scan_tmp.ensure_zeroed(accord::scan_temp_bytes(C), st));
    HIPCHECK(s, s->status_totals.ensure(sizeof(HostTotals)));
    uint32_t *flag = accord::carry_flags(s->carry_tmp.p, nkeys);
    // (the entries are on the device: accord_redundant_before_set_ex uploaded them first)
    hipLaunchKernelGGL(truncate_mark_kernel, dim3(grid_for(C)), dim3(256), 0, st, C, s->cy_key.as<uint32_t>(),
                       s->cy_ent.as<uint32_t>(), key_lo, m, s->rb_start.as<uint32_t>(), s->rb_end.as<uint32_t>(),
                       s->rb_bound.as<uint32_t>(), flag);
    HostTotals *dev = s->status_totals.as<HostTotals>();
    accord::launch_carry(C, nkeys, 0u, s->cy_key.as<uint32_t>(), s->cy_ent.as<uint32_t>(), nullptr, nullptr,
                         accord::HistoryViews{}, s->carry_tmp.p, s->scan_tmp.p, s->cy_key2.as<uint32_t>(),
                         s->cy_ent2.as<uint32_t>(), &dev->totals[8], true, st);
    HIPCHECK(s, hipMemcpyAsync(&s->pinned->totals[8], &dev->totals[8], 8, hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    HIPCHECK(s, hipGetLastError());
    const unsigned long long kept = s->pinned->totals[8];
    std::swap(s->cy_key, s->cy_key2);
    std::swap(s->cy_ent, s->cy_ent2);
    s->carry_n = (uint32_t)kept;
    ++s->carry_version;
    if (s->rdy_event_mode) return accord_impl::ready_truncate_events(s, tkeys);
    return ACCORD_OK;
}

// A computed batch of a registered-status store joins its txn tables (after the compute succeeded).
// queued inside the compute, before its final host read (the launch's host cost overlaps the device
// work); the kernel checks the compute's status itself, and status_join_commit takes the batch into
// the host bookkeeping once the compute has succeeded
int32_t status_join_queue(accord_store *s, const accord::DevStatus *guard)
{
    const uint32_t n = s->n;
    if (n == 0) return ACCORD_OK;
    hipStream_t st = s->stream;
    const size_t tx = s->rg_tx_n, G = s->b_end;
    HIPCHECK(s, grow_keep(s->rg_tmsb, (tx + n) * 8, tx * 8, st));
    HIPCHECK(s, grow_keep(s->rg_tlsb, (tx + n) * 8, tx * 8, st));
    HIPCHECK(s, grow_keep(s->rg_tnode, (tx + n) * 4, tx * 4, st));
    HIPCHECK(s, grow_keep(s->rg_tg, (tx + n) * 4, tx * 4, st));
    const size_t known = s->rg_known;
    HIPCHECK(s, grow_keep(s->rg_status, G, known, st));
    HIPCHECK(s, grow_keep(s->rg_emsb, G * 8, known * 8, st));
    HIPCHECK(s, grow_keep(s->rg_elsb, G * 8, known * 8, st));
    HIPCHECK(s, grow_keep(s->rg_enode, G * 4, known * 4, st));
    HIPCHECK(s, grow_keep(s->rg_chg, G * 4, known * 4, st));
    HIPCHECK(s, grow_keep(s->rg_cchg, G * 4, known * 4, st));
    // (the new positions' change words and statuses are initialised by the kernel: three memsets fewer)
    hipLaunchKernelGGL(join_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, (uint32_t)tx, s->msb.as<uint64_t>(),
                       s->lsb.as<uint64_t>(), s->node.as<int32_t>(), s->txn_index.as<uint32_t>(),
                       s->rg_tmsb.as<uint64_t>(), s->rg_tlsb.as<uint64_t>(), s->rg_tnode.as<int32_t>(),
                       s->rg_tg.as<uint32_t>(), s->rg_status.as<uint8_t>(), s->rg_emsb.as<uint64_t>(),
                       s->rg_elsb.as<uint64_t>(), s->rg_enode.as<int32_t>(), s->rg_chg.as<uint32_t>(), s->rg_epoch + 1u,
                       s->rg_cchg.as<uint32_t>(), (uint32_t)known, (uint32_t)G, guard);
    HIPCHECK(s, hipGetLastError());          // stream-ordered before anything that reads the tables
    return ACCORD_OK;
}

void status_join_commit(accord_store *s)
{
    if (s->n == 0) return;
    ++s->rg_epoch;
    s->rg_tx_n += s->n;
    s->rg_known = (uint32_t)s->b_end;
}

} // namespace accord_impl

extern "C" int32_t accord_txn_register(accord_store *s, uint32_t n, const uint64_t *msb, const uint64_t *lsb,
                                       const int32_t *node, const uint8_t *status, const uint64_t *exec_msb,
                                       const uint64_t *exec_lsb, const int32_t *exec_node)
{
    if (!s) return fail(nullptr, ACCORD_ERR_ARG, "null store");
    if (!accord_impl::registered_mode(s))
        return fail(s, ACCORD_ERR_STATE, "accord_txn_register needs a resident store with window ACCORD_WINDOW_NONE");
    if (n == 0) return ACCORD_OK;
    if (!msb || !lsb || !node || !status) return fail(s, ACCORD_ERR_ARG, "accord_txn_register: null argument");
    bool need_exec = false;
    for (uint32_t r = 0; r < n; ++r) {
        if (status[r] > ST_TRUNC_APPLY) return fail(s, ACCORD_ERR_ARG, "event %u: status ordinal %u", r, status[r]);
        need_exec |= (status[r] >= ST_ACCEPTED && status[r] <= ST_APPLIED) || status[r] == ST_TRUNC_APPLY;
    }
    if (need_exec && (!exec_msb || !exec_lsb || !exec_node))
        return fail(s, ACCORD_ERR_ARG, "ACCEPTED..APPLIED events need an executeAt");
    HIPCHECK(s, hipSetDevice(s->cfg.device));
    hipStream_t st = s->stream;
    // the events in one host-to-device copy: packed into a pinned staging buffer (msb | lsb | exec
    // msb | exec lsb | node | exec node | status), the device copy in op_tmp[0]
    DevBuf *T = s->op_tmp;
    // (+ the check's status words, staged as "no failure": no memset of their own)
    const size_t o_lsb = (size_t)n * 8, o_emsb = o_lsb + (size_t)n * 8, o_elsb = o_emsb + (size_t)n * 8,
                 o_node = o_elsb + (size_t)n * 8, o_enode = o_node + (size_t)n * 4, o_st = o_enode + (size_t)n * 4,
                 o_err = (o_st + n + 15) & ~(size_t)15, bytes = o_err + ((sizeof(accord::DevStatus) + 15) & ~(size_t)15);
    if (s->reg_host_cap < bytes) {
        if (s->reg_host) (void)hipHostFree(s->reg_host);
        s->reg_host = nullptr; s->reg_host_cap = 0;
        HIPCHECK(s, hipHostMalloc(&s->reg_host, bytes * 2, hipHostMallocDefault));
        s->reg_host_cap = bytes * 2;
    }
    char *h = (char *)s->reg_host;
    std::memcpy(h, msb, (size_t)n * 8);
    std::memcpy(h + o_lsb, lsb, (size_t)n * 8);
    std::memcpy(h + o_node, node, (size_t)n * 4);
    std::memcpy(h + o_st, status, n);
    std::memset(h + o_err, 0xFF, sizeof(accord::DevStatus));
    if (need_exec) {
        std::memcpy(h + o_emsb, exec_msb, (size_t)n * 8);
        std::memcpy(h + o_elsb, exec_lsb, (size_t)n * 8);
        std::memcpy(h + o_enode, exec_node, (size_t)n * 4);
    }
    HIPCHECK(s, T[0].ensure(bytes)); HIPCHECK(s, T[7].ensure((size_t)n * 4));
    HIPCHECK(s, s->status_totals.ensure(sizeof(HostTotals)));
    HIPCHECK(s, hipMemcpyAsync(T[0].p, h, bytes, hipMemcpyHostToDevice, st));
    RegParams p{};
    p.n = n; p.tx_n = s->rg_tx_n;
    char *d = (char *)T[0].p;
    p.msb = (const uint64_t *)d; p.lsb = (const uint64_t *)(d + o_lsb); p.node = (const int32_t *)(d + o_node);
    p.status = (const uint8_t *)(d + o_st);
    p.emsb = (const uint64_t *)(d + o_emsb); p.elsb = (const uint64_t *)(d + o_elsb); p.enode = (const int32_t *)(d + o_enode);
    p.tmsb = s->rg_tmsb.as<uint64_t>(); p.tlsb = s->rg_tlsb.as<uint64_t>(); p.tnode = s->rg_tnode.as<int32_t>();
    p.tg = s->rg_tg.as<uint32_t>();
    p.st = s->rg_status.as<uint8_t>();
    p.xmsb = s->rg_emsb.as<uint64_t>(); p.xlsb = s->rg_elsb.as<uint64_t>(); p.xnode = s->rg_enode.as<int32_t>();
    p.pos = T[7].as<uint32_t>();
    p.err = (accord::DevStatus *)(d + o_err);
    p.chg = s->rg_chg.as<uint32_t>();
    p.cchg = s->rg_cchg.as<uint32_t>();
    p.epoch = s->rg_epoch + 1;
    if (p.tx_n == 0) return fail(s, ACCORD_ERR_ARG, "accord_txn_register: the store holds no txn yet");
    uint32_t stride_log = 0;
    while (((uint64_t)p.tx_n + (1ull << stride_log) - 1) >> stride_log > REG_SAMPLES) ++stride_log;
    hipLaunchKernelGGL(reg_check_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, stride_log);
    HIPCHECK(s, hipMemcpyAsync(&s->pinned->reg_status, p.err, sizeof(accord::DevStatus), hipMemcpyDeviceToHost, st));
    HIPCHECK(s, hipStreamSynchronize(st));
    const accord::DevStatus hs = s->pinned->reg_status;
    if (hs.first != ~0ull) {
        const uint32_t r = (uint32_t)(hs.first >> 32);
        const int32_t code = -(int32_t)(uint32_t)hs.first;
        const char *why = code == ACCORD_ERR_UNSORTED ? "TxnIds not strictly ascending"
                        : code == ACCORD_ERR_STATE ? "status goes back, or a committed executeAt changes"
                        : "unknown TxnId, or executeAt before TxnId";
        return fail(s, code, "accord_txn_register: event %u rejected (%s); nothing applied", r, why);
    }
    ++s->rg_epoch;
    if (s->rdy_event_mode) {      // event-exact readiness: the events replayed in order (ready.hip)
        const int32_t rc = accord_impl::ready_register_events(s, n, p.pos, p.status, p.emsb, p.elsb, p.enode, p.epoch);
        if (rc != ACCORD_OK) return rc;
    } else {
        hipLaunchKernelGGL(reg_apply_kernel, dim3(grid_for(n)), dim3(256), 0, st, p);
    }
    if (s->rc_n)
        hipLaunchKernelGGL(reg_erase_ranges_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, s->rc_n,
                           s->rc_owner.as<uint32_t>(), s->rc_kind.as<uint32_t>());
    // no wait: the host inputs were consumed before the check's read-back, and every later use of
    // the tables is ordered after these kernels on the store's stream
    HIPCHECK(s, hipGetLastError());
    return ACCORD_OK;
}
