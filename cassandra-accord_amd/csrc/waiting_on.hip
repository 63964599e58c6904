// WaitingOn bitsets and execution levelling (config 5).
//
// Reference:
//   Commands.initialiseWaitingOn   local/Commands.java:735-753   (bits [0,R) range-dep txnIds,
//   WaitingOn.Update               local/Command.java:1403-1437   [R, R+K) keyDeps keys)
//   Commands.updateWaitingOn       local/Commands.java:755-830   (clears deps executing later /
//                                                                 applied / invalidated)
//   CommandsForKey.notify          local/CommandsForKey.java:1501-1635 (execution in executeAt order)
// Model of config 5: every txn STABLE with executeAt = txnId, none applied, so
// every dep executes earlier and no bit is cleared: the bitset is R+K ones.  Levelling
// abstraction (§8a a13): level(T) = 0 if no dep executes before T, else 1 + max level(dep).
//
// Levelling on a reduced DAG.  For a key txn i and key k, its deps on k are the witnessed entries
// of k's history in [lo, i).  Every Write w in that slice depends on every earlier witnessed entry
// of the slice (their slices nest), so max level over the slice = max over {the last Write lw of
// the slice} and, when i is a Write, the Reads after lw.  Only those are kept as predecessors.
// Then one persistent workgroup sweeps the txns in order, 1024 at a time: a txn publishes its level
// in LDS once all its predecessors have (frontier rounds with a ready flag per txn; predecessors
// of earlier chunks are final in HBM).  The chain depth of the batch bounds this kernel.
#include "device_common.h"
#include "kernels.h"
#include "../../include/accord_deps.h"

namespace accord {

namespace {

__global__ __launch_bounds__(256) void wo_bits_kernel(uint32_t n, const uint32_t *__restrict__ kd_key_off,
                                                      const uint32_t *__restrict__ rd_val_off,
                                                      const uint32_t *__restrict__ wo_off,
                                                      unsigned long long *__restrict__ words)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t bits = (rd_val_off[i + 1] - rd_val_off[i]) + (kd_key_off[i + 1] - kd_key_off[i]);
        const uint32_t w0 = wo_off[i], nw = wo_off[i + 1] - w0;
        for (uint32_t q = 0; q < nw; ++q) {
            const uint32_t hi = bits - q * 64;
            words[w0 + q] = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
        }
    }
}

__global__ __launch_bounds__(256) void wo_words_count_kernel(uint32_t n, const uint32_t *__restrict__ kd_key_off,
                                                             const uint32_t *__restrict__ rd_val_off,
                                                             uint32_t *__restrict__ cnt)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t bits = (rd_val_off[i + 1] - rd_val_off[i]) + (kd_key_off[i + 1] - kd_key_off[i]);
        cnt[i] = (bits + 63) / 64;
    }
}

// Reduced predecessors of every txn (count pass: FILL=false; fill pass: FILL=true).
// The reduction needs witnesses(i) ⊆ witnesses(Write) = {R, W}; SyncPoints (which also witness
// SyncPoints, that a Write does not) and range txns (whose KeyDeps come from rangekeys, not from
// key histories) keep their full dependency lists.
template <bool FILL>
__global__ __launch_bounds__(256) void wo_preds_kernel(WaitingOnParams p)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.n; i += gridDim.x * blockDim.x) {
        const uint64_t l = p.lsb[i];
        const uint32_t kind = (uint32_t)(l >> 1) & 7;
        const uint32_t wmask = witness_mask(kind);
        const bool reduce = (l & 1) == 0 && (wmask & ~0x3u) == 0;
        uint32_t cnt = 0;
        uint32_t o = FILL ? p.pred_off[i] : 0;
        if (reduce) {
            for (uint32_t q = p.key_off[i]; q < p.key_off[i + 1]; ++q) {
                const PairSlice ps = p.slice[q];
                const uint32_t pos = ps.pos, lo = ps.lo;
                if (pos == lo) continue;
                const uint32_t x = pos - 1;
                const uint32_t pw = max(p.pw_local[x], p.pw_carry[x / p.pw_tile]);   // (last Write <= x) + 1
                uint32_t from = lo;
                if (pw > lo) {                                                      // lw inside the slice
                    ++cnt;
                    if (FILL) p.preds[o++] = p.hist[pw - 1] & ENT_TXN_MASK;
                    from = pw;
                }
                if (wmask & 1u) {                                                   // Reads after lw
                    for (uint32_t e = from; e < pos; ++e) {
                        const uint32_t ev = p.hist[e];
                        if ((wmask >> (ev >> ENT_KIND_SHIFT)) & 1u) {
                            ++cnt;
                            if (FILL) p.preds[o++] = ev & ENT_TXN_MASK;
                        }
                    }
                }
            }
        } else {
            for (uint32_t v = p.kd_val_off[i]; v < p.kd_val_off[i + 1]; ++v) {
                ++cnt;
                if (FILL) p.preds[o++] = p.kd_vals[v];
            }
        }
        for (uint32_t v = p.rd_val_off[i]; v < p.rd_val_off[i + 1]; ++v) {     // range deps: all
            ++cnt;
            if (FILL) p.preds[o++] = p.rd_vals[v];
        }
        if (!FILL) p.pred_cnt[i] = cnt;
    }
}

constexpr int LV_THREADS = 1024;
constexpr int LV_PREG = 8;        // in-chunk predecessors held in registers; more go the slow way

// One workgroup; txns in chunks of LV_THREADS.  At chunk start every lane folds its predecessors
// from earlier chunks (final in HBM) into `best` and keeps the in-chunk ones as LDS slot indices
// in registers.  Then lanes poll the slots (lv[s] = level + 1, 0 = pending) until all are final;
// lanes never block (a wave retries in rounds, since lanes of one wave cannot wait on each
// other) and the lowest pending txn of a chunk can always finish, so each chunk drains.
// A hop along a dependency chain costs one LDS round trip.  info[0] = 1 + the chunk that hit the
// (defensive) round bound, then all stop; info[1] = max level.
__global__ __launch_bounds__(LV_THREADS) void level_kernel(uint32_t n, const uint32_t *__restrict__ pred_off,
                                                           const uint32_t *__restrict__ preds,
                                                           uint32_t *__restrict__ level, uint32_t *__restrict__ info)
{
    __shared__ uint32_t lv[LV_THREADS];
    __shared__ uint32_t smax, sabort;
    const uint32_t t = threadIdx.x;
    uint32_t mymax = 0;
    if (t == 0) { smax = 0; sabort = 0; }
    for (uint32_t base = 0; base < n; base += LV_THREADS) {
        const uint32_t i = base + t;
        lv[t] = 0;
        bool done = i >= n;
        uint32_t best = 0;                 // 1 + max over folded predecessors
        uint32_t slot[LV_PREG];
        uint32_t nslot = 0;
        uint32_t slow_next = 0, slow_end = 0;   // in-chunk predecessors beyond LV_PREG (global list)
        if (!done) {
            const uint32_t q0 = pred_off[i], q1 = pred_off[i + 1];
            for (uint32_t q = q0; q < q1; ++q) {
                const uint32_t j = preds[q];
                if (j < base) {
                    best = max(best, level[j] + 1);
                } else if (nslot < LV_PREG) {
#pragma unroll
                    for (int r = 0; r < LV_PREG; ++r)
                        if (r == (int)nslot) slot[r] = j - base;
                    ++nslot;
                } else {
                    if (slow_end == 0) slow_next = q;
                    slow_end = q + 1;
                }
            }
        }
        // gate: the latest in-chunk predecessor (the one a chain waits on); poll only it, then
        // confirm the others once it is final
        uint32_t gate = 0;
#pragma unroll
        for (int r = 0; r < LV_PREG; ++r)
            if (r < (int)nslot) gate = max(gate, slot[r]);
        __syncthreads();
        uint32_t rounds = 0;
        while (true) {
            bool moved = false;
            if (!done && (nslot == 0 || __hip_atomic_load(&lv[gate], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0)) {
                bool ok = true;
                uint32_t b2 = best;
#pragma unroll
                for (int r = 0; r < LV_PREG; ++r) {
                    if (r < (int)nslot) {
                        const uint32_t v = __hip_atomic_load(&lv[slot[r]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (v == 0 && ok) gate = slot[r];
                        ok = ok && v != 0;
                        b2 = max(b2, v);
                    }
                }
                while (ok && slow_next < slow_end) {
                    const uint32_t j = preds[slow_next];
                    if (j >= base) {
                        const uint32_t v = __hip_atomic_load(&lv[j - base], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (v == 0) { ok = false; break; }
                        best = max(best, v);
                    }
                    ++slow_next;
                }
                if (ok) {
                    best = max(best, b2);
                    __hip_atomic_store(&lv[t], best + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    level[i] = best;
                    mymax = max(mymax, best);
                    done = moved = true;
                }
            }
            if (__all(done)) break;
            if (++rounds > (1u << 22)) { sabort = 1; break; }   // defensive bound: never hit by a DAG
            // no s_sleep: a chain hop is one LDS round trip of the waiting wave
        }
        __syncthreads();
        if (sabort) {
            if (t == 0) info[0] = 1 + base / LV_THREADS;
            break;
        }
    }
    atomicMax(&smax, mymax);
    __syncthreads();
    if (t == 0) info[1] = smax;
}

} // namespace

void launch_wo_words_count(uint32_t n, const uint32_t *kd_key_off, const uint32_t *rd_val_off, uint32_t *cnt,
                           hipStream_t s)
{
    if (n == 0) return;
    uint32_t b = (n + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(wo_words_count_kernel, dim3(b), dim3(256), 0, s, n, kd_key_off, rd_val_off, cnt);
}

void launch_wo_bits(uint32_t n, const uint32_t *kd_key_off, const uint32_t *rd_val_off, const uint32_t *wo_off,
                    unsigned long long *words, hipStream_t s)
{
    if (n == 0) return;
    uint32_t b = (n + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(wo_bits_kernel, dim3(b), dim3(256), 0, s, n, kd_key_off, rd_val_off, wo_off, words);
}

void launch_wo_preds_count(const WaitingOnParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t b = (p.n + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(wo_preds_kernel<false>, dim3(b), dim3(256), 0, s, p);
}

void launch_wo_preds_fill(const WaitingOnParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t b = (p.n + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(wo_preds_kernel<true>, dim3(b), dim3(256), 0, s, p);
}

void launch_levels(uint32_t n, const uint32_t *pred_off, const uint32_t *preds, uint32_t *level, uint32_t *info,
                   hipStream_t s)
{
    if (n == 0) return;
    hipLaunchKernelGGL(level_kernel, dim3(1), dim3(LV_THREADS), 0, s, n, pred_off, preds, level, info);
}

} // namespace accord
