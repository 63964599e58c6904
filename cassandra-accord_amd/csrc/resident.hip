// Resident CommandsForKey state of a store across batches.
//
// A store created with ACCORD_STORE_RESIDENT keeps, between accord_deps_compute calls, the part
// of every key's history (the CFK txns[] of local/CommandsForKey.java:415, key-major, TxnId order)
// that a later txn can still reach, and prepends it to the next batch's (key, entry) pairs before
// the bucketing sort.  Under the status-at-time model a later txn i (global position gi >= G_end,
// the end of this batch) starts its slice at the last Write j < gi - W of the key
// (mapReduceActive's maxCommittedBefore bound, :620-645), which is at or after
//     keep(key) = the last Write j < G_end - W of the key (else the key's first entry),
// so every entry before keep(key) is pruned for good (the committed entries the prune at :634-645
// would skip forever, the analogue of CommandsForKey.withRedundantBefore, :1654-1684).
// Entries carry global stream positions, so the window tests, the near/far split of the fill and
// the output txnIds are those of the single-batch run over the concatenated stream.
#include "device_common.h"
#include "kernels.h"

namespace accord {

namespace {

__global__ __launch_bounds__(256) void gen_index_kernel(uint32_t n, uint32_t base, uint32_t *__restrict__ out)
{
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) out[t] = base + t;
}

// keep[k] for every key with a segment: first position of the key's history that stays.
__global__ __launch_bounds__(256) void carry_keep_kernel(uint32_t nkeys, uint32_t thr, const uint32_t *__restrict__ hist,
                                                         const uint32_t *__restrict__ seg_start,
                                                         const uint32_t *__restrict__ seg_end,
                                                         const uint32_t *__restrict__ pw_local,
                                                         const uint32_t *__restrict__ pw_carry, uint32_t tile,
                                                         uint32_t *__restrict__ keep)
{
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nkeys; k += gridDim.x * blockDim.x) {
        const uint32_t a = seg_start[k], e = seg_end[k];
        if (e <= a) continue;                          // no entry on this key
        // x = last position of the segment whose txn < thr (entries ascend by txn)
        uint32_t lo = a, hi = e;
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if ((hist[m] & ENT_TXN_MASK) < thr) lo = m + 1; else hi = m;
        }
        uint32_t kp = a;
        if (lo > a) {
            const uint32_t x = lo - 1;
            const uint32_t lw = max(pw_local[x], pw_carry[x / tile]);   // (last Write <= x) + 1
            if (lw > a) kp = lw - 1;
        }
        keep[k] = kp;
    }
}

__global__ __launch_bounds__(256) void carry_mark_kernel(uint32_t P, const uint32_t *__restrict__ sorted_key,
                                                         const uint32_t *__restrict__ keep, uint32_t *__restrict__ flag)
{
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x)
        flag[p] = p >= keep[sorted_key[p]] ? 1u : 0u;
}

__global__ __launch_bounds__(256) void carry_scatter_kernel(uint32_t P, const uint32_t *__restrict__ flag,
                                                            const uint32_t *__restrict__ off,
                                                            const uint32_t *__restrict__ sorted_key,
                                                            const uint32_t *__restrict__ hist,
                                                            uint32_t *__restrict__ out_key, uint32_t *__restrict__ out_ent)
{
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x)
        if (flag[p]) {
            const uint32_t o = off[p];
            out_key[o] = sorted_key[p];
            out_ent[o] = hist[p];
        }
}

inline uint32_t grid_for(uint64_t n)
{
    uint64_t b = (n + 255) / 256;
    return (uint32_t)(b < 1 ? 1 : b > 8192 ? 8192 : b);
}

} // namespace

void launch_gen_index(uint32_t n, uint32_t base, uint32_t *out, hipStream_t s)
{
    if (n) hipLaunchKernelGGL(gen_index_kernel, dim3(grid_for(n)), dim3(256), 0, s, n, base, out);
}

// flags and offsets start on 16-byte boundaries, so their scan takes the register-resident path
// (sc_single_pass DIRECT: 4.8 against 8.9 us on a registered batch's carry)
inline size_t carry_round4(size_t w) { return (w + 3) & ~(size_t)3; }
uint32_t *carry_flags(void *temp, uint32_t nkeys) { return (uint32_t *)temp + carry_round4(nkeys); }

size_t carry_temp_bytes(uint32_t P, uint32_t nkeys)
{
    return (carry_round4(nkeys) + 2 * carry_round4((size_t)P + 1)) * 4 + 64;
}

void launch_carry(uint32_t P, uint32_t nkeys, uint32_t thr, const uint32_t *sorted_key, const uint32_t *hist,
                  const uint32_t *seg_start, const uint32_t *seg_end, const HistoryViews &hv, void *temp,
                  void *scan_state, uint32_t *out_key, uint32_t *out_ent, unsigned long long *total, bool flags_given,
                  hipStream_t s)
{
    uint32_t *keep = (uint32_t *)temp;
    uint32_t *flag = carry_flags(temp, nkeys);
    uint32_t *off = flag + carry_round4((size_t)P + 1);
    if (P == 0) {
        (void)hipMemsetAsync(total, 0, sizeof(*total), s);
        return;
    }
    if (!flags_given) {
        hipLaunchKernelGGL(carry_keep_kernel, dim3(grid_for(nkeys)), dim3(256), 0, s, nkeys, thr, hist, seg_start,
                           seg_end, hv.pw_local, hv.pw_carry, HISTORY_TILE, keep);
        hipLaunchKernelGGL(carry_mark_kernel, dim3(grid_for(P)), dim3(256), 0, s, P, sorted_key, keep, flag);
    }
    exclusive_scan_u32(flag, off, P, total, scan_state, s);
    hipLaunchKernelGGL(carry_scatter_kernel, dim3(grid_for(P)), dim3(256), 0, s, P, flag, off, sorted_key, hist, out_key,
                       out_ent);
}

} // namespace accord
