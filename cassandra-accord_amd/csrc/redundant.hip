// RedundantBefore.collectDeps on the device (include/accord_deps.h
// accord_redundant_before_set).
//
// Reference semantics (paths relative to accord-core/src/main/java/accord/):
//   PreAccept.calculatePartialDeps   messages/PreAccept.java:245-265  (builder.build().with(redundant))
//   RedundantBefore.collectDeps      local/RedundantBefore.java:418-421 -> foldl(participants, collectDep)
//   Entry.collectDep                 local/RedundantBefore.java:181-190 (outOfBounds :260-263, NONE skipped)
//   ReducingRangeMap.foldl           utils/ReducingRangeMap.java:111-194 (keys / ranges: every entry
//                                    the participants touch, once, ascending)
// The store's map is the list of its non-null entries: (start, end] ascending and disjoint, each with
// [start_epoch, end_epoch) and shardAppliedOrInvalidatedBefore as a global stream position.  Per txn
// the redundant builder receives (entry.range, bound) for every visited entry in bounds; its build()
// is a RangeDeps whose ranges are those entries (ascending = Range.compare order, each once) and
// whose txnIds are the distinct bounds.  One thread per txn: the map is small and a txn touches few
// entries, so the count pass and the fill pass each walk the txn's keys / ranges once.
#include "device_common.h"
#include "kernels.h"

namespace accord {

namespace {

// last entry whose start < k (entries ascending by start), or -1
__device__ __forceinline__ int32_t rb_last_start_below(const RbParams &p, uint32_t k)
{
    int32_t lo = 0, hi = (int32_t)p.m;
    while (lo < hi) {
        const int32_t mid = (lo + hi) >> 1;
        if (p.e_start[mid] < k) lo = mid + 1; else hi = mid;
    }
    return lo - 1;
}

// first entry whose end > s (ends ascend too: the entries are disjoint)
__device__ __forceinline__ uint32_t rb_first_end_above(const RbParams &p, uint32_t s)
{
    uint32_t lo = 0, hi = p.m;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (p.e_end[mid] > s) hi = mid; else lo = mid + 1;
    }
    return lo;
}

// Entry.collectDep: in bounds (ub = executeAt, lb = minEpoch) and a bound other than NONE
__device__ __forceinline__ bool rb_emits(const RbParams &p, uint32_t e, uint64_t exec_epoch)
{
    if (p.e_bound[e] == RB_NONE) return false;
    return !(exec_epoch < p.e_start_epoch[e] || p.min_epoch >= p.e_end_epoch[e]);
}

// visit every entry txn t's keys or ranges touch, ascending, once (ReducingRangeMap.foldl)
template <typename F> __device__ __forceinline__ void rb_for_each(const RbParams &p, uint32_t t, F f)
{
    const uint64_t em = p.exec_msb ? p.exec_msb[t] : p.msb[t];
    const uint64_t epoch = em >> 15;                            // Timestamp.epoch (primitives/Timestamp.java:308-311)
    int32_t last = -1;
    const uint32_t r0 = p.rng_off ? p.rng_off[t] : 0u, r1 = p.rng_off ? p.rng_off[t + 1] : 0u;
    if (r1 > r0) {                                              // Range domain: (s, e] meets (es, ee]
        for (uint32_t r = r0; r < r1; ++r) {
            const uint32_t s = p.rng_start[r], e = p.rng_end[r];
            for (uint32_t x = rb_first_end_above(p, s); x < p.m && p.e_start[x] < e; ++x) {
                if ((int32_t)x <= last) continue;
                last = (int32_t)x;
                if (rb_emits(p, x, epoch)) f(x);
            }
        }
        return;
    }
    for (uint32_t q = p.key_off[t]; q < p.key_off[t + 1]; ++q) {   // Key domain: es < k <= ee
        const uint32_t k = p.key_ord[q];
        const int32_t x = rb_last_start_below(p, k);
        if (x < 0 || x == last || k > p.e_end[x]) continue;
        last = x;
        if (rb_emits(p, (uint32_t)x, epoch)) f((uint32_t)x);
    }
}

// The visited entries of txn t (at most RB_MAX, else the txn is reported as a capacity overflow)
__device__ __forceinline__ uint32_t rb_collect(const RbParams &p, uint32_t t, uint32_t (&ent)[RB_MAX])
{
    uint32_t r = 0;
    rb_for_each(p, t, [&](uint32_t x) {
        if (r < RB_MAX) ent[r] = x;
        ++r;
    });
    if (r > RB_MAX) {
        atomicAdd(&p.status->overflow, 1u);
        atomicMin(&p.status->overflow_first, t);
        r = 0;
    }
    return r;
}

// first visit of its bound among the txn's entries (the builder de-duplicates txnIds)
__device__ __forceinline__ bool rb_first_of_bound(const RbParams &p, const uint32_t (&ent)[RB_MAX], uint32_t i)
{
    const uint32_t b = p.e_bound[ent[i]];
    for (uint32_t j = 0; j < i; ++j)
        if (p.e_bound[ent[j]] == b) return false;
    return true;
}

// ranges = visited entries; txnIds = their distinct bounds
__global__ __launch_bounds__(256) void rb_count_kernel(RbParams p)
{
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < p.n; t += gridDim.x * blockDim.x) {
        uint32_t ent[RB_MAX];
        const uint32_t r = rb_collect(p, t, ent);
        uint32_t u = 0;
        for (uint32_t i = 0; i < r; ++i) u += rb_first_of_bound(p, ent, i) ? 1u : 0u;
        p.cnt_rngs[t] = r;
        p.cnt_vals[t] = u;
        p.cnt_r2v[t] = 2 * r;                                    // header + one body entry per range
    }
}

// RangeDeps.Builder.build of the redundant builder: ranges ascending, txnIds ascending unique,
// keysToTxnIds = end offsets (from keyCount on) then the rank of each range's single txnId
__global__ __launch_bounds__(256) void rb_fill_kernel(RbParams p)
{
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < p.n; t += gridDim.x * blockDim.x) {
        uint32_t ent[RB_MAX];
        const uint32_t r = rb_collect(p, t, ent);
        const uint32_t ro = p.rng_off_out[t], vo = p.val_off_out[t], xo = p.r2v_off_out[t];
        for (uint32_t i = 0; i < r; ++i) {
            const uint32_t x = ent[i], b = p.e_bound[x];
            uint32_t rank = 0;                                   // distinct bounds below b
            for (uint32_t j = 0; j < r; ++j)
                if (p.e_bound[ent[j]] < b && rb_first_of_bound(p, ent, j)) ++rank;
            p.out_start[ro + i] = p.e_start[x];
            p.out_end[ro + i] = p.e_end[x];
            p.out_r2v[xo + i] = (int32_t)(r + i + 1);
            p.out_r2v[xo + r + i] = (int32_t)rank;
            if (rb_first_of_bound(p, ent, i)) p.out_vals[vo + rank] = b;
        }
    }
}

} // namespace

void launch_rb_count(const RbParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t b = (p.n + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(rb_count_kernel, dim3(b), dim3(256), 0, s, p);
}

void launch_rb_fill(const RbParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t b = (p.n + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(rb_fill_kernel, dim3(b), dim3(256), 0, s, p);
}

} // namespace accord
