// SearchableRangeList stabbing of every txn's RangeDeps on the device (SURVEY.md §8a row a11,
// §8f row 3): the index RangeDeps builds lazily (primitives/RangeDeps.java:709-720,
// utils/SearchableRangeList.java:79-133) and the query RangeDeps.forEach(key | range) runs over it
// (utils/CheckpointIntervalArray.java:100-221), batched over a whole deps set.
//
// Index.  A txn's RangeDeps ranges are sorted by (start, end) (RangeDeps layout).  Every RI_C-th
// range is a checkpoint; list(c) holds, ascending, the ranges before checkpoint c that end after its
// start -- the ranges a stab landing in the block may still intersect although they start earlier
// (CheckpointIntervalArrayBuilder keeps the same "tails" per checkpoint, choosing checkpoints
// greedily to bound the scan distance; here the stride is fixed, the lists exact).
//
// Query (qs, qe] (a key k is (k-1, k]; Range.EndInclusive).  Let lo = first range with start >= qs
// and end = first range with start >= qe.  The ranges [lo, end) intersect (their start lies in
// [qs, qe)); of those before lo, exactly the ones ending after qs do: list(cp) and the block
// [cp*RI_C, lo), cp = (lo - 1) / RI_C (a checkpoint whose start is < qs, so list(cp) holds every
// earlier range that reaches past qs).  The result is RangeDeps.computeTxnIds over the matches:
// the union of their txnIds, ascending (an LDS bitmap over the txn's value indices).
#include "device_common.h"
#include "kernels.h"
#include "../../include/accord_deps.h"

namespace accord {

namespace {

constexpr int RI_WAVES = 4;

__global__ __launch_bounds__(256) void ri_chk_count_kernel(RangeIndexParams p)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < p.n; i += gridDim.x * blockDim.x) {
        const uint32_t nr = p.rng_off[i + 1] - p.rng_off[i];
        if (nr > RI_MAX_RANGES) {
            atomicAdd(&p.status->overflow, 1u);
            atomicMin(&p.status->overflow_first, i);
        }
        p.chk_cnt[i] = nr > RI_MAX_RANGES ? 0u : (nr + RI_C - 1) / RI_C;
    }
}

// thread per checkpoint (global index g): its txn by binary search over chk_off
template <bool FILL>
__global__ __launch_bounds__(256) void ri_list_kernel(RangeIndexParams p, uint32_t nchk)
{
    for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < nchk; g += gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = p.n;                 // last txn with chk_off <= g
        while (hi - lo > 1) {
            const uint32_t m = (lo + hi) >> 1;
            if (p.chk_off[m] <= g) lo = m; else hi = m;
        }
        const uint32_t i = lo, c = g - p.chk_off[i], base = p.rng_off[i];
        const uint32_t s0 = p.rs[base + c * RI_C];
        uint32_t cnt = 0, o = FILL ? p.list_off[g] : 0u;
        for (uint32_t r = 0; r < c * RI_C; ++r)
            if (p.re[base + r] > s0) {
                if (FILL) p.lists[o + cnt] = r;
                ++cnt;
            }
        if (!FILL) p.list_cnt[g] = cnt;
    }
}

__global__ __launch_bounds__(256) void ri_qtxn_kernel(uint32_t n, const uint32_t *__restrict__ q_off,
                                                      uint32_t *__restrict__ q_txn)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        for (uint32_t q = q_off[i]; q < q_off[i + 1]; ++q) q_txn[q] = i;
}

// first index in [lo, hi) of the txn's ranges with start >= x (wave-uniform)
__device__ __forceinline__ uint32_t ri_lower(const uint32_t *__restrict__ rs, uint32_t lo, uint32_t hi, uint32_t x)
{
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (rs[m] < x) lo = m + 1; else hi = m;
    }
    return lo;
}

// set the value bits of range r (txn-local index) in the LDS bitmap
__device__ __forceinline__ void ri_mark(const RangeIndexParams &p, uint32_t xb, uint32_t nr, uint32_t r,
                                        uint32_t *bm)
{
    const uint32_t b = r == 0 ? nr : (uint32_t)p.r2v[xb + r - 1], e = (uint32_t)p.r2v[xb + r];
    for (uint32_t x = b; x < e; ++x) {
        const uint32_t v = (uint32_t)p.r2v[xb + x];
        atomicOr(&bm[v >> 5], 1u << (v & 31));
    }
}

// one wave per query: count pass writes |txnIds|, fill pass the txnIds ascending
template <bool FILL>
__global__ __launch_bounds__(RI_WAVES * 64) void ri_stab_kernel(RangeIndexParams p)
{
    __shared__ uint32_t bm_all[RI_WAVES][RI_UMAX / 32];
    const uint32_t w = wave_id(), lane = lane_id();
    uint32_t *bm = bm_all[w];
    for (uint32_t q = blockIdx.x * RI_WAVES + w; q < p.nq; q += gridDim.x * RI_WAVES) {
        const uint32_t i = p.q_txn[q], qs = p.q_s[q], qe = p.q_e[q];
        const uint32_t base = p.rng_off[i], nr = p.rng_off[i + 1] - base;
        const uint32_t vb = p.val_off[i], U = p.val_off[i + 1] - vb, xb = p.r2v_off[i];
        if (U > RI_UMAX || nr > RI_MAX_RANGES || qs >= qe) {
            if (!FILL) {
                if (lane == 0) p.out_cnt[q] = 0;
                if (lane == 0 && (U > RI_UMAX || nr > RI_MAX_RANGES)) {
                    atomicAdd(&p.status->overflow, 1u);
                    atomicMin(&p.status->overflow_first, i);
                }
            }
            continue;
        }
        const uint32_t words = (U + 31) / 32;
        for (uint32_t k = lane; k < words; k += 64) bm[k] = 0;
        wave_lds_sync();
        const uint32_t *rs = p.rs + base, *re = p.re + base;
        const uint32_t lo = ri_lower(rs, 0, nr, qs), end = ri_lower(rs, lo, nr, qe);
        // the run [lo, end): every range starts inside [qs, qe)
        for (uint32_t r = lo + lane; r < end; r += 64) ri_mark(p, xb, nr, r, bm);
        if (lo > 0) {
            const uint32_t cp = (lo - 1) / RI_C;
            // the block [cp * RI_C, lo) and list(cp): earlier ranges reaching past qs
            for (uint32_t r = cp * RI_C + lane; r < lo; r += 64)
                if (re[r] > qs) ri_mark(p, xb, nr, r, bm);
            const uint32_t g = p.chk_off[i] + cp, lb = p.list_off[g], le = p.list_off[g + 1];
            for (uint32_t x = lb + lane; x < le; x += 64) {
                const uint32_t r = p.lists[x];
                if (re[r] > qs) ri_mark(p, xb, nr, r, bm);
            }
        }
        wave_lds_sync();
        if (!FILL) {
            uint32_t c = 0;
            for (uint32_t k = lane; k < words; k += 64) c += (uint32_t)__popc(bm[k]);
            c = wave_sum(c);
            if (lane == 0) p.out_cnt[q] = c;
            continue;
        }
        uint32_t o = p.out_off[q];
        for (uint32_t k0 = 0; k0 < words; k0 += 64) {
            const uint32_t k = k0 + lane;
            const uint32_t bits = k < words ? bm[k] : 0u;
            const uint32_t c = (uint32_t)__popc(bits);
            const uint32_t incl = wave_incl_scan(c);
            uint32_t at = o + incl - c, b = bits;
            while (b) {
                const uint32_t t = (uint32_t)__builtin_ctz(b);
                b &= b - 1;
                p.out[at++] = p.vals[vb + k * 32 + t];
            }
            o += __shfl(incl, 63, 64);
        }
    }
}

inline uint32_t ri_grid(uint64_t n, uint32_t per)
{
    uint64_t b = (n + per - 1) / per;
    return (uint32_t)(b < 1 ? 1 : b > 8192 ? 8192 : b);
}

} // namespace

void launch_ri_chk_count(const RangeIndexParams &p, hipStream_t s)
{
    if (p.n) hipLaunchKernelGGL(ri_chk_count_kernel, dim3(ri_grid(p.n, 256)), dim3(256), 0, s, p);
}

void launch_ri_lists(const RangeIndexParams &p, uint32_t nchk, bool fill, hipStream_t s)
{
    if (!nchk) return;
    if (fill) hipLaunchKernelGGL(ri_list_kernel<true>, dim3(ri_grid(nchk, 256)), dim3(256), 0, s, p, nchk);
    else hipLaunchKernelGGL(ri_list_kernel<false>, dim3(ri_grid(nchk, 256)), dim3(256), 0, s, p, nchk);
}

void launch_ri_qtxn(uint32_t n, const uint32_t *q_off, uint32_t *q_txn, hipStream_t s)
{
    if (n) hipLaunchKernelGGL(ri_qtxn_kernel, dim3(ri_grid(n, 256)), dim3(256), 0, s, n, q_off, q_txn);
}

void launch_ri_stab(const RangeIndexParams &p, bool fill, hipStream_t s)
{
    if (!p.nq) return;
    const uint32_t g = ri_grid(p.nq, RI_WAVES);
    if (fill) hipLaunchKernelGGL(ri_stab_kernel<true>, dim3(g), dim3(RI_WAVES * 64), 0, s, p);
    else hipLaunchKernelGGL(ri_stab_kernel<false>, dim3(g), dim3(RI_WAVES * 64), 0, s, p);
}

} // namespace accord
