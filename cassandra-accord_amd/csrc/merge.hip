// K6: union of per-store partial KeyDeps of the same txns.
//
// Reference: PreAccept.reduce unions the PartialDeps of every CommandStore of a node
// (messages/PreAccept.java:140-156 -> PartialDeps.with -> RelationMultiMap.linearUnion,
// utils/RelationMultiMap.java:561-816).  The stores of a node partition the keyspace
// (local/ShardDistributor.java:46-157), so their KeyDeps have disjoint, store-ordered keys: the
// union's keys are the concatenation, its txnIds the sorted union of the parts' txnIds, and every
// body index is remapped from its part's txnIds into the union (remapToSuperset,
// utils/SortedArrays.java:1197-1223).  Keys that overlap across parts (a coordinator-side
// Deps.merge of replica replies) are rejected here with ACCORD_ERR_KEYS.
//
// One wave per txn; the txnId union uses the same near-bitmap / far-list scheme as keydeps.hip.
#include "device_common.h"
#include "kernels.h"
#include "../../include/accord_deps.h"

namespace accord {

namespace {

constexpr int MG_WAVES = 4;
constexpr uint32_t MG_GCAP = 64;       // parts
constexpr uint32_t MG_FARCAP = 512;
constexpr int MG_WPL = 2;              // bitmap span 8192 txns

struct MgLds {
    unsigned long long bitmap[64 * MG_WPL];
    uint32_t wprefix[64 * MG_WPL];
    uint32_t far[MG_FARCAP];
    uint32_t vbase[MG_GCAP + 1];   // flattened prefix of part txnId counts
    uint32_t voff[MG_GCAP];        // part's txnIds start
    uint32_t kbase[MG_GCAP + 1];   // flattened prefix of part key counts
    uint32_t koff[MG_GCAP];
    uint32_t bbase[MG_GCAP + 1];   // flattened prefix of part body counts
    uint32_t xoff[MG_GCAP];        // part's keysToTxnIds start
    uint32_t klast[MG_GCAP];
    uint32_t knk[MG_GCAP];
    uint32_t far_count;
    uint32_t pad[3];
};

__device__ __forceinline__ uint32_t find_part(const uint32_t *base, uint32_t G, uint32_t r)
{
    uint32_t l = 0, h = G;                      // last part with base <= r (base[G] = total)
    while (h - l > 1) {
        const uint32_t m = (l + h) >> 1;
        if (base[m] <= r) l = m; else h = m;
    }
    return l;
}

template <bool FILL>
__global__ __launch_bounds__(MG_WAVES * 64) void merge_kernel(MergeParams p)
{
    __shared__ MgLds lds_all[MG_WAVES];
    const uint32_t w = wave_id(), lane = lane_id();
    MgLds &L = lds_all[w];
    constexpr uint32_t SPAN = 64u * 64u * MG_WPL;
    const uint32_t G = p.G;
    for (uint32_t t = blockIdx.x * MG_WAVES + w; t < p.n; t += gridDim.x * MG_WAVES) {
        const uint32_t txn = p.txn_lo + t;          // global txn index (txnIds are < txn)
        uint32_t nv = 0, nk = 0, nb = 0, vo = 0, ko = 0, xo = 0, first_key = 0, last_key = 0;
        if (lane < G) {
            const uint32_t *vof = p.val_off[lane], *kof = p.key_off[lane], *xof = p.k2v_off[lane];
            vo = vof[t] - vof[0];                             // offsets relative to the part's slice
            nv = p.val_cnt[lane] ? p.val_cnt[lane][t] : vof[t + 1] - vof[t];   // gapped txnIds: counts
            ko = kof[t] - kof[0]; nk = kof[t + 1] - kof[t];
            xo = xof[t] - xof[0]; nb = (xof[t + 1] - xof[t]) - nk;
            if (nk) { first_key = p.keys[lane][ko]; last_key = p.keys[lane][ko + nk - 1]; }
        }
        // key blocks must be disjoint and ascending with the part index
        if (lane < G) { L.klast[lane] = last_key; L.knk[lane] = nk; }
        wave_lds_sync();
        {
            bool bad = false;
            if (lane < G && nk)
                for (int h = (int)lane - 1; h >= 0; --h)
                    if (L.knk[h]) { bad = L.klast[h] >= first_key; break; }
            if (!FILL && __any(bad) && lane == 0) {
                const unsigned long long v = ((unsigned long long)txn << 32) | (uint32_t)(-ACCORD_ERR_KEYS);
                atomicMin(&p.status->first, v);
            }
        }
        const uint32_t vinc = wave_incl_scan(nv), kinc = wave_incl_scan(nk), binc = wave_incl_scan(nb);
        if (lane < G) {
            L.vbase[lane] = vinc - nv; L.voff[lane] = vo;
            L.kbase[lane] = kinc - nk; L.koff[lane] = ko;
            L.bbase[lane] = binc - nb; L.xoff[lane] = xo;
        }
        const uint32_t VT = __shfl(vinc, 63, 64), KT = __shfl(kinc, 63, 64), BT = __shfl(binc, 63, 64);
        if (lane == 0) { L.vbase[G] = VT; L.kbase[G] = KT; L.bbase[G] = BT; L.far_count = 0; }
#pragma unroll
        for (int q = 0; q < MG_WPL; ++q) L.bitmap[lane * MG_WPL + q] = 0ull;
        wave_lds_sync();

        // txnId union: near bitmap over [txn-SPAN, txn), far list below
        const int64_t base = (int64_t)txn - (int64_t)SPAN;
        for (uint32_t r = lane; r < VT; r += 64) {
            const uint32_t g = find_part(L.vbase, G, r);
            const uint32_t j = p.vals[g][L.voff[g] + (r - L.vbase[g])];
            if ((int64_t)j >= base) {
                const uint32_t b = (uint32_t)((int64_t)j - base);
                atomicOr(&L.bitmap[b >> 6], 1ull << (b & 63));
            } else {
                const uint32_t f = atomicAdd(&L.far_count, 1u);
                if (f < MG_FARCAP) L.far[f] = j;
            }
        }
        wave_lds_sync();
        const uint32_t F = L.far_count;
        if (F > MG_FARCAP) {
            if (!FILL && lane == 0) {
                atomicAdd(&p.status->overflow, 1u);
                atomicMin(&p.status->overflow_first, txn);
                p.cnt_vals[t] = 0;
            }
            continue;
        }
        uint32_t pc[MG_WPL], mysum = 0;
#pragma unroll
        for (int q = 0; q < MG_WPL; ++q) { pc[q] = (uint32_t)__popcll(L.bitmap[lane * MG_WPL + q]); mysum += pc[q]; }
        const uint32_t incl2 = wave_incl_scan(mysum);
        const uint32_t near_u = __shfl(incl2, 63, 64);
        uint32_t far_u = 0;
        for (uint32_t f = lane; f < F; f += 64) {
            const uint32_t x = L.far[f] & 0x7FFFFFFFu;
            bool owner = true;
            for (uint32_t g = 0; g < f; ++g)
                if ((L.far[g] & 0x7FFFFFFFu) == x) { owner = false; break; }
            far_u += owner ? 1u : 0u;
            if (FILL && owner) L.far[f] = x | 0x80000000u;
        }
        far_u = wave_sum(far_u);
        if (!FILL) {
            if (lane == 0) p.cnt_vals[t] = far_u + near_u;
            continue;
        }
        {
            uint32_t ex = incl2 - mysum;
#pragma unroll
            for (int q = 0; q < MG_WPL; ++q) { L.wprefix[lane * MG_WPL + q] = ex; ex += pc[q]; }
        }
        wave_lds_sync();
        auto rank_of = [&](uint32_t j) -> uint32_t {
            if ((int64_t)j >= base) {
                const uint32_t b = (uint32_t)((int64_t)j - base);
                return far_u + L.wprefix[b >> 6] + (uint32_t)__popcll(L.bitmap[b >> 6] & ((1ull << (b & 63)) - 1ull));
            }
            uint32_t rank = 0;
            for (uint32_t g = 0; g < F; ++g) {
                const uint32_t y = L.far[g];
                rank += ((y & 0x80000000u) && (y & 0x7FFFFFFFu) < j) ? 1u : 0u;
            }
            return rank;
        };
        const uint32_t ob_k = p.out_key_off[t], ob_v = p.out_val_off[t], ob_x = p.out_k2v_off[t];
        // txnIds: every part's entry writes its own value at its rank
        for (uint32_t r = lane; r < VT; r += 64) {
            const uint32_t g = find_part(L.vbase, G, r);
            const uint32_t j = p.vals[g][L.voff[g] + (r - L.vbase[g])];
            p.out_vals[ob_v + rank_of(j)] = j;
        }
        // keys (concatenation) and header: end = KT + bodies of earlier parts + (part end - part kc)
        for (uint32_t r = lane; r < KT; r += 64) {
            const uint32_t g = find_part(L.kbase, G, r);
            const uint32_t m = r - L.kbase[g];
            const uint32_t nkg = L.kbase[g + 1] - L.kbase[g];
            p.out_keys[ob_k + r] = p.keys[g][L.koff[g] + m];
            const int32_t end_g = p.k2v[g][L.xoff[g] + m];
            p.out_k2v[ob_x + r] = (int32_t)(KT + L.bbase[g] + ((uint32_t)end_g - nkg));
        }
        // body: remap every part's index into the union
        for (uint32_t r = lane; r < BT; r += 64) {
            const uint32_t g = find_part(L.bbase, G, r);
            const uint32_t q = r - L.bbase[g];
            const uint32_t nkg = L.kbase[g + 1] - L.kbase[g];
            const int32_t v = p.k2v[g][L.xoff[g] + nkg + q];
            const uint32_t j = p.vals[g][L.voff[g] + (uint32_t)v];
            p.out_k2v[ob_x + KT + r] = (int32_t)rank_of(j);
        }
    }
}

__global__ __launch_bounds__(256) void merge_sizes_kernel(MergeParams p)
{
    // keys and keysToTxnIds sizes of the union are the sums over the parts
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < p.n; t += gridDim.x * blockDim.x) {
        uint32_t nk = 0, nx = 0;
        for (uint32_t g = 0; g < p.G; ++g) {
            nk += p.key_off[g][t + 1] - p.key_off[g][t];
            nx += p.k2v_off[g][t + 1] - p.k2v_off[g][t];
        }
        p.cnt_keys[t] = nk;
        p.cnt_k2v[t] = nx;
    }
}

__global__ void scatter_ones_kernel(uint32_t n, const uint32_t *__restrict__ idx, uint32_t *__restrict__ ind)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) ind[idx[i]] = 1u;
}

__global__ void expand_offsets_kernel(uint32_t n_total, const uint32_t *__restrict__ c, XchgOffsets in, XchgOffsets out)
{
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t <= n_total; t += gridDim.x * blockDim.x) {
        const uint32_t q = c[t];
#pragma unroll
        for (int a = 0; a < XCHG_NA; ++a) out.p[a][t] = in.p[a][q];
    }
}

// Per destination rank d (its txns [d*n_total/G, (d+1)*n_total/G)) and offset array a: the element
// count and first element of what this rank sends, read off the (expanded) offset arrays, plus a
// status word (0 = this rank goes ahead).
__global__ void xchg_counts_kernel(uint32_t G, uint32_t n_total, XchgOffsets e, unsigned long long *__restrict__ counts)
{
    constexpr uint32_t W = 2 * XCHG_NA;
    for (uint32_t x = threadIdx.x; x < G * XCHG_NA; x += blockDim.x) {
        const uint32_t d = x / XCHG_NA, a = x % XCHG_NA;
        const uint32_t t0 = (uint32_t)(((unsigned long long)d * n_total) / G);
        const uint32_t t1 = (uint32_t)(((unsigned long long)(d + 1) * n_total) / G);
        const uint32_t b0 = e.p[a][t0], b1 = e.p[a][t1];
        counts[W * d + a] = b1 - b0;
        counts[W * d + XCHG_NA + a] = b0;
    }
    if (threadIdx.x == 0) counts[W * G] = 0ull;
}

} // namespace

void launch_expand_index(uint32_t n, uint32_t n_total, const uint32_t *txn_index, uint32_t *ind, uint32_t *c,
                         void *scan_tmp, unsigned long long *total, hipStream_t s)
{
    (void)hipMemsetAsync(ind, 0, (size_t)n_total * 4 + 4, s);
    uint32_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (n) hipLaunchKernelGGL(scatter_ones_kernel, dim3(blocks ? blocks : 1), dim3(256), 0, s, n, txn_index, ind);
    exclusive_scan_u32(ind, c, n_total, total, scan_tmp, s);
}

void launch_expand_offsets(uint32_t n_total, const uint32_t *c, const XchgOffsets &in, const XchgOffsets &out,
                           hipStream_t s)
{
    uint32_t b2 = (n_total + 256) / 256;
    if (b2 > 4096) b2 = 4096;
    hipLaunchKernelGGL(expand_offsets_kernel, dim3(b2), dim3(256), 0, s, n_total, c, in, out);
}

void launch_xchg_counts(uint32_t G, uint32_t n_total, const XchgOffsets &e, unsigned long long *counts, hipStream_t s)
{
    hipLaunchKernelGGL(xchg_counts_kernel, dim3(1), dim3(256), 0, s, G, n_total, e, counts);
}

void launch_merge_count(const MergeParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t blocks = (p.n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(merge_sizes_kernel, dim3(blocks), dim3(256), 0, s, p);
    uint32_t wb = (p.n + MG_WAVES - 1) / MG_WAVES;
    if (wb > 4096) wb = 4096;
    hipLaunchKernelGGL(merge_kernel<false>, dim3(wb), dim3(MG_WAVES * 64), 0, s, p);
}

void launch_merge_fill(const MergeParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t wb = (p.n + MG_WAVES - 1) / MG_WAVES;
    if (wb > 4096) wb = 4096;
    hipLaunchKernelGGL(merge_kernel<true>, dim3(wb), dim3(MG_WAVES * 64), 0, s, p);
}

} // namespace accord
