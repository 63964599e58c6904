// KeyDeps construction for a PreAccept batch (SURVEY.md §8a rows a3 + a8, kernels K2-K4).
//
// Reference semantics (paths relative to accord-core/src/main/java/accord/):
//   CommandsForKey.mapReduceActive          local/CommandsForKey.java:614-650
//   PreAccept.calculatePartialDeps          messages/PreAccept.java:245-265
//   RelationMultiMap.AbstractBuilder.build  utils/RelationMultiMap.java:201-260
//   KeyDeps layout                          primitives/KeyDeps.java:150-187
// Under the status-at-time model the deps of (txn i, key) are the entries of
// the key's history (all (key, txn) pairs of the batch sorted by TxnId) in [lcw, i) whose kind
// is witnessed by kind(i), where lcw is the last Write entry j < i-W (APPLIED, so it bounds
// PRUNE_TRANSITIVE_DEPENDENCIES at :620-645) or the start of the history.
//
// One wave builds one txn's KeyDeps:
//   slots   : lanes < k locate each key's segment [lo, pos) by binary search (+ walk back to lcw)
//   phase 1 : the wave streams the raw entries of all slots; witnessed ones set a bit in an LDS
//             bitmap over [i-SPAN, i) ("near") or go to an LDS list ("far")
//   union   : |txnIds| = #distinct far + popcount(bitmap); ranks = prefix popcounts
//   fill    : txnIds (ascending == TxnId order), keysToTxnIds header (end offsets starting at
//             keyCount) and body (rank of every witnessed entry, in key order)
// The count pass writes per-txn sizes; an exclusive scan gives the CSR offsets; the fill pass
// recomputes and writes.
#include "device_common.h"
#include "kernels.h"
#include "../../include/accord_deps.h"

namespace accord {

namespace {

constexpr int KD_WAVES = 4;
constexpr int KD_THREADS = KD_WAVES * 64;
constexpr uint32_t KD_KCAP = 64;
constexpr uint32_t KD_FARCAP = 256;

__device__ __forceinline__ void record_error(DevStatus *st, uint32_t i, int32_t code)
{
    unsigned long long v = ((unsigned long long)i << 32) | (uint32_t)(-code);
    atomicMin(&st->first, v);
}

__global__ __launch_bounds__(256) void validate_pack_kernel(
    uint32_t n, const uint64_t *__restrict__ msb, const uint64_t *__restrict__ lsb, const int32_t *__restrict__ node,
    const uint32_t *__restrict__ key_off, const uint32_t *__restrict__ key_ord, const uint32_t *__restrict__ rng_off,
    const uint32_t *__restrict__ rng_start, const uint32_t *__restrict__ rng_end, uint32_t key_lo, uint32_t key_hi,
    uint32_t *__restrict__ pair_key, uint32_t *__restrict__ pair_val, DevStatus *st)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t l = lsb[i];
        const uint32_t kind = (uint32_t)(l >> 1) & 7, domain = (uint32_t)l & 1;
        if (witness_mask(kind) == 0) record_error(st, i, ACCORD_ERR_KIND);
        if (i > 0 && ts_cmp(msb[i - 1], lsb[i - 1], node[i - 1], msb[i], l, node[i]) >= 0)
            record_error(st, i, ACCORD_ERR_UNSORTED);
        const uint32_t k0 = key_off[i], k1 = key_off[i + 1];
        const uint32_t r0 = rng_off ? rng_off[i] : 0, r1 = rng_off ? rng_off[i + 1] : 0;
        if (k1 < k0 || r1 < r0) { record_error(st, i, ACCORD_ERR_ARG); continue; }
        if ((domain == 1 && k1 != k0) || (domain == 0 && r1 != r0)) record_error(st, i, ACCORD_ERR_DOMAIN);
        uint32_t prev = 0;
        for (uint32_t p = k0; p < k1; ++p) {
            const uint32_t key = key_ord[p];
            const bool in_range = key >= key_lo && key < key_hi;
            if ((p > k0 && key <= prev) || !in_range) record_error(st, i, ACCORD_ERR_KEYS);
            prev = key;
            pair_key[p] = in_range ? key - key_lo : 0u;      // keep the pipeline in bounds on error
            pair_val[p] = (kind << ENT_KIND_SHIFT) | i;
        }
        for (uint32_t r = r0; r < r1; ++r) {
            if (rng_start[r] >= rng_end[r] || (r > r0 && rng_end[r - 1] > rng_start[r]))
                record_error(st, i, ACCORD_ERR_RANGES);
        }
    }
}

__global__ __launch_bounds__(256) void segments_kernel(uint32_t P, const uint32_t *__restrict__ keys,
                                                       uint32_t *__restrict__ seg_start, uint32_t *__restrict__ seg_end)
{
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
        const uint32_t k = keys[p];
        if (p == 0 || keys[p - 1] != k) seg_start[k] = p;
        if (p == P - 1 || keys[p + 1] != k) seg_end[k] = p + 1;
    }
}

template <int WPL>
struct WaveLds {
    unsigned long long bitmap[64 * WPL];
    uint32_t wprefix[64 * WPL];
    uint32_t far[KD_FARCAP];          // value | (owner << 31)
    uint32_t slot_lo[KD_KCAP];
    uint32_t slot_rawbase[KD_KCAP + 1];
    uint32_t slot_key[KD_KCAP];
    uint32_t slot_ne[KD_KCAP];        // slot has >= 1 witnessed entry
    uint32_t slot_ns[KD_KCAP];        // index among non-empty slots
    uint32_t far_count;
    uint32_t pad[3];
};

template <int WPL, bool FILL>
__global__ __launch_bounds__(KD_THREADS) void keydeps_kernel(KeyDepsParams p)
{
    __shared__ WaveLds<WPL> lds_all[KD_WAVES];
    const uint32_t w = threadIdx.x >> 6, lane = lane_id();
    WaveLds<WPL> &L = lds_all[w];
    const uint64_t lt = lanemask_lt();
    constexpr uint32_t SPAN = 64u * 64u * WPL;

    for (uint32_t i = blockIdx.x * KD_WAVES + w; i < p.n; i += gridDim.x * KD_WAVES) {
        const uint64_t lsb_i = p.lsb[i];
        const uint32_t wmask = witness_mask((uint32_t)(lsb_i >> 1) & 7);
        const uint32_t k0 = p.key_off[i], k = p.key_off[i + 1] - k0;
        if (k > KD_KCAP) {
            if (!FILL && lane == 0) {
                atomicAdd(&p.status->overflow, 1u);
                atomicMin(&p.status->overflow_first, i);
                p.cnt_keys[i] = 0; p.cnt_vals[i] = 0; p.cnt_k2v[i] = 0;
            }
            continue;
        }

        // ---- slots: segment of each key, [lo, pos) ----
        uint32_t raw = 0;
        if (lane < k) {
            const uint32_t key = p.key_ord[k0 + lane] - p.key_lo;
            const bool in_range = key < p.key_hi - p.key_lo;  // out-of-range keys fail validation
            const uint32_t a = in_range ? p.seg_start[key] : 0u, b = in_range ? p.seg_end[key] : 0u;
            uint32_t lo = a, hi = b;                       // pos = first entry with txn >= i
            while (lo < hi) {
                uint32_t m = (lo + hi) >> 1;
                if ((p.hist[m] & ENT_TXN_MASK) < i) lo = m + 1; else hi = m;
            }
            const uint32_t pos = lo;
            uint32_t start = a;
            if (i > p.window) {                            // j < i-W are APPLIED
                const uint32_t ab = i - p.window;
                uint32_t l2 = a, h2 = pos;
                while (l2 < h2) {
                    uint32_t m = (l2 + h2) >> 1;
                    if ((p.hist[m] & ENT_TXN_MASK) < ab) l2 = m + 1; else h2 = m;
                }
                int64_t q = (int64_t)l2 - 1;               // last applied entry; walk back to a Write
                while (q >= (int64_t)a && (p.hist[q] >> ENT_KIND_SHIFT) != 1u) --q;
                if (q >= (int64_t)a) start = (uint32_t)q;
            }
            raw = pos - start;
            L.slot_lo[lane] = start;
            L.slot_key[lane] = key;
            L.slot_ne[lane] = 0;
        }
        const uint32_t incl = wave_incl_scan(raw);
        if (lane < k) L.slot_rawbase[lane] = incl - raw;
        const uint32_t raw_total = __shfl(incl, 63, 64);
#pragma unroll
        for (int q = 0; q < WPL; ++q) L.bitmap[lane * WPL + q] = 0ull;
        if (lane == 0) { L.far_count = 0; L.slot_rawbase[k] = raw_total; }
        wave_lds_sync();

        // ---- phase 1: witness filter, near bitmap / far list ----
        const int64_t base = (int64_t)i - (int64_t)SPAN;
        uint32_t witnessed_here = 0;
        {
            uint32_t s = 0;
            for (uint32_t r = lane; r < raw_total; r += 64) {
                while (L.slot_rawbase[s + 1] <= r) ++s;
                const uint32_t e = p.hist[L.slot_lo[s] + (r - L.slot_rawbase[s])];
                const uint32_t j = e & ENT_TXN_MASK;
                if ((wmask >> (e >> ENT_KIND_SHIFT)) & 1u) {
                    ++witnessed_here;
                    L.slot_ne[s] = 1;
                    if ((int64_t)j >= base) {
                        const uint32_t b = (uint32_t)((int64_t)j - base);
                        atomicOr(&L.bitmap[b >> 6], 1ull << (b & 63));
                    } else {
                        const uint32_t f = atomicAdd(&L.far_count, 1u);
                        if (f < KD_FARCAP) L.far[f] = j;
                    }
                }
            }
        }
        wave_lds_sync();
        const uint32_t F = L.far_count;
        if (F > KD_FARCAP) {
            if (!FILL && lane == 0) {
                atomicAdd(&p.status->overflow, 1u);
                atomicMin(&p.status->overflow_first, i);
                p.cnt_keys[i] = 0; p.cnt_vals[i] = 0; p.cnt_k2v[i] = 0;
            }
            continue;
        }

        // ---- union: near popcounts, far owners ----
        uint32_t pc[WPL];
        uint32_t mysum = 0;
#pragma unroll
        for (int q = 0; q < WPL; ++q) { pc[q] = (uint32_t)__popcll(L.bitmap[lane * WPL + q]); mysum += pc[q]; }
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
        const uint32_t ne = lane < k ? L.slot_ne[lane] : 0u;
        const uint64_t ne_bal = __ballot(ne != 0);
        const uint32_t kc = (uint32_t)__popcll(ne_bal);

        if (!FILL) {
            const uint32_t body = wave_sum(witnessed_here);
            if (lane == 0) {
                p.cnt_keys[i] = kc;
                p.cnt_vals[i] = far_u + near_u;
                p.cnt_k2v[i] = kc + body;
            }
            continue;
        }

        // ---- fill ----
        {
            uint32_t ex = incl2 - mysum;
#pragma unroll
            for (int q = 0; q < WPL; ++q) { L.wprefix[lane * WPL + q] = ex; ex += pc[q]; }
        }
        if (lane < k) L.slot_ns[lane] = (uint32_t)__popcll(ne_bal & lt);
        wave_lds_sync();
        const uint32_t key_base = p.kd_key_off[i], val_base = p.kd_val_off[i], k2v_base = p.kd_k2v_off[i];
        if (lane < k && ne) p.kd_keys[key_base + L.slot_ns[lane]] = L.slot_key[lane] + p.key_lo;
        // txnIds: far owners by rank, then near bits in order
        for (uint32_t f = lane; f < F; f += 64) {
            const uint32_t v = L.far[f];
            if (v & 0x80000000u) {
                const uint32_t x = v & 0x7FFFFFFFu;
                uint32_t rank = 0;
                for (uint32_t g = 0; g < F; ++g) {
                    const uint32_t y = L.far[g];
                    rank += ((y & 0x80000000u) && (y & 0x7FFFFFFFu) < x) ? 1u : 0u;
                }
                p.kd_vals[val_base + rank] = x;
            }
        }
#pragma unroll
        for (int q = 0; q < WPL; ++q) {
            unsigned long long word = L.bitmap[lane * WPL + q];
            uint32_t o = val_base + far_u + L.wprefix[lane * WPL + q];
            const int64_t wbase = base + (int64_t)(lane * WPL + q) * 64;
            while (word) {
                const int b = __builtin_ctzll(word);
                p.kd_vals[o++] = (uint32_t)(wbase + b);
                word &= word - 1;
            }
        }
        // keysToTxnIds body (+ header at each non-empty slot's last witnessed entry)
        {
            uint32_t running = 0, s = 0;
            for (uint32_t r0 = 0; r0 < raw_total; r0 += 64) {
                const uint32_t r = r0 + lane;
                bool wit = false;
                uint32_t rank = 0;
                if (r < raw_total) {
                    while (L.slot_rawbase[s + 1] <= r) ++s;
                    const uint32_t e = p.hist[L.slot_lo[s] + (r - L.slot_rawbase[s])];
                    const uint32_t j = e & ENT_TXN_MASK;
                    wit = (wmask >> (e >> ENT_KIND_SHIFT)) & 1u;
                    if (wit) {
                        if ((int64_t)j >= base) {
                            const uint32_t b = (uint32_t)((int64_t)j - base);
                            rank = far_u + L.wprefix[b >> 6] + (uint32_t)__popcll(L.bitmap[b >> 6] & ((1ull << (b & 63)) - 1ull));
                        } else {
                            for (uint32_t g = 0; g < F; ++g) {
                                const uint32_t y = L.far[g];
                                rank += ((y & 0x80000000u) && (y & 0x7FFFFFFFu) < j) ? 1u : 0u;
                            }
                        }
                    }
                }
                const uint64_t bal = __ballot(wit);
                const uint32_t pos = running + (uint32_t)__popcll(bal & lt);
                if (wit) p.kd_k2v[k2v_base + kc + pos] = (int32_t)rank;
                running += (uint32_t)__popcll(bal);
                // header: a slot's end offset is known at the wave step holding its last raw entry
                if (r < raw_total && r + 1 == L.slot_rawbase[s + 1] && L.slot_ne[s])
                    p.kd_k2v[k2v_base + L.slot_ns[s]] = (int32_t)(kc + pos + (wit ? 1u : 0u));
            }
        }
    }
}

template <bool FILL>
void launch_keydeps(const KeyDepsParams &p, int wpl, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t blocks = (p.n + KD_WAVES - 1) / KD_WAVES;
    if (blocks > 256u * 16u) blocks = 256u * 16u;
    switch (wpl) {
    case 1: hipLaunchKernelGGL((keydeps_kernel<1, FILL>), dim3(blocks), dim3(KD_THREADS), 0, s, p); break;
    case 2: hipLaunchKernelGGL((keydeps_kernel<2, FILL>), dim3(blocks), dim3(KD_THREADS), 0, s, p); break;
    default: hipLaunchKernelGGL((keydeps_kernel<4, FILL>), dim3(blocks), dim3(KD_THREADS), 0, s, p); break;
    }
}

} // namespace

void launch_validate_pack(uint32_t n, const uint64_t *msb, const uint64_t *lsb, const int32_t *node,
                          const uint32_t *key_off, const uint32_t *key_ord, const uint32_t *rng_off,
                          const uint32_t *rng_start, const uint32_t *rng_end, uint32_t key_lo, uint32_t key_hi,
                          uint32_t *pair_key, uint32_t *pair_val, DevStatus *status, hipStream_t s)
{
    if (n == 0) return;
    uint32_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(validate_pack_kernel, dim3(blocks), dim3(256), 0, s, n, msb, lsb, node, key_off, key_ord,
                       rng_off, rng_start, rng_end, key_lo, key_hi, pair_key, pair_val, status);
}

void launch_segments(uint32_t P, const uint32_t *sorted_keys, uint32_t *seg_start, uint32_t *seg_end, hipStream_t s)
{
    if (P == 0) return;
    uint32_t blocks = (P + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(segments_kernel, dim3(blocks), dim3(256), 0, s, P, sorted_keys, seg_start, seg_end);
}

void launch_keydeps_count(const KeyDepsParams &p, int wpl, hipStream_t s) { launch_keydeps<false>(p, wpl, s); }
void launch_keydeps_fill(const KeyDepsParams &p, int wpl, hipStream_t s) { launch_keydeps<true>(p, wpl, s); }

} // namespace accord
