// Range transactions: RangeDeps for every txn and the KeyDeps
// of range-domain txns.
//
// Reference semantics (paths relative to accord-core/src/main/java/accord/):
//   range-command scan       impl/InMemoryCommandStore.java:883-1016 (Erased skipped :891,
//                            txnId < startedBefore :901-902, witness :927, each range of the
//                            command intersecting the query -> (range, txnId) :950-959, collected
//                            in a TreeMap by Range.compare and replayed in that order)
//   range query over CFKs    impl/InMemoryCommandStore.java:274-289 (every CFK key in (start,end])
//   RangeDeps layout         primitives/RangeDeps.java:81-99 (RelationMultiMap with Range keys)
// Under the status-at-time model a range command j is live for txn i iff i-W <= j < i, so the
// candidate ranges of txn i are exactly the contiguous span rng[rng_off[max(0,i-W)], rng_off[i])
// of the batch's range CSR (the window bounds the live set; each wave stabs it directly).
#include "device_common.h"
#include "kernels.h"
#include "../../include/accord_deps.h"

namespace accord {

namespace {

constexpr int RD_WAVES = 4;
constexpr uint32_t RD_HCAP = 512;

__device__ __forceinline__ void rd_overflow(DevStatus *st, uint32_t i)
{
    atomicAdd(&st->overflow, 1u);
    atomicMin(&st->overflow_first, i);
}

struct RdLds {
    unsigned long long code[RD_HCAP];   // start << 32 | end
    uint32_t j[RD_HCAP];
    uint32_t jrank[RD_HCAP];
    uint32_t first[RD_HCAP];            // first hit (lowest txn) of its range
};

// Does (s, e] intersect the query of txn i?  Key query: some key k with s < k <= e.  Range query:
// some (qs, qe] with s < qe && qs < e (Range.compareIntersecting semantics, Range.java:296-308).
__device__ __forceinline__ bool rd_hits(const RangeDepsParams &p, uint32_t s, uint32_t e, bool key_query, uint32_t q0,
                                        uint32_t q1)
{
    if (key_query) {
        uint32_t lo = q0, hi = q1;                       // first key > s
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (p.key_ord[m] <= s) lo = m + 1; else hi = m;
        }
        return lo < q1 && p.key_ord[lo] <= e;
    }
    uint32_t lo = q0, hi = q1;                           // first query range with end > s
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (p.rng_end[m] <= s) lo = m + 1; else hi = m;
    }
    return lo < q1 && p.rng_start[lo] < e;
}

template <bool FILL>
__global__ __launch_bounds__(RD_WAVES * 64) void rangedeps_kernel(RangeDepsParams p)
{
    __shared__ RdLds lds_all[RD_WAVES];
    const uint32_t w = wave_id(), lane = lane_id();
    RdLds &L = lds_all[w];
    const uint64_t lt = lanemask_lt();
    for (uint32_t i = blockIdx.x * RD_WAVES + w; i < p.n; i += gridDim.x * RD_WAVES) {
        const uint64_t lsb_i = p.lsb[i];
        const uint32_t wmask = witness_mask((uint32_t)(lsb_i >> 1) & 7);
        const bool key_query = (lsb_i & 1) == 0;
        const uint32_t q0 = key_query ? p.key_off[i] : p.rng_off[i];
        const uint32_t q1 = key_query ? p.key_off[i + 1] : p.rng_off[i + 1];
        const uint32_t r_lo = p.rng_off[i > p.window ? i - p.window : 0], r_hi = p.rng_off[i];
        uint32_t H = 0;
        if (q1 > q0) {
            for (uint32_t r0 = r_lo; r0 < r_hi; r0 += 64) {
                const uint32_t r = r0 + lane;
                bool hit = false;
                uint32_t j = 0, s = 0, e = 0;
                if (r < r_hi) {
                    j = p.rng_owner[r];
                    s = p.rng_start[r];
                    e = p.rng_end[r];
                    hit = ((wmask >> ((uint32_t)(p.lsb[j] >> 1) & 7)) & 1u) && rd_hits(p, s, e, key_query, q0, q1);
                }
                const uint64_t bal = __ballot(hit);
                const uint32_t h = H + (uint32_t)__popcll(bal & lt);
                if (hit && h < RD_HCAP) {
                    L.code[h] = ((unsigned long long)s << 32) | e;
                    L.j[h] = j;
                }
                H += (uint32_t)__popcll(bal);
            }
        }
        if (H > RD_HCAP) {
            if (!FILL && lane == 0) {
                rd_overflow(p.status, i);
                p.cnt_rngs[i] = 0; p.cnt_vals[i] = 0; p.cnt_r2v[i] = 0;
            }
            continue;
        }
        wave_lds_sync();
        // hits arrive in range-CSR order, i.e. TxnId order: distinct txnIds are the transitions
        uint32_t run = 0;
        for (uint32_t h0 = 0; h0 < H; h0 += 64) {
            const uint32_t h = h0 + lane;
            const bool tr = h < H && (h == 0 || L.j[h] != L.j[h - 1]);
            const uint64_t bal = __ballot(tr);
            if (h < H) L.jrank[h] = run + (uint32_t)__popcll(bal & ((lt << 1) | 1ull)) - 1u;
            run += (uint32_t)__popcll(bal);
        }
        const uint32_t uj = run;
        wave_lds_sync();
        // distinct ranges (Range.compare order) and sorted positions: O(H^2) over a tiny H
        uint32_t ur = 0;
        for (uint32_t h = lane; h < H; h += 64) {
            const unsigned long long c = L.code[h];
            bool first = true;
            for (uint32_t g = 0; g < H; ++g)
                if (L.code[g] == c && L.j[g] < L.j[h]) { first = false; break; }
            ur += first ? 1u : 0u;
            L.first[h] = first ? 1u : 0u;
        }
        ur = wave_sum(ur);
        wave_lds_sync();
        if (!FILL) {
            if (lane == 0) { p.cnt_rngs[i] = ur; p.cnt_vals[i] = uj; p.cnt_r2v[i] = ur + H; }
            continue;
        }
        const uint32_t rb = p.rd_rng_off[i], vb = p.rd_val_off[i], xb = p.rd_r2v_off[i];
        for (uint32_t h = lane; h < H; h += 64) {
            const unsigned long long c = L.code[h];
            const uint32_t jh = L.j[h];
            uint32_t le_code = 0, before = 0, first_before = 0;
            const bool first = L.first[h] != 0;
            for (uint32_t g = 0; g < H; ++g) {
                const unsigned long long cg = L.code[g];
                const uint32_t jg = L.j[g];
                le_code += cg <= c ? 1u : 0u;
                before += (cg < c || (cg == c && jg < jh)) ? 1u : 0u;
                first_before += (cg < c && L.first[g]) ? 1u : 0u;   // distinct ranges below c
            }
            p.rd_vals[vb + L.jrank[h]] = jh;
            p.rd_r2v[xb + ur + before] = (int32_t)L.jrank[h];
            if (first) {
                p.rd_rng_start[rb + first_before] = (uint32_t)(c >> 32);
                p.rd_rng_end[rb + first_before] = (uint32_t)c;
                p.rd_r2v[xb + first_before] = (int32_t)(ur + le_code);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// KeyDeps of range txns: one block per range txn.  Every key in its ranges with a non-empty
// history gets the same [lcw, pos) slice as a key txn (CommandsForKey.mapReduceActive
// :614-650); the union of the witnessed entries is sorted in LDS (bitonic) and de-duplicated.
// ---------------------------------------------------------------------------------------------
constexpr int RK_THREADS = 256;
constexpr uint32_t RK_SCAP = 2048;     // keys with entries per range txn
constexpr uint32_t RK_CCAP = 8192;     // witnessed entries per range txn

struct RkLds {
    uint32_t slot_key[RK_SCAP];
    uint32_t slot_lo[RK_SCAP];
    uint32_t slot_base[RK_SCAP + 1];   // exclusive prefix of raw counts
    uint32_t slot_cnt[RK_SCAP];        // witnessed per slot
    uint32_t buf[RK_CCAP];             // witnessed txn indices (sorted in place)
    uint32_t wsum[RK_THREADS / 64];
    uint32_t nslots, raw_total, nwit, nuniq, overflow;
};

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *wsum, uint32_t &total)
{
    const uint32_t tid = threadIdx.x, w = tid >> 6;
    const uint32_t inc = wave_incl_scan(v);
    if (lane_id() == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (uint32_t q = 0; q < RK_THREADS / 64; ++q) { if (q < w) off += wsum[q]; tot += wsum[q]; }
    total = tot;
    __syncthreads();
    return off + inc - v;
}

template <bool FILL>
__global__ __launch_bounds__(RK_THREADS) void rangekeys_kernel(RangeDepsParams p)
{
    __shared__ RkLds L;
    const uint32_t tid = threadIdx.x;
    for (uint32_t li = blockIdx.x; li < p.n_range_txns; li += gridDim.x) {
        const uint32_t i = p.range_txns[li];
        const uint32_t wmask = witness_mask((uint32_t)(p.lsb[i] >> 1) & 7);
        const uint32_t q0 = p.rng_off[i], q1 = p.rng_off[i + 1];
        if (tid == 0) { L.nslots = 0; L.raw_total = 0; L.overflow = 0; }
        __syncthreads();
        // ---- slots: keys of the ranges (ascending) with entries before i ----
        uint32_t nslots = 0, raw_base = 0;
        for (uint32_t r = q0; r < q1; ++r) {
            const uint32_t ks = p.rng_start[r] + 1, ke = p.rng_end[r];   // keys (s, e]
            for (uint32_t c0 = ks; c0 <= ke; c0 += RK_THREADS) {
                const uint32_t key = c0 + tid;
                uint32_t raw = 0, lo = 0;
                if (key <= ke && key >= p.key_lo && key < p.key_hi) {
                    const uint32_t kk = key - p.key_lo;
                    const uint32_t a = p.seg_start[kk], b = p.seg_end[kk];
                    if (a < b && (p.hist[a] & ENT_TXN_MASK) < i) {
                        uint32_t l = a, h = b;               // pos = first entry with txn >= i
                        while (l < h) { const uint32_t m = (l + h) >> 1; if ((p.hist[m] & ENT_TXN_MASK) < i) l = m + 1; else h = m; }
                        const uint32_t pos = l;
                        lo = a;
                        if (i > p.window) {
                            const uint32_t thr = i - p.window;
                            uint32_t l2 = a, h2 = pos;
                            while (l2 < h2) { const uint32_t m = (l2 + h2) >> 1; if ((p.hist[m] & ENT_TXN_MASK) < thr) l2 = m + 1; else h2 = m; }
                            if (l2 > a) {
                                const uint32_t x = l2 - 1;
                                const uint32_t pw = max(p.pw_local[x], p.pw_carry[x / p.pw_tile]);
                                if (pw > a) lo = pw - 1;
                            }
                        }
                        raw = pos - lo;
                    }
                }
                uint32_t tot;
                const uint32_t flag = raw > 0 ? 1u : 0u;
                const uint32_t sidx = nslots + block_excl_scan(flag, L.wsum, tot);
                const uint32_t nflag = tot;
                const uint32_t rbase = raw_base + block_excl_scan(raw, L.wsum, tot);
                if (flag && sidx < RK_SCAP) {
                    L.slot_key[sidx] = key;
                    L.slot_lo[sidx] = lo;
                    L.slot_base[sidx] = rbase;
                    L.slot_cnt[sidx] = 0;
                }
                nslots += nflag;
                raw_base += tot;
            }
        }
        if (nslots > RK_SCAP) {
            if (!FILL && tid == 0) { rd_overflow(p.status, i); p.cnt_keys[i] = 0; p.cnt_vals_k[i] = 0; p.cnt_k2v[i] = 0; }
            __syncthreads();
            continue;
        }
        if (tid == 0) L.slot_base[nslots] = raw_base;
        __syncthreads();
        // ---- candidates: witnessed entries in key order ----
        const uint32_t raw_total = raw_base;
        uint32_t nwit = 0;
        for (uint32_t c0 = 0; c0 < raw_total; c0 += RK_THREADS) {
            const uint32_t r = c0 + tid;
            bool wit = false;
            uint32_t j = 0, s = 0;
            if (r < raw_total) {
                uint32_t l = 0, h = nslots;                  // slot: last base <= r
                while (h - l > 1) { const uint32_t m = (l + h) >> 1; if (L.slot_base[m] <= r) l = m; else h = m; }
                s = l;
                const uint32_t e = p.hist[L.slot_lo[s] + (r - L.slot_base[s])];
                j = e & ENT_TXN_MASK;
                wit = (wmask >> (e >> ENT_KIND_SHIFT)) & 1u;
            }
            uint32_t tot;
            const uint32_t pos = nwit + block_excl_scan(wit ? 1u : 0u, L.wsum, tot);
            if (wit) {
                atomicAdd(&L.slot_cnt[s], 1u);
                if (pos < RK_CCAP) L.buf[pos] = j;
            }
            nwit += tot;
        }
        if (nwit > RK_CCAP) {
            if (!FILL && tid == 0) { rd_overflow(p.status, i); p.cnt_keys[i] = 0; p.cnt_vals_k[i] = 0; p.cnt_k2v[i] = 0; }
            __syncthreads();
            continue;
        }
        // ---- sort + unique (bitonic over the next power of two) ----
        uint32_t np2 = 1;
        while (np2 < nwit) np2 <<= 1;
        for (uint32_t x = nwit + tid; x < np2; x += RK_THREADS) L.buf[x] = 0xFFFFFFFFu;
        __syncthreads();
        for (uint32_t size = 2; size <= np2; size <<= 1) {
            for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
                for (uint32_t t = tid; t < np2 / 2; t += RK_THREADS) {
                    const uint32_t x = 2 * t - (t & (stride - 1));
                    const uint32_t y = x + stride;
                    const bool up = (x & size) == 0;
                    const uint32_t a = L.buf[x], b = L.buf[y];
                    if ((a > b) == up) { L.buf[x] = b; L.buf[y] = a; }
                }
                __syncthreads();
            }
        }
        // in-place unique
        uint32_t nuniq = 0;
        for (uint32_t c0 = 0; c0 < nwit; c0 += RK_THREADS) {
            const uint32_t x = c0 + tid;
            const uint32_t v = x < nwit ? L.buf[x] : 0u;
            const bool f = x < nwit && (x == 0 || L.buf[x - 1] != v);
            uint32_t tot;
            const uint32_t u = nuniq + block_excl_scan(f ? 1u : 0u, L.wsum, tot);   // contains barriers
            if (f) L.buf[u] = v;
            nuniq += tot;
            __syncthreads();
        }
        // non-empty slots
        uint32_t kc = 0;
        for (uint32_t c0 = 0; c0 < nslots; c0 += RK_THREADS) {
            const uint32_t s = c0 + tid;
            const uint32_t f = (s < nslots && L.slot_cnt[s] > 0) ? 1u : 0u;
            uint32_t tot;
            (void)block_excl_scan(f, L.wsum, tot);
            kc += tot;
        }
        if (!FILL) {
            if (tid == 0) { p.cnt_keys[i] = kc; p.cnt_vals_k[i] = nuniq; p.cnt_k2v[i] = kc + nwit; }
            __syncthreads();
            continue;
        }
        const uint32_t key_base = p.kd_key_off[i], val_base = p.kd_val_off[i], k2v_base = p.kd_k2v_off[i];
        for (uint32_t x = tid; x < nuniq; x += RK_THREADS) p.kd_vals[val_base + x] = L.buf[x];
        // keys + header: non-empty slots in order, end offset = kc + witnessed through the slot
        uint32_t ns = 0, wrun = 0;
        for (uint32_t c0 = 0; c0 < nslots; c0 += RK_THREADS) {
            const uint32_t s = c0 + tid;
            const uint32_t cnt = s < nslots ? L.slot_cnt[s] : 0u;
            uint32_t tot1, tot2;
            const uint32_t idx = ns + block_excl_scan(cnt > 0 ? 1u : 0u, L.wsum, tot1);
            const uint32_t wend = wrun + block_excl_scan(cnt, L.wsum, tot2) + cnt;
            if (cnt > 0) {
                p.kd_keys[key_base + idx] = L.slot_key[s];
                p.kd_k2v[k2v_base + idx] = (int32_t)(kc + wend);
            }
            ns += tot1;
            wrun += tot2;
        }
        // body: re-walk the candidates in key order; rank = index in the unique sorted txnIds
        uint32_t wpos = 0;
        for (uint32_t c0 = 0; c0 < raw_total; c0 += RK_THREADS) {
            const uint32_t r = c0 + tid;
            bool wit = false;
            uint32_t j = 0;
            if (r < raw_total) {
                uint32_t l = 0, h = nslots;
                while (h - l > 1) { const uint32_t m = (l + h) >> 1; if (L.slot_base[m] <= r) l = m; else h = m; }
                const uint32_t e = p.hist[L.slot_lo[l] + (r - L.slot_base[l])];
                j = e & ENT_TXN_MASK;
                wit = (wmask >> (e >> ENT_KIND_SHIFT)) & 1u;
            }
            uint32_t tot;
            const uint32_t pos = wpos + block_excl_scan(wit ? 1u : 0u, L.wsum, tot);
            if (wit) {
                uint32_t l = 0, h = nuniq;
                while (l < h) { const uint32_t m = (l + h) >> 1; if (L.buf[m] < j) l = m + 1; else h = m; }
                p.kd_k2v[k2v_base + kc + pos] = (int32_t)l;
            }
            wpos += tot;
        }
        __syncthreads();
    }
}

} // namespace

void launch_rangedeps_count(const RangeDepsParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t blocks = (p.n + RD_WAVES - 1) / RD_WAVES;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(rangedeps_kernel<false>, dim3(blocks), dim3(RD_WAVES * 64), 0, s, p);
}

void launch_rangedeps_fill(const RangeDepsParams &p, hipStream_t s)
{
    if (p.n == 0) return;
    uint32_t blocks = (p.n + RD_WAVES - 1) / RD_WAVES;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(rangedeps_kernel<true>, dim3(blocks), dim3(RD_WAVES * 64), 0, s, p);
}

void launch_rangekeys_count(const RangeDepsParams &p, hipStream_t s)
{
    if (p.n_range_txns == 0) return;
    uint32_t blocks = p.n_range_txns < 2048 ? p.n_range_txns : 2048;
    hipLaunchKernelGGL(rangekeys_kernel<false>, dim3(blocks), dim3(RK_THREADS), 0, s, p);
}

void launch_rangekeys_fill(const RangeDepsParams &p, hipStream_t s)
{
    if (p.n_range_txns == 0) return;
    uint32_t blocks = p.n_range_txns < 2048 ? p.n_range_txns : 2048;
    hipLaunchKernelGGL(rangekeys_kernel<true>, dim3(blocks), dim3(RK_THREADS), 0, s, p);
}

} // namespace accord
