// Execution levelling by stripes (config 5) -- round 6.
//
// level(T) = 0 without predecessors, else 1 + max level(p) over T's predecessors p < T (the
// reduced WaitingOn DAG of waiting_on.hip; CommandsForKey.notify releases T one round after its
// last dependency, local/CommandsForKey.java:1501-1635).  The serial resolver (lv_staged_kernel)
// walks the whole chain on one workgroup: config 5's longest path is ~0.36 n txns.  Here the chain
// is cut into stripes of Z txns that are walked concurrently, one wave each:
//
//   A (lv_stripe_kernel, a wave per stripe): the stripe's levels as a max-plus function of what
//     lies before it.  Lane 0 carries L0(T), the longest path to T inside the stripe (predecessors
//     before the stripe ignored); lane k >= 1 carries D_k(T), the longest path from source sigma_k
//     to T (-inf when none), sigma_1..63 = the 63 most recent txns before the stripe that its txns
//     depend on.  Rows of 64 int16 per txn go to HBM.
//   B (lv_chain_kernel, one wave): the sources' levels in stripe order,
//     X_s[k] = A(sigma_k) = max(L0(sigma_k), max_j X_{s'}[j] + D_j(sigma_k)), s' = sigma_k's stripe.
//   C (lv_apply_kernel): A(T) = max(L0(T), max_k X_s[k] + D_k(T)) for every T.
//   D (lv_relax_kernel, repeated): A(T) = max(A(T), 1 + max A(p)) until a sweep changes nothing.
//
// Exactness does not rest on the choice of sources: every value A ever holds is the length of a
// real path into T (a lower bound of level(T)), and a vector of lower bounds with A(T) >= 1 + max
// A(p) everywhere equals level() -- by induction in TxnId order, the DAG's topological order.  A
// sweep without a change proves that.  The sources decide only how many sweeps it takes (config 5:
// the entries the sources miss are cold keys' old last Writes; a few sweeps).  If `relax` sweeps do
// not reach the fixpoint, info[3] tells the caller to run the serial resolver instead.
#include "device_common.h"
#include "kernels.h"

namespace accord {

namespace {

constexpr uint32_t SL_LANES = 64;               // lane 0: L0, lanes 1..63: sources
constexpr uint32_t SL_SRC = SL_LANES - 1;
constexpr int32_t SL_NEG = -(1 << 30);          // no path
constexpr int16_t SL_NEG16 = -32768;
constexpr uint32_t SL_WIN = 16384;              // sources: the most recent entries this close before the stripe
constexpr uint32_t SL_WORDS = SL_WIN / 32;      // 512 bitmap words, 8 per lane
constexpr uint32_t SL_CH = 64;                  // txns per chunk of the walk
constexpr uint32_t SL_XR = 32;                  // phase B: stripes of X kept in LDS (>= SL_WIN / 1024 + 2)
constexpr uint32_t SL_NONE = 0xFFFFFFFFu;
constexpr uint32_t SL_MIN_STRIPE = 1024, SL_MAX_STRIPE = 16384;   // D fits int16; phase C blocks of 256

struct SlShared {
    union {
        int32_t rows[SL_CH][SL_LANES];          // the current chunk, a row per txn
        uint32_t bitmap[SL_WORDS];              // source selection (before the walk)
    };
    uint32_t sig[SL_SRC];
    uint32_t ep[128], eo[128];                  // a batch's earlier-chunk edges (0..), edges before the stripe (64..)
    uint32_t icnt[SL_CH];                       // per txn of the chunk: predecessors inside the chunk
    uint32_t ic[SL_CH];                         // ... the first four as byte offsets
};
static_assert(sizeof(int32_t) * SL_CH * SL_LANES >= 4 * SL_WORDS, "bitmap inside the rows");

__device__ __forceinline__ int32_t sl_fin(int32_t m, uint32_t lane)
{
    // lane 0 (L0): 0 without a predecessor inside the stripe; sources: -inf without a path
    return m < 0 ? (lane == 0 ? 0 : SL_NEG) : m + 1;
}

// one gather slot: the row of predecessor lane u of the batch (an earlier chunk of the stripe, HBM)
// for this lane's vector.  The load is unconditional: under a select (an earlier form also served
// predecessors before the stripe here) it was sunk into a branch followed by its own wait, one HBM
// round trip per predecessor on the chain.
__device__ __forceinline__ int32_t sl_gather(const int16_t *__restrict__ D, uint32_t lane, uint32_t pf, int u)
{
    return (int32_t)D[(size_t)readlane(pf, u) * SL_LANES + lane];   // (SL_NEG16 -> SL_NEG at the fold)
}

constexpr int SL_PB = 6;                        // edge batches of a chunk loaded at its start

__global__ __launch_bounds__(64) void lv_stripe_kernel(uint32_t n, uint32_t Z, const uint32_t *__restrict__ pred_off,
                                                       const uint32_t *__restrict__ preds, int16_t *__restrict__ D,
                                                       uint32_t *__restrict__ src, uint32_t *__restrict__ info)
{
    __shared__ __attribute__((aligned(16))) SlShared S;
    const uint32_t lane = lane_id();
    const uint32_t s = blockIdx.x;
    const uint32_t a = s * Z, b = min(n, a + Z);

    // ---- sources: the 63 most recent distinct txns in [a - SL_WIN, a) the stripe depends on
    uint32_t sig = SL_NONE;
    if (a > 0) {
        for (uint32_t w = lane; w < SL_WORDS; w += 64) S.bitmap[w] = 0u;
        wave_lds_sync();
        const uint32_t lo = a > SL_WIN ? a - SL_WIN : 0u;
        const uint32_t e1 = pred_off[b];
        for (uint32_t e = pred_off[a] + lane; e < e1; e += 64) {
            const uint32_t p = preds[e];
            if (p < a && p >= lo) atomicOr(&S.bitmap[(p - lo) >> 5], 1u << ((p - lo) & 31u));
        }
        wave_lds_sync();
        uint32_t wv[8], c = 0;                  // lane l: words [8l, 8l + 8); ranks from the top
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            wv[q] = S.bitmap[lane * 8 + q];
            c += (uint32_t)__popc(wv[q]);
        }
        const uint32_t incl = wave_incl_scan(c), total = readlane(incl, 63);
        uint32_t rank = total - incl;           // set bits in the lanes above (more recent txns)
        for (int q = 7; q >= 0 && rank < SL_SRC; --q) {
            uint32_t v = wv[q];
            while (v && rank < SL_SRC) {
                const uint32_t bit = 31u - (uint32_t)__clz(v);
                v &= ~(1u << bit);
                S.sig[rank++] = lo + (lane * 8u + (uint32_t)q) * 32u + bit;
            }
        }
        wave_lds_sync();
        const uint32_t ns = min(total, SL_SRC);
        sig = (lane >= 1 && lane <= ns) ? S.sig[lane - 1] : SL_NONE;
        wave_lds_sync();
    }
    src[(size_t)s * SL_LANES + lane] = sig;

    // ---- the walk, a chunk of 64 txns at a time.  Every earlier chunk's rows are read from HBM: the
    // wait at a chunk's start (for the previous chunk's row stores) is the only one on the chain
    // besides the gathers, and the other waves of the CU fill it.
    const int4 neg4 = make_int4(SL_NEG, SL_NEG, SL_NEG, SL_NEG);
    for (uint32_t c0 = a; c0 < b; c0 += SL_CH) {
        const uint32_t cnt = min(SL_CH, b - c0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // the previous chunk's rows are in memory
        const uint32_t off_l = pred_off[c0 + min(lane, cnt)];   // lanes >= cnt: the chunk's end
        const uint32_t e1 = pred_off[c0 + cnt];
#pragma unroll
        for (uint32_t q = 0; q < SL_CH * SL_LANES / 4 / 64; ++q) ((int4 *)S.rows)[q * 64 + lane] = neg4;
        S.icnt[lane] = 0u;
        S.ic[lane] = 0u;
        const uint32_t e0 = readlane(off_l, 0);
        uint32_t pb[SL_PB];                                      // the chunk's predecessor lists, up front
#pragma unroll
        for (int q = 0; q < SL_PB; ++q) {
            const uint32_t e = e0 + 64u * q + lane;
            pb[q] = e < e1 ? preds[e] : 0u;
        }
        wave_lds_sync();
        for (uint32_t bi = 0, eb = e0; eb < e1; ++bi, eb += 64) {
            const uint32_t e = eb + lane;
            const bool valid = e < e1;
            uint32_t p = 0;
#pragma unroll
            for (int q = 0; q < SL_PB; ++q)
                if (bi == (uint32_t)q) p = pb[q];
            if (bi >= (uint32_t)SL_PB) p = valid ? preds[e] : 0u;
            uint32_t o = 0;                     // owner: the largest l < cnt with off_l <= e
#pragma unroll
            for (uint32_t step = 32; step >= 1; step >>= 1) {
                const uint32_t c = o + step;
                const uint32_t oc = (uint32_t)__shfl((int)off_l, (int)(c & 63u), 64);
                if (c < cnt && oc <= e) o = c;
            }
            const uint32_t t = c0 + o;
            if (valid && p >= t) atomicOr(&info[2], 1u);   // a predecessor that does not precede its txn
            const bool ok = valid && p < t;
            const bool inch = ok && p >= c0;
            if (inch) {
                const uint32_t slot = atomicAdd(&S.icnt[o], 1u);
                if (slot < 4) ((uint8_t *)S.ic)[o * 4 + slot] = (uint8_t)(p - c0);
            }
            // earlier-chunk edges of the stripe: compacted into lanes 0..nf-1, then every slot's row
            // gathered at once; edges before the stripe: only the lane whose source it is folds a 0
            const bool far = ok && !inch && p >= a, ext = ok && p < a;
            const uint64_t fm = __ballot(far), xm = __ballot(ext);
            if (far) {
                const uint32_t f = (uint32_t)__popcll(fm & lanemask_lt());
                S.ep[f] = p;
                S.eo[f] = o;
            }
            if (ext) {
                const uint32_t f = 64u + (uint32_t)__popcll(xm & lanemask_lt());
                S.ep[f] = p;
                S.eo[f] = o;
            }
            const uint32_t nf = (uint32_t)__popcll(fm), nx = (uint32_t)__popcll(xm);
            wave_lds_sync();
            for (uint32_t u = 0; u < nx; ++u)
                if (S.ep[64 + u] == sig) atomicMax(&S.rows[S.eo[64 + u]][lane], 0);
            // lanes >= nf hold nothing of this batch: the pad row (their slots are gathered, not folded)
            const uint32_t pf = lane < nf ? S.ep[lane] : n, of = lane < nf ? S.eo[lane] : 0u;
            int32_t v[64];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                if (nf > 16u * g) {
#pragma unroll
                    for (int u = 16 * g; u < 16 * g + 16; ++u) v[u] = sl_gather(D, lane, pf, u);
                }
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                if (nf > 16u * g) {
#pragma unroll
                    for (int u = 16 * g; u < 16 * g + 16; ++u)
                        if ((uint32_t)u < nf) atomicMax(&S.rows[readlane(of, u)][lane], v[u] == SL_NEG16 ? SL_NEG : v[u]);
                }
            }
            wave_lds_sync();
        }
        // serial step: the chunk's own predecessors (lane i: txn i's count and first four offsets)
        const uint32_t icw = S.ic[lane], icn = S.icnt[lane];
        for (uint32_t i = 0; i < cnt; ++i) {
            const uint32_t w = readlane(icw, (int)i), k = readlane(icn, (int)i);
            int32_t m = S.rows[i][lane];
            const int32_t r0 = S.rows[w & 63u][lane], r1 = S.rows[(w >> 8) & 63u][lane];
            const int32_t r2 = S.rows[(w >> 16) & 63u][lane], r3 = S.rows[(w >> 24) & 63u][lane];
            m = max(m, k > 0 ? r0 : SL_NEG);
            m = max(m, k > 1 ? r1 : SL_NEG);
            m = max(m, k > 2 ? r2 : SL_NEG);
            m = max(m, k > 3 ? r3 : SL_NEG);
            if (k > 4) {                                          // more: walk the txn's list
                const uint32_t t = c0 + i, q1 = pred_off[t + 1];
                for (uint32_t q = pred_off[t]; q < q1; ++q) {
                    const uint32_t p = preds[q];
                    if (p >= c0 && p < t) m = max(m, S.rows[p - c0][lane]);
                }
            }
            S.rows[i][lane] = sl_fin(m, lane);
        }
        wave_lds_sync();
        for (uint32_t i = 0; i < cnt; ++i) {
            const int32_t v = S.rows[i][lane];
            D[(size_t)(c0 + i) * SL_LANES + lane] = v < 0 ? SL_NEG16 : (int16_t)min(v, 32767);
        }
        wave_lds_sync();
    }
}

// Phase B: one wave, the stripes in order; lane k resolves source k of stripe s.  Rows and source
// ids are loaded a stripe ahead into alternating register sets (no copy that would wait for them):
// only the X reads of the previous stripes sit on the chain.
__device__ __forceinline__ void sl_row(const int16_t *__restrict__ D, uint32_t sg, int4 (&r)[8])
{
    const int4 *rp = (const int4 *)(D + (size_t)(sg == SL_NONE ? 0u : sg) * SL_LANES);
#pragma unroll
    for (int q = 0; q < 8; ++q) r[q] = rp[q];
}

__device__ __forceinline__ int32_t sl_resolve(const int4 (&r)[8], uint32_t sg, uint32_t s, uint32_t Z,
                                              const int32_t (*xr)[SL_LANES])
{
    if (sg == SL_NONE) return SL_NEG;
    const int16_t *rv = (const int16_t *)r;
    int32_t A = rv[0];
    const uint32_t sp = sg / Z;
    // (a source more than SL_XR stripes back keeps L0: a lower bound, the sweeps complete it)
    if (sp > 0 && s - sp < SL_XR) {
        // the whole X row read first and every term in arithmetic form (x + d, d = -inf when no
        // path; X >= -2^30, so the sum stays above INT_MIN): a read under a select had been sunk
        // into a branch of its own with its own wait
        const int4 *x4 = (const int4 *)xr[sp % SL_XR];
        int4 xv[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) xv[q] = x4[q];
        const int32_t *x = (const int32_t *)xv;
        int32_t A2 = SL_NEG;
#pragma unroll
        for (int j = 1; j < (int)SL_LANES; ++j) {
            const int32_t d = rv[j];
            const int32_t t = x[j] + (d == SL_NEG16 ? SL_NEG : d);
            if (j & 1) A = max(A, t); else A2 = max(A2, t);
        }
        A = max(A, A2);
    }
    return A;
}

__global__ __launch_bounds__(64) void lv_chain_kernel(uint32_t S_, uint32_t Z, const int16_t *__restrict__ D,
                                                      const uint32_t *__restrict__ src, int32_t *__restrict__ X)
{
    __shared__ __attribute__((aligned(16))) int32_t xr[SL_XR][SL_LANES];
    const uint32_t lane = lane_id();
    X[lane] = SL_NEG;                             // stripe 0 has no sources
    auto sid = [&](uint32_t s) { return s < S_ ? src[(size_t)s * SL_LANES + lane] : SL_NONE; };
    uint32_t ga = sid(1), gb = sid(2);
    int4 ra[8], rb[8];
    sl_row(D, ga, ra);
    for (uint32_t s = 1; s < S_; s += 2) {
        // stripe s from set a; set b (stripe s + 1) is in flight
        sl_row(D, gb, rb);
        const uint32_t gc = sid(s + 2);
        int32_t A = sl_resolve(ra, ga, s, Z, xr);
        xr[s % SL_XR][lane] = A;
        X[(size_t)s * SL_LANES + lane] = A;
        wave_lds_sync();
        if (s + 1 >= S_) break;
        // stripe s + 1 from set b; set a takes stripe s + 2
        sl_row(D, gc, ra);
        const uint32_t gd = sid(s + 3);
        A = sl_resolve(rb, gb, s + 1, Z, xr);
        xr[(s + 1) % SL_XR][lane] = A;
        X[(size_t)(s + 1) * SL_LANES + lane] = A;
        wave_lds_sync();
        ga = gc;
        gb = gd;
    }
}

// Phase C: every txn from its row and its stripe's X (a block of 256 txns lies in one stripe).
// Block 0 also clears the sweeps' change flags.
__global__ __launch_bounds__(256) void lv_apply_kernel(uint32_t n, uint32_t Z, const int16_t *__restrict__ D,
                                                       const int32_t *__restrict__ X, uint32_t *__restrict__ level,
                                                       uint32_t *__restrict__ flags, uint32_t nflags)
{
    __shared__ int32_t xs[SL_LANES];
    if (blockIdx.x == 0 && threadIdx.x < nflags) flags[threadIdx.x] = 0u;
    const uint32_t t0 = blockIdx.x * 256u, s = t0 / Z;
    if (threadIdx.x < SL_LANES) xs[threadIdx.x] = X[(size_t)s * SL_LANES + threadIdx.x];
    __syncthreads();
    const uint32_t t = t0 + threadIdx.x;
    if (t >= n) return;
    int4 r[8];
    const int4 *rp = (const int4 *)(D + (size_t)t * SL_LANES);
#pragma unroll
    for (int q = 0; q < 8; ++q) r[q] = rp[q];
    const int16_t *rv = (const int16_t *)r;
    int32_t A = rv[0];
    if (s > 0) {
#pragma unroll
        for (int j = 1; j < (int)SL_LANES; ++j) {
            const int32_t d = rv[j];
            A = max(A, d == SL_NEG16 ? SL_NEG : xs[j] + d);
        }
    }
    level[t] = (uint32_t)max(A, 0);
}

// Phase D: one sweep, A(T) = max(A(T), 1 + max A(p)), in place (values only grow and stay lower
// bounds, so reading a neighbour's old or new value is equally valid).  A sweep after one without
// a change exits at once.
__global__ __launch_bounds__(256) void lv_relax_kernel(uint32_t n, const uint32_t *__restrict__ pred_off,
                                                       const uint32_t *__restrict__ preds, uint32_t *level,
                                                       uint32_t *__restrict__ flags, uint32_t it,
                                                       uint32_t *__restrict__ info)
{
    if (it > 0 && flags[it - 1] == 0u) return;
    bool changed = false, bad = false;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) {
        const uint32_t e0 = pred_off[t], e1 = pred_off[t + 1];
        if (e0 == e1) continue;
        uint32_t m = 0;
        for (uint32_t e = e0; e < e1; ++e) {
            const uint32_t p = preds[e];
            if (p < t) m = max(m, level[p] + 1u);
            else bad = true;
        }
        if (m > level[t]) {
            level[t] = m;
            changed = true;
        }
    }
    if (__any(changed) && lane_id() == 0) flags[it] = 1u;
    if (bad) info[2] = 1u;
}

__global__ __launch_bounds__(256) void lv_max_kernel(uint32_t n, const uint32_t *__restrict__ level,
                                                     const uint32_t *__restrict__ flags, uint32_t last,
                                                     uint32_t *__restrict__ info)
{
    uint32_t m = 0;
    for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < n; t += gridDim.x * blockDim.x) m = max(m, level[t]);
    m = readlane(wave_incl_max(m), 63);
    if (lane_id() == 0 && m) atomicMax(&info[1], m);
    if (blockIdx.x == 0 && threadIdx.x == 0 && flags[last]) info[3] = 1u;
}

struct SlTemp {
    int16_t *D;
    uint32_t *src;
    int32_t *X;
    uint32_t *flags;
};

inline size_t sl_align(size_t x) { return (x + 255) & ~(size_t)255; }

SlTemp sl_temp(void *temp, uint32_t n, uint32_t Z)
{
    const size_t S = ((size_t)n + Z - 1) / Z;
    char *c = (char *)temp;
    SlTemp t;
    t.D = (int16_t *)c;
    c += sl_align((size_t)n * SL_LANES * 2 + 256);
    t.src = (uint32_t *)c;
    c += sl_align(S * SL_LANES * 4);
    t.X = (int32_t *)c;
    c += sl_align(S * SL_LANES * 4);
    t.flags = (uint32_t *)c;
    return t;
}

} // namespace

uint32_t levels_stripe_default(uint32_t n)
{
    // about 512 stripes (two waves per CU) for large n, never below SL_MIN_STRIPE
    uint32_t z = SL_MIN_STRIPE;
    while (z < SL_MAX_STRIPE && (uint64_t)z * 512u < n) z <<= 1;
    return z;
}

size_t levels_striped_temp_bytes(uint32_t n, uint32_t Z)
{
    const size_t S = ((size_t)n + Z - 1) / Z;
    return sl_align((size_t)n * SL_LANES * 2 + 256) + 2 * sl_align(S * SL_LANES * 4) + 256;
}

void launch_levels_striped(uint32_t n, const uint32_t *pred_off, const uint32_t *preds, uint32_t *level,
                           uint32_t *info, void *temp, uint32_t Z, uint32_t relax, hipStream_t s)
{
    if (n == 0) return;
    if (Z < SL_MIN_STRIPE || Z > SL_MAX_STRIPE || (Z & (Z - 1))) Z = levels_stripe_default(n);
    const uint32_t S = (n + Z - 1) / Z;
    const SlTemp t = sl_temp(temp, n, Z);
    hipLaunchKernelGGL(lv_stripe_kernel, dim3(S), dim3(64), 0, s, n, Z, pred_off, preds, t.D, t.src, info);
    hipLaunchKernelGGL(lv_chain_kernel, dim3(1), dim3(64), 0, s, S, Z, t.D, t.src, t.X);
    hipLaunchKernelGGL(lv_apply_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, Z, t.D, t.X, level, t.flags, 64u);
    launch_levels_sweeps(n, pred_off, preds, level, info, temp, Z, 0, relax, s);
}

void launch_levels_sweeps(uint32_t n, const uint32_t *pred_off, const uint32_t *preds, uint32_t *level,
                          uint32_t *info, void *temp, uint32_t Z, uint32_t from, uint32_t to, hipStream_t s)
{
    if (n == 0) return;
    if (Z < SL_MIN_STRIPE || Z > SL_MAX_STRIPE || (Z & (Z - 1))) Z = levels_stripe_default(n);
    to = std::max<uint32_t>(from + 1u, std::min<uint32_t>(to, 64u));
    const SlTemp t = sl_temp(temp, n, Z);
    const uint32_t rb = std::min<uint32_t>((n + 255) / 256, 4096u);
    for (uint32_t it = from; it < to; ++it)
        hipLaunchKernelGGL(lv_relax_kernel, dim3(rb), dim3(256), 0, s, n, pred_off, preds, level, t.flags, it, info);
    (void)hipMemsetAsync(info + 1, 0, 4, s);
    (void)hipMemsetAsync(info + 3, 0, 4, s);
    hipLaunchKernelGGL(lv_max_kernel, dim3(std::min<uint32_t>((n + 255) / 256, 1024u)), dim3(256), 0, s, n, level,
                       t.flags, to - 1, info);
}

} // namespace accord
