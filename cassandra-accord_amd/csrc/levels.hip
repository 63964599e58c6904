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
    int32_t rows[SL_CH][SL_LANES];              // the current chunk, a row per txn
    uint32_t bitmap[SL_WORDS];                  // entries before the stripe within SL_WIN
    uint16_t above[SL_WORDS];                   // per bitmap word: set bits in the words above it
    uint32_t ep[64], eo[64];                    // a batch's earlier-chunk edges of the stripe: predecessor, owner
    uint32_t icnt[SL_CH];                       // per txn of the chunk: predecessors inside the chunk
    uint32_t ic[SL_CH];                         // ... the first four as byte offsets
};

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

// Diagnostic build only (-DACCORD_LV_STAMPS, scripts/lv_stamps.py): s_memtime stamps at the
// segment boundaries of the stripe walk, summed per segment over every wave.
#ifdef ACCORD_LV_STAMPS
__device__ unsigned long long g_lv_stamps[16];
#define LV_STAMP(seg)                                                                          \
    do {                                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        unsigned long long t_;                                                                 \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");           \
        __builtin_amdgcn_sched_barrier(0);                                                     \
        lv_sum[seg] += t_ - lv_last;                                                           \
        lv_last = t_;                                                                          \
    } while (0)
#else
#define LV_STAMP(seg) do {} while (0)
#endif

constexpr int SL_PB = 6;                        // edge batches of a chunk loaded at its start

// the in-chunk reads of one txn of the serial step: its F row and up to four predecessors' rows
struct SlReads {
    int32_t f, r0, r1, r2, r3;
};
__device__ __forceinline__ SlReads sl_reads(const SlShared &S, uint32_t i, uint32_t w, uint32_t lane)
{
    return SlReads{S.rows[i & 63u][lane], S.rows[w & 63u][lane], S.rows[(w >> 8) & 63u][lane],
                   S.rows[(w >> 16) & 63u][lane], S.rows[(w >> 24) & 63u][lane]};
}

__global__ __launch_bounds__(64) void lv_stripe_kernel(uint32_t n, uint32_t Z, const uint32_t *__restrict__ pred_off,
                                                       const uint32_t *__restrict__ preds,
                                                       const uint8_t *__restrict__ pred_own, int16_t *__restrict__ D,
                                                       uint32_t *__restrict__ src, uint32_t *__restrict__ info)
{
    __shared__ __attribute__((aligned(16))) SlShared S;
    const uint32_t lane = lane_id();
    const uint32_t s = blockIdx.x;
    const uint32_t a = s * Z, b = min(n, a + Z);

    // ---- sources: the 63 most recent distinct txns in [a - SL_WIN, a) the stripe depends on.  The
    // bitmap of those entries stays: an entry's rank from the top (set bits above it) is its source
    // index, so a predecessor before the stripe finds its lane with two LDS reads.
    const uint32_t lo = a > SL_WIN ? a - SL_WIN : 0u;
    uint32_t sig = SL_NONE;
    for (uint32_t w = lane; w < SL_WORDS; w += 64) S.bitmap[w] = 0u;
    wave_lds_sync();
    if (a > 0) {
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
#pragma unroll
        for (int q = 7; q >= 0; --q) {
            S.above[lane * 8 + q] = (uint16_t)min(rank, 65535u);
            rank += (uint32_t)__popc(wv[q]);
        }
        // lane k >= 1: the entry of rank k - 1, written to ep[] by the lane owning it
        rank = total - incl;
        for (int q = 7; q >= 0 && rank < SL_SRC; --q) {
            uint32_t v = wv[q];
            while (v && rank < SL_SRC) {
                const uint32_t bit = 31u - (uint32_t)__clz(v);
                v &= ~(1u << bit);
                S.ep[rank++] = lo + (lane * 8u + (uint32_t)q) * 32u + bit;
            }
        }
        wave_lds_sync();
        const uint32_t ns = min(total, SL_SRC);
        sig = (lane >= 1 && lane <= ns) ? S.ep[lane - 1] : SL_NONE;
        wave_lds_sync();
    }
    src[(size_t)s * SL_LANES + lane] = sig;

    // ---- the walk, a chunk of 64 txns at a time.  Every earlier chunk's rows are read from HBM: the
    // wait at a chunk's start (for the previous chunk's row stores) is the only one on the chain
    // besides the gathers, and the other waves of the CU fill it.
    const int4 neg4 = make_int4(SL_NEG, SL_NEG, SL_NEG, SL_NEG);
#ifdef ACCORD_LV_STAMPS
    unsigned long long lv_sum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, lv_last = 0, lv_n = 0;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(lv_last)::"memory");
#endif
    for (uint32_t c0 = a; c0 < b; c0 += SL_CH) {
        const uint32_t cnt = min(SL_CH, b - c0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // the previous chunk's rows are in memory
        const uint32_t e0 = pred_off[c0], e1 = pred_off[c0 + cnt];
#pragma unroll
        for (uint32_t q = 0; q < SL_CH * SL_LANES / 4 / 64; ++q) ((int4 *)S.rows)[q * 64 + lane] = neg4;
        S.icnt[lane] = 0u;
        S.ic[lane] = 0u;
        uint32_t pb[SL_PB], ob[SL_PB];                           // the chunk's predecessor lists, up front
#pragma unroll
        for (int q = 0; q < SL_PB; ++q) {
            const uint32_t e = e0 + 64u * q + lane;
            pb[q] = e < e1 ? preds[e] : 0u;
            ob[q] = e < e1 ? pred_own[e] : 0u;
        }
        wave_lds_sync();
        LV_STAMP(0);                                             // chunk start: wait, offsets, pred lists
        for (uint32_t bi = 0, eb = e0; eb < e1; ++bi, eb += 64) {
            const uint32_t e = eb + lane;
            const bool valid = e < e1;
            uint32_t p = 0, o = 0;
#pragma unroll
            for (int q = 0; q < SL_PB; ++q)
                if (bi == (uint32_t)q) { p = pb[q]; o = ob[q]; }
            if (bi >= (uint32_t)SL_PB && valid) { p = preds[e]; o = pred_own[e]; }
            const uint32_t t = c0 + o;
            if (valid && p >= t) atomicOr(&info[2], 1u);   // a predecessor that does not precede its txn
            const bool ok = valid && p < t;
            const bool inch = ok && p >= c0;
            if (inch) {
                const uint32_t slot = atomicAdd(&S.icnt[o], 1u);
                if (slot < 4) ((uint8_t *)S.ic)[o * 4 + slot] = (uint8_t)(p - c0);
            }
            // before the stripe: a source (rank < 63 from the top) folds a 0 into its own column
            if (ok && p < a && p >= lo) {
                const uint32_t x = p - lo, wd = x >> 5, bt = x & 31u;
                const uint32_t r = S.above[wd] + (uint32_t)__popc((S.bitmap[wd] >> bt) >> 1);
                if (r < SL_SRC) atomicMax(&S.rows[o][r + 1], 0);
            }
            // earlier-chunk edges of the stripe: compacted into lanes 0..nf-1, every slot's row gathered at once
            const bool far = ok && !inch && p >= a;
            const uint64_t fm = __ballot(far);
            if (far) {
                const uint32_t f = (uint32_t)__popcll(fm & lanemask_lt());
                S.ep[f] = p;
                S.eo[f] = o;
            }
            const uint32_t nf = (uint32_t)__popcll(fm);
            wave_lds_sync();
            LV_STAMP(1);                                         // classification, sources, compaction
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
            LV_STAMP(3);                                         // gather + fold
        }
        // serial step: the chunk's own predecessors (lane i: txn i's count and first four offsets).
        // Txn i + 1's reads are issued before row i is written: every row it can need but row i is
        // final then, and row i comes from the register holding it.  Two read sets alternate, so no
        // register copy waits for a read.
        const uint32_t icw = S.ic[lane], icn = S.icnt[lane];
        int32_t prev = SL_NEG;
        auto step = [&](uint32_t i, const SlReads &R) {
            const uint32_t w = readlane(icw, (int)i), k = readlane(icn, (int)i), ip = i - 1u;
            int32_t m = R.f;
            m = max(m, k > 0 ? ((w & 63u) == ip ? prev : R.r0) : SL_NEG);
            m = max(m, k > 1 ? (((w >> 8) & 63u) == ip ? prev : R.r1) : SL_NEG);
            m = max(m, k > 2 ? (((w >> 16) & 63u) == ip ? prev : R.r2) : SL_NEG);
            m = max(m, k > 3 ? ((w >> 24) == ip ? prev : R.r3) : SL_NEG);
            if (k > 4) {                                          // more: walk the txn's list
                const uint32_t t = c0 + i, q1 = pred_off[t + 1];
                for (uint32_t q = pred_off[t]; q < q1; ++q) {
                    const uint32_t p = preds[q];
                    if (p >= c0 && p < t) m = max(m, p - c0 == ip ? prev : S.rows[p - c0][lane]);
                }
            }
            prev = sl_fin(m, lane);
        };
        SlReads ra = sl_reads(S, 0, readlane(icw, 0), lane), rb;
        for (uint32_t i = 0; i < cnt; i += 2) {
            rb = sl_reads(S, i + 1, readlane(icw, (int)((i + 1) & 63u)), lane);
            step(i, ra);
            S.rows[i][lane] = prev;
            if (i + 1 >= cnt) break;
            ra = sl_reads(S, i + 2, readlane(icw, (int)((i + 2) & 63u)), lane);
            step(i + 1, rb);
            S.rows[i + 1][lane] = prev;
        }
        wave_lds_sync();
        LV_STAMP(4);                                             // serial step
        for (uint32_t i = 0; i < cnt; ++i) {
            const int32_t v = S.rows[i][lane];
            D[(size_t)(c0 + i) * SL_LANES + lane] = v < 0 ? SL_NEG16 : (int16_t)min(v, 32767);
        }
        wave_lds_sync();
        LV_STAMP(5);                                             // row stores
#ifdef ACCORD_LV_STAMPS
        ++lv_n;
#endif
    }
#ifdef ACCORD_LV_STAMPS
    if (lane == 0) {
        for (int q = 0; q < 6; ++q) atomicAdd(&g_lv_stamps[q], lv_sum[q]);
        atomicAdd(&g_lv_stamps[7], lv_n);
        atomicAdd(&g_lv_stamps[8], 1ull);
    }
#endif
}

// Phase B0: every stripe's source rows gathered into one contiguous block per stripe (R[s][k], 128
// bytes each; -inf rows for absent sources), with each source's stripe (SP[s][k]), so the chain
// reads them at addresses known stripes ahead.
__global__ __launch_bounds__(64) void lv_srcrow_kernel(uint32_t S_, uint32_t Z, const int16_t *__restrict__ D,
                                                       const uint32_t *__restrict__ src, int4 *__restrict__ R,
                                                       uint32_t *__restrict__ SP)
{
    const uint32_t s = blockIdx.x + 1, lane = lane_id();
    if (s >= S_) return;
    const uint32_t sg = src[(size_t)s * SL_LANES + lane];
    const int4 *rp = (const int4 *)(D + (size_t)(sg == SL_NONE ? 0u : sg) * SL_LANES);
    const bool none = sg == SL_NONE;
    const int neg = (int)0x80008000u;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int4 v = rp[q];
        R[((size_t)s * SL_LANES + lane) * 8 + q] =
            make_int4(none ? neg : v.x, none ? neg : v.y, none ? neg : v.z, none ? neg : v.w);
    }
    SP[(size_t)s * SL_LANES + lane] = sg == SL_NONE ? SL_NONE : sg / Z;
}

// X rows kept for the chain in packed int16, relative to the row's maximum: rel = X - base in
// [-16383, 0], or -32768 (no source, or lower than that: the term is dropped -- a lower bound, the
// sweeps complete it).  D entries are in [0, Z <= 16384] or -32768.  With saturating packed adds a
// term with a real path sums to >= -16383 and one without to <= -16384, so the 63 terms take 32
// v_pk_add_i16 (clamp) + 32 v_pk_max_i16 instead of 63 unpacks, adds and maxes.
typedef short sl_short2 __attribute__((ext_vector_type(2)));
constexpr int32_t SL_REL_MIN = -16383;

__device__ __forceinline__ int32_t sl_resolve(const int4 (&r)[8], uint32_t sp, uint32_t s,
                                              const uint32_t (*xr)[SL_LANES / 2], const int32_t *xb)
{
    if (sp == SL_NONE) return SL_NEG;
    const int32_t L0 = (int32_t)(int16_t)(r[0].x & 0xFFFF);
    if (!(sp > 0 && s - sp < SL_XR)) return L0;          // stripe 0 (exact), or too far back: L0
    const int4 *x4 = (const int4 *)xr[sp % SL_XR];
    int4 xv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) xv[q] = x4[q];
    const sl_short2 *xs = (const sl_short2 *)xv, *ds = (const sl_short2 *)r;
    sl_short2 acc0 = {-32768, -32768}, acc1 = {-32768, -32768};
#pragma unroll
    for (int q = 0; q < 32; q += 2) {                     // (term 0 pairs L0 with X_s'[0] = -32768: dropped)
        acc0 = __builtin_elementwise_max(acc0, __builtin_elementwise_add_sat(xs[q], ds[q]));
        acc1 = __builtin_elementwise_max(acc1, __builtin_elementwise_add_sat(xs[q + 1], ds[q + 1]));
    }
    acc0 = __builtin_elementwise_max(acc0, acc1);
    const int32_t rel = max((int32_t)acc0.x, (int32_t)acc0.y);
    return rel >= SL_REL_MIN ? max(L0, xb[sp % SL_XR] + rel) : L0;
}

// Phase B: one wave, the stripes in order; lane k resolves source k of stripe s from the gathered
// rows R[s], loaded four stripes ahead into rotating register sets (no copy that would wait for
// them): only the LDS round trip of the X rows sits on the chain.
__global__ __launch_bounds__(64) void lv_chain_kernel(uint32_t S_, const int4 *__restrict__ R,
                                                      const uint32_t *__restrict__ SP, int32_t *__restrict__ X)
{
    __shared__ __attribute__((aligned(16))) uint32_t xr[SL_XR][SL_LANES / 2];
    __shared__ int32_t xb[SL_XR];
    const uint32_t lane = lane_id();
    X[lane] = SL_NEG;                             // stripe 0 has no sources
    if (S_ < 2) return;
    // unconditional loads (past the end: the last stripe's block again, unused); a conditional
    // load had made the compiler wait for every load in flight at each use
    auto load = [&](uint32_t s, int4 (&r)[8], uint32_t &sp) {
        const uint32_t ss = min(s, S_ - 1u);
#pragma unroll
        for (int q = 0; q < 8; ++q) r[q] = R[((size_t)ss * SL_LANES + lane) * 8 + q];
        sp = SP[(size_t)ss * SL_LANES + lane];
    };
    auto publish = [&](uint32_t s, int32_t A) {
        X[(size_t)s * SL_LANES + lane] = A;
        const int32_t base = (int32_t)readlane(wave_incl_max((uint32_t)(A + (1 << 30))), 63) - (1 << 30);
        const int32_t d = A - base;
        ((int16_t *)xr[s % SL_XR])[lane] = (int16_t)(A == SL_NEG || d < SL_REL_MIN ? -32768 : d);
        if (lane == 0) xb[s % SL_XR] = base;
        wave_lds_sync();
    };
    int4 r0[8], r1[8], r2[8], r3[8];
    uint32_t p0, p1, p2, p3;
    load(1, r0, p0);
    load(2, r1, p1);
    load(3, r2, p2);
    load(4, r3, p3);
    for (uint32_t s = 1; s < S_; s += 4) {
        publish(s, sl_resolve(r0, p0, s, xr, xb));
        load(s + 4, r0, p0);
        if (s + 1 >= S_) break;
        publish(s + 1, sl_resolve(r1, p1, s + 1, xr, xb));
        load(s + 5, r1, p1);
        if (s + 2 >= S_) break;
        publish(s + 2, sl_resolve(r2, p2, s + 2, xr, xb));
        load(s + 6, r2, p2);
        if (s + 3 >= S_) break;
        publish(s + 3, sl_resolve(r3, p3, s + 3, xr, xb));
        load(s + 7, r3, p3);
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
    int4 *R;
    uint32_t *SP;
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
    c += 256;
    t.R = (int4 *)c;
    c += sl_align(S * SL_LANES * 128);
    t.SP = (uint32_t *)c;
    return t;
}

} // namespace

uint32_t levels_stripe_default(uint32_t n)
{
    // about 2048 stripes (eight waves per CU) for large n, never below SL_MIN_STRIPE: config 5 (4 Mi
    // txns) levels in 3.07 ms with 2048-txn stripes, 3.32 with 4096, 4.47 with 1024 (the walk
    // shortens with the stripe, the chain over the stripes lengthens; profiles/r06_levels)
    uint32_t z = SL_MIN_STRIPE;
    while (z < SL_MAX_STRIPE && (uint64_t)z * 2048u < n) z <<= 1;
    return z;
}

size_t levels_striped_temp_bytes(uint32_t n, uint32_t Z)
{
    const size_t S = ((size_t)n + Z - 1) / Z;
    return sl_align((size_t)n * SL_LANES * 2 + 256) + 2 * sl_align(S * SL_LANES * 4) + 256 +
           sl_align(S * SL_LANES * 128) + sl_align(S * SL_LANES * 4);
}

void launch_levels_striped(uint32_t n, const uint32_t *pred_off, const uint32_t *preds, const uint8_t *pred_own,
                           uint32_t *level, uint32_t *info, void *temp, uint32_t Z, uint32_t relax, hipStream_t s)
{
    if (n == 0) return;
    if (Z < SL_MIN_STRIPE || Z > SL_MAX_STRIPE || (Z & (Z - 1))) Z = levels_stripe_default(n);
    const uint32_t S = (n + Z - 1) / Z;
    const SlTemp t = sl_temp(temp, n, Z);
    hipLaunchKernelGGL(lv_stripe_kernel, dim3(S), dim3(64), 0, s, n, Z, pred_off, preds, pred_own, t.D, t.src, info);
    if (S > 1) hipLaunchKernelGGL(lv_srcrow_kernel, dim3(S - 1), dim3(64), 0, s, S, Z, t.D, t.src, t.R, t.SP);
    hipLaunchKernelGGL(lv_chain_kernel, dim3(1), dim3(64), 0, s, S, t.R, t.SP, t.X);
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

#ifdef ACCORD_LV_STAMPS
extern "C" int accord_dbg_lv_stamps(unsigned long long *out)
{
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(accord::g_lv_stamps), 16 * 8) != hipSuccess) return -1;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(accord::g_lv_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
