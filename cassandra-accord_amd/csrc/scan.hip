// Exclusive prefix sums of u32 counts (CSR offsets of the per-txn PartialDeps, radix digit offsets,
// stream compaction).  One launch per scan, up to four arrays of the same length at once: a
// single-pass scan with decoupled look-back.
//
//   * a block takes the next tile id from a counter (ids follow start order, so a block only ever
//     waits on tiles whose blocks are already running), reduces its 4096 items per array and
//     publishes the aggregate; wave 0 then walks back over the predecessors' status words 64 tiles
//     at a time until it meets an inclusive prefix, publishes its own inclusive prefix, and the
//     block writes its tile of offsets;
//   * a status word is one 8-byte agent-scope atomic (flag | epoch | value), so no payload has to be
//     ordered behind it (MI355X_MICROARCH.md, inter-workgroup visibility: the 8-B granule);
//   * the state buffer is self-resetting: it must be zero when allocated (DevBuf::ensure_zeroed).
//     The tile counter and the epoch share one 64-bit word, so a block draws its id and learns the
//     launch's epoch in one atomic; the block that draws the last id (every other block has drawn
//     one already) rewinds the counter and advances the epoch for the next launch.  Status words
//     of an older epoch read as unpublished.  30-bit epochs: the store re-zeroes the buffer long
//     before they wrap (accord_deps_compute);
//   * values are 32 bits: a prefix that reaches 2^32 is published with the overflow flag, which
//     propagates, and the total reports >= 2^32 (every caller checks its totals);
//   * a look-back that spins for too long falls back to summing the predecessors' inputs itself,
//     so termination does not depend on dispatch order;
//   * counters after the header (ScanCounters) accumulate the look-back spins and fallbacks of
//     every launch, for the store's profile.
// Totals are carried in u64 so an overflow of the u32 offset space is detectable on the host.
#include "device_common.h"
#include "kernels.h"

#include <cstdio>
#include <cstdlib>

namespace accord {

namespace {
constexpr int SC_THREADS = 256;
constexpr int SC_ITEMS = 16;
constexpr uint32_t SC_TILE = SC_THREADS * SC_ITEMS;
constexpr int SC_MAX_ARRAYS = 4;

// status word: flag (2 bits: 0 none, 1 aggregate, 2 inclusive prefix, 3 inclusive prefix that
// reached 2^32) | epoch (30 bits) | value (32 bits)
constexpr uint32_t ST_EPOCH_MASK = (1u << 30) - 1;
__device__ __forceinline__ uint64_t st_make(uint32_t flag, uint32_t epoch, uint32_t v)
{
    return ((uint64_t)flag << 62) | ((uint64_t)(epoch & ST_EPOCH_MASK) << 32) | v;
}

struct ScanHeader {
    unsigned long long ctl;      // next tile id (low 32 bits, 0 between launches) | epoch of the previous launch
    unsigned long long pad;
    ScanCounters counters;       // at scan_counters(temp)
};
static_assert(sizeof(ScanHeader) == 32, "scan header");

struct ScanArgs {
    const uint32_t *in[SC_MAX_ARRAYS];
    uint32_t *out[SC_MAX_ARRAYS];
    unsigned long long *total[SC_MAX_ARRAYS];
    SpecCheck spec;
    uint32_t has_spec;
};

// the speculative fill's check, by the thread that writes the totals (kernels.h SpecCheck)
__device__ __forceinline__ void spec_eval(const ScanArgs &a, const uint64_t *tot)
{
    const SpecCheck &c = a.spec;
    const bool bad = tot[0] > c.cap[0] || tot[1] > c.cap[1] || tot[2] > c.cap[2] || c.status->first != ~0ull ||
                     c.status->overflow || (c.xtot && *c.xtot > c.cap_x);
    *c.abort = bad ? 1u : 0u;
}

__device__ __forceinline__ uint64_t ld_status(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_status(uint64_t *p, uint64_t v)
{
    (void)__hip_atomic_exchange(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr uint64_t OVF = 1ull << 32;

// DIRECT (every array 16-byte aligned): a thread loads its 16 consecutive items with four 16-byte
// loads and keeps them in registers -- no LDS staging of the tile (48 KB of LDS for three arrays
// had held the kernel to a few blocks per CU)
template <int NA, bool DIRECT>
__global__ __launch_bounds__(SC_THREADS) void sc_single_pass(ScanArgs a, uint32_t n, uint32_t tiles,
                                                             ScanHeader *__restrict__ hdr, uint64_t *__restrict__ status)
{
    __shared__ uint32_t s_id, s_epoch;
    __shared__ uint64_t s_wsum[NA][SC_THREADS / 64];
    __shared__ uint64_t s_excl[NA];
    __shared__ uint32_t tile[DIRECT ? 1 : NA][DIRECT ? 1 : SC_TILE];
    uint32_t vals[DIRECT ? NA : 1][DIRECT ? SC_ITEMS : 1];
    const uint32_t tid = threadIdx.x, w = wave_id(), lane = lane_id();
    if (tid == 0) {
        const unsigned long long old = atomicAdd(&hdr->ctl, 1ull);
        s_id = (uint32_t)old;
        s_epoch = ((uint32_t)(old >> 32) + 1u) & ST_EPOCH_MASK;
    }
    __syncthreads();
    const uint32_t b = s_id, e = s_epoch;
    if (b >= tiles) return;      // only a corrupted state buffer hands out more ids than tiles
    const uint32_t base = b * SC_TILE;

    // load the tile (coalesced), then each thread owns 16 consecutive items
    uint64_t local[NA];
    const uint32_t mine = base + tid * SC_ITEMS;       // DIRECT: this thread's first item
    if constexpr (DIRECT) {
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            if (mine + SC_ITEMS <= n) {
                const uint4 *q = reinterpret_cast<const uint4 *>(a.in[k] + mine);
#pragma unroll
                for (int j = 0; j < SC_ITEMS / 4; ++j) {
                    const uint4 v = q[j];
                    vals[k][4 * j] = v.x; vals[k][4 * j + 1] = v.y; vals[k][4 * j + 2] = v.z; vals[k][4 * j + 3] = v.w;
                }
            } else {
#pragma unroll
                for (int j = 0; j < SC_ITEMS; ++j) vals[k][j] = mine + j < n ? a.in[k][mine + j] : 0u;
            }
            uint64_t acc = 0;
#pragma unroll
            for (int j = 0; j < SC_ITEMS; ++j) acc += vals[k][j];
            local[k] = acc;
        }
    } else {
#pragma unroll
        for (int k = 0; k < NA; ++k) {
#pragma unroll
            for (int j = 0; j < SC_ITEMS; ++j) {
                const uint32_t idx = base + j * SC_THREADS + tid;
                tile[k][j * SC_THREADS + tid] = idx < n ? a.in[k][idx] : 0u;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            uint64_t acc = 0;
#pragma unroll
            for (int j = 0; j < SC_ITEMS; ++j) acc += tile[k][tid * SC_ITEMS + j];
            local[k] = acc;
        }
    }
    // block scan of the per-thread sums
    uint64_t incl[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        incl[k] = wave_incl_scan64(local[k]);
        if (lane == 63) s_wsum[k][w] = incl[k];
    }
    __syncthreads();
    uint64_t agg[NA], woff[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        uint64_t t = 0, o = 0;
#pragma unroll
        for (uint32_t q = 0; q < SC_THREADS / 64; ++q) {
            if (q < w) o += s_wsum[k][q];
            t += s_wsum[k][q];
        }
        agg[k] = t;
        woff[k] = o;
    }
    // publish + look back (wave 0)
    if (w == 0) {
        uint64_t excl[NA];
#pragma unroll
        for (int k = 0; k < NA; ++k) excl[k] = 0;
        if (b == 0) {
#pragma unroll
            for (int k = 0; k < NA; ++k)
                if (lane == 0) st_status(&status[(size_t)k * tiles + 0], st_make(agg[k] >= OVF ? 3 : 2, e, (uint32_t)agg[k]));
        } else {
            // an aggregate that alone reaches 2^32 makes every later prefix overflow: publish it as such
#pragma unroll
            for (int k = 0; k < NA; ++k)
                if (lane == 0) st_status(&status[(size_t)k * tiles + b], st_make(agg[k] >= OVF ? 3 : 1, e, (uint32_t)agg[k]));
            int32_t j = (int32_t)b - 1;       // walk back from here
            uint32_t spins = 0, spins_all = 0;
            bool done = false;
            while (!done) {
                const int32_t t = j - (int32_t)lane;
                // a tile counts once all its arrays carry the same flag of this epoch (an
                // aggregate, or an inclusive prefix, overflowed or not); tiles before 0 are an
                // empty prefix
                uint32_t gmin = 2, gmax = 2;
                uint64_t val[NA];
                bool ovf[NA];
#pragma unroll
                for (int k = 0; k < NA; ++k) {
                    val[k] = 0;
                    ovf[k] = false;
                    if (t >= 0) {
                        const uint64_t sw = ld_status(&status[(size_t)k * tiles + t]);
                        const bool cur = (uint32_t)((sw >> 32) & ST_EPOCH_MASK) == e;
                        const uint32_t f = cur ? (uint32_t)(sw >> 62) : 0u;
                        const uint32_t g = f > 2 ? 2u : f;
                        gmin = min(gmin, g);
                        gmax = k == 0 ? g : max(gmax, g);
                        val[k] = (uint32_t)sw;
                        ovf[k] = f == 3;
                    }
                }
                const uint32_t flag = gmin == gmax ? gmin : 0u;
                const uint64_t pm = __ballot(flag == 2);          // lanes holding an inclusive prefix
                const uint64_t nm = __ballot(flag == 0);          // lanes not published yet
                const uint32_t first_p = pm ? (uint32_t)__builtin_ctzll(pm) : 64u;
                const uint64_t below = first_p >= 64 ? ~0ull : ((1ull << first_p) - 1);
                if (nm & below) {                                  // a predecessor is still working
                    ++spins_all;
                    if (++spins > (1u << 20)) break;               // defensive: fall back below
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                spins = 0;
#pragma unroll
                for (int k = 0; k < NA; ++k) {
                    const bool mine = lane <= first_p;
                    uint64_t v = mine ? val[k] : 0ull;
                    if (__any(mine && ovf[k])) v = lane == 0 ? OVF : 0ull;   // the prefix reached 2^32
#pragma unroll
                    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
                    excl[k] += v;
                }
                if (first_p < 64) done = true;
                else j -= 64;
            }
            if (!done) {                       // dispatch order gave no progress: sum the inputs
#pragma unroll
                for (int k = 0; k < NA; ++k) {
                    uint64_t v = 0;
                    for (uint32_t x = lane; x < base; x += 64) v += a.in[k][x];
#pragma unroll
                    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
                    excl[k] = v;
                }
            }
#pragma unroll
            for (int k = 0; k < NA; ++k) {
                const uint64_t inc = excl[k] + agg[k];
                if (lane == 0) st_status(&status[(size_t)k * tiles + b], st_make(inc >= OVF ? 3 : 2, e, (uint32_t)inc));
            }
            if (lane == 0 && (spins_all || !done)) {
                if (spins_all) atomicAdd(&hdr->counters.spins, (unsigned long long)spins_all);
                if (!done) atomicAdd(&hdr->counters.fallbacks, 1ull);
            }
        }
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < NA; ++k) s_excl[k] = excl[k];
        }
    }
    __syncthreads();
    if constexpr (DIRECT) {
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            uint64_t run = s_excl[k] + woff[k] + incl[k] - local[k];
#pragma unroll
            for (int j = 0; j < SC_ITEMS; ++j) {
                const uint32_t v = vals[k][j];
                vals[k][j] = (uint32_t)run;
                run += v;
            }
            if (mine + SC_ITEMS <= n) {
                uint4 *q = reinterpret_cast<uint4 *>(a.out[k] + mine);
#pragma unroll
                for (int j = 0; j < SC_ITEMS / 4; ++j)
                    q[j] = make_uint4(vals[k][4 * j], vals[k][4 * j + 1], vals[k][4 * j + 2], vals[k][4 * j + 3]);
            } else {
#pragma unroll
                for (int j = 0; j < SC_ITEMS; ++j)
                    if (mine + j < n) a.out[k][mine + j] = vals[k][j];
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            uint64_t run = s_excl[k] + woff[k] + incl[k] - local[k];
#pragma unroll
            for (int j = 0; j < SC_ITEMS; ++j) {
                const uint32_t v = tile[k][tid * SC_ITEMS + j];
                tile[k][tid * SC_ITEMS + j] = (uint32_t)run;
                run += v;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NA; ++k) {
#pragma unroll
            for (int j = 0; j < SC_ITEMS; ++j) {
                const uint32_t idx = base + j * SC_THREADS + tid;
                if (idx < n) a.out[k][idx] = tile[k][j * SC_THREADS + tid];
            }
        }
    }
    if (b == tiles - 1 && tid == 0) {
        uint64_t tt[NA];
#pragma unroll
        for (int k = 0; k < NA; ++k) {
            const uint64_t tot = s_excl[k] + agg[k];
            tt[k] = tot;
            a.out[k][n] = (uint32_t)tot;
            if (a.total[k]) *a.total[k] = tot;
        }
        if constexpr (NA == 3)
            if (a.has_spec) spec_eval(a, tt);
        // every block has drawn its id (this one drew the last): rewind for the next launch
        __hip_atomic_store(&hdr->ctl, (unsigned long long)e << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
// n <= one tile: the same block scan without the tile id draw, the status publication or the look
// back -- three device-scope atomics fewer on a small batch's many short scans (the state buffer's
// epoch is untouched: the next multi-tile launch continues from it)
template <int NA>
__global__ __launch_bounds__(SC_THREADS) void sc_one_tile(ScanArgs a, uint32_t n)
{
    __shared__ uint64_t s_wsum[NA][SC_THREADS / 64];
    __shared__ uint32_t tile[NA][SC_TILE];
    const uint32_t tid = threadIdx.x, w = wave_id(), lane = lane_id();
#pragma unroll
    for (int k = 0; k < NA; ++k)
#pragma unroll
        for (int j = 0; j < SC_ITEMS; ++j) {
            const uint32_t idx = j * SC_THREADS + tid;
            tile[k][idx] = idx < n ? a.in[k][idx] : 0u;
        }
    __syncthreads();
    uint64_t local[NA], incl[NA], tt[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        uint64_t acc = 0;
#pragma unroll
        for (int j = 0; j < SC_ITEMS; ++j) acc += tile[k][tid * SC_ITEMS + j];
        local[k] = acc;
        incl[k] = wave_incl_scan64(acc);
        if (lane == 63) s_wsum[k][w] = incl[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        uint64_t o = 0, t = 0;
#pragma unroll
        for (uint32_t q = 0; q < SC_THREADS / 64; ++q) {
            if (q < w) o += s_wsum[k][q];
            t += s_wsum[k][q];
        }
        uint64_t run = o + incl[k] - local[k];
#pragma unroll
        for (int j = 0; j < SC_ITEMS; ++j) {
            const uint32_t v = tile[k][tid * SC_ITEMS + j];
            tile[k][tid * SC_ITEMS + j] = (uint32_t)run;
            run += v;
        }
        tt[k] = t;
        if (tid == 0) {
            a.out[k][n] = (uint32_t)t;
            if (a.total[k]) *a.total[k] = t;
        }
    }
    if constexpr (NA == 3)
        if (tid == 0 && a.has_spec) spec_eval(a, tt);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NA; ++k)
#pragma unroll
        for (int j = 0; j < SC_ITEMS; ++j) {
            const uint32_t idx = j * SC_THREADS + tid;
            if (idx < n) a.out[k][idx] = tile[k][idx];
        }
}
// n <= 1024 (a small batch's per-txn counts): four consecutive items per thread in registers --
// a fraction of sc_one_tile's code (its 16 items per array are unrolled whatever n is, ~1,150
// instructions for three arrays), which a short launch on a cold CU pays for in instruction fetch
constexpr uint32_t SC_SMALL = SC_THREADS * 4;
template <int NA>
__global__ __launch_bounds__(SC_THREADS) void sc_small(ScanArgs a, uint32_t n)
{
    __shared__ uint64_t s_wsum[NA][SC_THREADS / 64];
    const uint32_t tid = threadIdx.x, w = wave_id(), lane = lane_id(), first = tid * 4;
    uint32_t v[NA][4];
    uint64_t local[NA], incl[NA], tt[NA];
#pragma unroll
    for (int k = 0; k < NA; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[k][j] = first + j < n ? a.in[k][first + j] : 0u;
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        local[k] = (uint64_t)v[k][0] + v[k][1] + v[k][2] + v[k][3];
        incl[k] = wave_incl_scan64(local[k]);
        if (lane == 63) s_wsum[k][w] = incl[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NA; ++k) {
        uint64_t o = 0, t = 0;
#pragma unroll
        for (uint32_t q = 0; q < SC_THREADS / 64; ++q) {
            if (q < w) o += s_wsum[k][q];
            t += s_wsum[k][q];
        }
        uint64_t run = o + incl[k] - local[k];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (first + j < n) a.out[k][first + j] = (uint32_t)run;
            run += v[k][j];
        }
        tt[k] = t;
        if (tid == 0) {
            a.out[k][n] = (uint32_t)t;
            if (a.total[k]) *a.total[k] = t;
        }
    }
    if constexpr (NA == 3)
        if (tid == 0 && a.has_spec) spec_eval(a, tt);
}
__global__ __launch_bounds__(256) void fill_words_kernel(FillList L)
{
    const FillDesc d = L.d[blockIdx.y];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < d.words; i += gridDim.x * blockDim.x) d.p[i] = d.value;
}
__global__ __launch_bounds__(256) void copy_words_kernel(CopyList L)
{
    const CopyDesc d = L.d[blockIdx.y];
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < d.words; i += gridDim.x * blockDim.x) d.dst[i] = d.src[i];
}
// fills and copies in one launch (a pipeline's small initialisations): blockIdx.y over the fills,
// then the copies
__global__ __launch_bounds__(256) void init_words_kernel(FillList F, CopyList L)
{
    const uint32_t y = blockIdx.y;
    if (y < F.nd) {
        const FillDesc d = F.d[y];
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < d.words; i += gridDim.x * blockDim.x) d.p[i] = d.value;
    } else {
        const CopyDesc d = L.d[y - F.nd];
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < d.words; i += gridDim.x * blockDim.x) d.dst[i] = d.src[i];
    }
}
} // namespace

void list_capacity_exceeded(const char *what)
{
    std::fprintf(stderr, "accord_deps: %s capacity exceeded (a build bug: raise its CAP)\n", what);
    std::abort();
}

void launch_init_words(const FillList &F, const CopyList &L, hipStream_t s)
{
    uint32_t mx = 0;
    for (uint32_t k = 0; k < F.nd; ++k) mx = F.d[k].words > mx ? F.d[k].words : mx;
    for (uint32_t k = 0; k < L.nd; ++k) mx = L.d[k].words > mx ? L.d[k].words : mx;
    if (F.nd + L.nd == 0 || mx == 0) return;
    uint32_t bx = (mx + 255) / 256;
    if (bx > 1024) bx = 1024;
    hipLaunchKernelGGL(init_words_kernel, dim3(bx, F.nd + L.nd), dim3(256), 0, s, F, L);
}

void launch_copy_words(const CopyList &L, hipStream_t s)
{
    uint32_t mx = 0;
    for (uint32_t k = 0; k < L.nd; ++k) mx = L.d[k].words > mx ? L.d[k].words : mx;
    if (L.nd == 0 || mx == 0) return;
    uint32_t bx = (mx + 255) / 256;
    if (bx > 2048) bx = 2048;
    hipLaunchKernelGGL(copy_words_kernel, dim3(bx, L.nd), dim3(256), 0, s, L);
}

void launch_fill_words(const FillList &L, hipStream_t s)
{
    uint32_t mx = 0;
    for (uint32_t k = 0; k < L.nd; ++k) mx = L.d[k].words > mx ? L.d[k].words : mx;
    if (L.nd == 0 || mx == 0) return;
    uint32_t bx = (mx + 255) / 256;
    if (bx > 1024) bx = 1024;
    hipLaunchKernelGGL(fill_words_kernel, dim3(bx, L.nd), dim3(256), 0, s, L);
}

size_t scan_temp_bytes(uint32_t n)
{
    const uint32_t tiles = (n + SC_TILE - 1) / SC_TILE;
    return sizeof(ScanHeader) + (size_t)SC_MAX_ARRAYS * (tiles ? tiles : 1) * sizeof(uint64_t);
}

void exclusive_scan_multi(int na, const uint32_t *const *in, uint32_t *const *out, unsigned long long *const *total,
                          uint32_t n, void *temp, hipStream_t s, const SpecCheck *spec)
{
    uint32_t tiles = (n + SC_TILE - 1) / SC_TILE;
    if (tiles == 0) tiles = 1;
    ScanArgs a{};
    for (int k = 0; k < na; ++k) { a.in[k] = in[k]; a.out[k] = out[k]; a.total[k] = total[k]; }
    if (spec && na == 3) { a.spec = *spec; a.has_spec = 1u; }
    if (n <= SC_SMALL) {
        switch (na) {
        case 1: hipLaunchKernelGGL(sc_small<1>, dim3(1), dim3(SC_THREADS), 0, s, a, n); break;
        case 2: hipLaunchKernelGGL(sc_small<2>, dim3(1), dim3(SC_THREADS), 0, s, a, n); break;
        case 3: hipLaunchKernelGGL(sc_small<3>, dim3(1), dim3(SC_THREADS), 0, s, a, n); break;
        default: hipLaunchKernelGGL(sc_small<4>, dim3(1), dim3(SC_THREADS), 0, s, a, n); break;
        }
        return;
    }
    if (tiles == 1) {
        switch (na) {
        case 1: hipLaunchKernelGGL(sc_one_tile<1>, dim3(1), dim3(SC_THREADS), 0, s, a, n); break;
        case 2: hipLaunchKernelGGL(sc_one_tile<2>, dim3(1), dim3(SC_THREADS), 0, s, a, n); break;
        case 3: hipLaunchKernelGGL(sc_one_tile<3>, dim3(1), dim3(SC_THREADS), 0, s, a, n); break;
        default: hipLaunchKernelGGL(sc_one_tile<4>, dim3(1), dim3(SC_THREADS), 0, s, a, n); break;
        }
        return;
    }
    ScanHeader *hdr = (ScanHeader *)temp;
    uint64_t *status = (uint64_t *)((char *)temp + sizeof(ScanHeader));
    bool direct = true;
    for (int k = 0; k < na; ++k)
        direct = direct && ((uintptr_t)in[k] & 15u) == 0 && ((uintptr_t)out[k] & 15u) == 0;
#define SC_LAUNCH(NA_)                                                                                              \
    do {                                                                                                            \
        if (direct) hipLaunchKernelGGL((sc_single_pass<NA_, true>), dim3(tiles), dim3(SC_THREADS), 0, s, a, n, tiles, hdr, status); \
        else hipLaunchKernelGGL((sc_single_pass<NA_, false>), dim3(tiles), dim3(SC_THREADS), 0, s, a, n, tiles, hdr, status); \
    } while (0)
    switch (na) {
    case 1: SC_LAUNCH(1); break;
    case 2: SC_LAUNCH(2); break;
    case 3: SC_LAUNCH(3); break;
    default: SC_LAUNCH(4); break;
    }
#undef SC_LAUNCH
}

void exclusive_scan_u32(const uint32_t *in, uint32_t *out, uint32_t n, unsigned long long *total_dev, void *temp,
                        hipStream_t s)
{
    exclusive_scan_multi(1, &in, &out, &total_dev, n, temp, s);
}

} // namespace accord
