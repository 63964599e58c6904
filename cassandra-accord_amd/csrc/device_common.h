// Device helpers shared by the deps kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ACC_WAVE 64

__device__ __forceinline__ uint32_t lane_id()
{
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
// Wave index inside the workgroup, as a wave-uniform (scalar) value: threadIdx.x >> 6 alone is a
// VGPR to the compiler, which then treats every loop and branch derived from it as divergent.
__device__ __forceinline__ uint32_t wave_id()
{
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}
__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// Order LDS traffic between lanes of ONE wave (waves of a workgroup run different txns, so a
// block barrier is not usable inside the per-txn loops).  LDS ops of a wave are processed in
// order; the waitcnt + memory clobber keeps the compiler from reordering across it.
__device__ __forceinline__ void wave_lds_sync()
{
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// DPP row_shr:N inside each row of 16 lanes; lanes whose source is outside the row read 0.
template <int N> __device__ __forceinline__ uint32_t dpp_row_shr(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 + N, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t readlane(uint32_t v, int l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// Inclusive wave scans: Hillis-Steele inside rows of 16 with DPP (no LDS traffic), then the row
// totals are added through three scalar readlanes.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    v += dpp_row_shr<1>(v);
    v += dpp_row_shr<2>(v);
    v += dpp_row_shr<4>(v);
    v += dpp_row_shr<8>(v);
    const uint32_t l = lane_id();
    const uint32_t r0 = readlane(v, 15), r1 = readlane(v, 31), r2 = readlane(v, 47);
    v += (l >= 16 ? r0 : 0u) + (l >= 32 ? r1 : 0u) + (l >= 48 ? r2 : 0u);
    return v;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v)
{
    v = max(v, dpp_row_shr<1>(v));
    v = max(v, dpp_row_shr<2>(v));
    v = max(v, dpp_row_shr<4>(v));
    v = max(v, dpp_row_shr<8>(v));
    const uint32_t l = lane_id();
    const uint32_t r0 = readlane(v, 15), r1 = max(r0, readlane(v, 31)), r2 = max(r1, readlane(v, 47));
    return l >= 48 ? max(v, r2) : l >= 32 ? max(v, r1) : l >= 16 ? max(v, r0) : v;
}
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v)
{
    const uint32_t l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint64_t t = __shfl_up(v, d, 64);
        if (l >= (uint32_t)d) v += t;
    }
    return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
    return readlane(wave_incl_scan(v), 63);
}

// ---- TxnId semantics (primitives/Timestamp.java:208-217, TxnId.java:124-157, Txn.java) ----
// Kind ordinals: Read 0, Write 1, EphemeralRead 2, SyncPoint 3, ExclusiveSyncPoint 4, LocalOnly 5
// witnesses(): Read/EphemeralRead -> Ws, Write -> RsOrWs, SyncPoints -> AnyGloballyVisible.
// Encoded as a bitmask over entry kinds: Ws = {W}, RsOrWs = {R,W}, AnyGV = {R,W,SP,ESP}.
// Read, EphemeralRead -> {W}; Write -> {R, W}; SyncPoint, ExclusiveSyncPoint -> {R, W, SP, XSP};
// LocalOnly / invalid -> {} (rejected by validation).  One byte per kind of a 64-bit table: a shift
// and a mask instead of a branch chain.
__host__ __device__ __forceinline__ uint32_t witness_mask(uint32_t kind)
{
    constexpr uint64_t T = 0x02ull | 0x03ull << 8 | 0x02ull << 16 | 0x1Bull << 24 | 0x1Bull << 32;
    return (uint32_t)(T >> ((kind & 7u) * 8u)) & 0xFFu;
}

// Timestamp.compareTo (primitives/Timestamp.java:209-217): unsigned msb, then the low hlc, then the
// identity flags, then the signed node.  Branch-free: every field is compared and the first
// difference selected, so the result is a value, not a control-flow join (a branchy form fed into a
// running max was miscompiled on gfx950: profiles/r05_eal).
__device__ __forceinline__ int ts_cmp(uint64_t am, uint64_t al, int32_t an, uint64_t bm, uint64_t bl, int32_t bn)
{
    const uint64_t ah = al >> 16, bh = bl >> 16;
    const uint32_t af = (uint32_t)al & 0x1Eu, bf = (uint32_t)bl & 0x1Eu;
    const int c0 = (int)(am > bm) - (int)(am < bm);
    const int c1 = (int)(ah > bh) - (int)(ah < bh);
    const int c2 = (int)(af > bf) - (int)(af < bf);
    const int c3 = (int)(an > bn) - (int)(an < bn);
    return c0 ? c0 : c1 ? c1 : c2 ? c2 : c3;
}

// History entry: txn index in the low 29 bits, entry kind in the top 3 bits.
#define ENT_TXN_MASK 0x1FFFFFFFu
#define ENT_KIND_SHIFT 29

// Packed per-position class counters of the key-major history (16-bit fields, tile-local):
// Writes | Reads << 16 | EphemeralReads << 32, completed by one ClassCarry per HISTORY_TILE
// positions.  They give, for any history range, the number of entries a txn kind witnesses
// (Ws = #W, RsOrWs = #W + #R, AnyGloballyVisible = len - #ER).
__host__ __device__ __forceinline__ uint64_t class_bits(uint32_t kind)
{
    return kind == 1u ? 1ull : kind == 0u ? (1ull << 16) : kind == 2u ? (1ull << 32) : 0ull;
}

struct ClassCarry {
    uint32_t w, r, er, pad;
};

// entries of [0, x] (global history positions) witnessed by wmask; tile = HISTORY_TILE
__device__ __forceinline__ uint32_t witnessed_upto(const uint64_t *__restrict__ c_local,
                                                   const ClassCarry *__restrict__ ccarry, uint32_t x, uint32_t wmask,
                                                   uint32_t tile = 4096u)
{
    const uint64_t c = c_local[x];
    const ClassCarry cc = ccarry[x / tile];
    const uint32_t w = (uint32_t)(c & 0xFFFFu) + cc.w;
    if (wmask == 0x2u) return w;
    if (wmask == 0x3u) return w + (uint32_t)((c >> 16) & 0xFFFFu) + cc.r;
    return x + 1 - ((uint32_t)((c >> 32) & 0xFFFFu) + cc.er);
}
