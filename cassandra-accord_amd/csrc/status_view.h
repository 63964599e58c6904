// Registered statuses as the device kernels read them (status.hip, ready.hip): InternalStatus and
// executeAt by global position (local/CommandsForKey.java:194-203).
#pragma once
#include "../../include/accord_deps.h"
#include "device_common.h"
#include "kernels.h"

#include <cstdint>

namespace accord_status {

constexpr uint8_t ST_TK = 0, ST_PREACCEPTED = 2, ST_ACCEPTED = 3, ST_COMMITTED = 4, ST_STABLE = 5, ST_APPLIED = 6,
                  ST_INVALID = 7,
                  ST_ERASED = 8,   // SaveStatus Erased / Invalidated: as INVALID for CFK, and off the range scan
                  // SaveStatus TruncatedApply* (local/SaveStatus.java:79-81): INVALID_OR_TRUNCATED for CFK
                  // (CommandsForKey.java:222-224), still visited by the range scan, and its executeAt known
                  ST_TRUNC_APPLY = 9;

__device__ __forceinline__ bool committed(uint32_t st) { return st >= ST_COMMITTED && st <= ST_APPLIED; }
// known().executeAt == ExecuteAtKnown once committed, including TruncatedApply (local/Commands.java:782)
__device__ __forceinline__ bool exec_known(uint32_t st) { return committed(st) || st == ST_TRUNC_APPLY; }
// the order statuses advance in (SaveStatus order: ... Applied < TruncatedApply < ErasedOrInvalidated
// / Invalidated (INVALID) < Erased)
__host__ __device__ __forceinline__ uint32_t status_rank(uint32_t st) { return st == ST_TRUNC_APPLY ? 13u : 2u * st; }

struct Ts {
    uint64_t msb, lsb;
    int32_t node;
};

// Invariants.checkState(dep.executeAt < waitingExecuteAt || awaitsOnlyDeps) for a TruncatedApply dep
// (local/Commands.java:789-791): an IllegalStateException in the reference, ACCORD_ERR_STATE here
__device__ __forceinline__ void trunc_check_fail(accord::DevStatus *err, uint32_t t)
{
    if (err) atomicMin(&err->first, ((unsigned long long)t << 32) | (uint32_t)(-ACCORD_ERR_STATE));
}

__device__ __forceinline__ int tcmp(const Ts &a, const Ts &b) { return ts_cmp(a.msb, a.lsb, a.node, b.msb, b.lsb, b.node); }

struct StatusView {
    const uint8_t *status;            // [next_global] InternalStatus by global position
    const uint64_t *emsb, *elsb;      // executeAt by global position
    const int32_t *enode;
    uint32_t known;                   // positions >= known are this batch's txns: PREACCEPTED
};

__device__ __forceinline__ uint32_t status_of(const StatusView &v, uint32_t g)
{
    return g < v.known ? v.status[g] : ST_PREACCEPTED;
}
__device__ __forceinline__ Ts exec_of(const StatusView &v, uint32_t g)
{
    return Ts{v.emsb[g], v.elsb[g], v.enode[g]};
}

} // namespace accord_status
