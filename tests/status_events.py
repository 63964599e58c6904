"""Random InternalStatus event schedules for resident stores without the status-at-time model
(shared by the CPU oracle tests and the GPU tests)."""
import numpy as np

TK, HISTORICAL, PREACCEPTED, ACCEPTED, COMMITTED, STABLE, APPLIED, INVALID, ERASED = range(9)


def events_for(s, lo, hi, status_now, exec_now, rng, frac=0.5, delay=40, erased=False):
    """Status events for a random subset of txns [lo, hi) of stream s (global positions == stream
    positions): each advances its status (never back) and, on first commit, fixes an executeAt
    >= txnId (hlc + U[0, delay], flags 0, a node id).  status_now/exec_now track the schedule.
    erased: ERASED (SaveStatus Erased / Invalidated) may follow as well.
    Returns (idx, status, exec_msb, exec_lsb, exec_node) sorted by position."""
    idx = np.sort(rng.choice(np.arange(lo, hi), size=int((hi - lo) * frac), replace=False))
    st = np.zeros(idx.size, np.uint8)
    em = np.zeros(idx.size, np.uint64); el = np.zeros(idx.size, np.uint64); en = np.zeros(idx.size, np.int32)
    for r, g in enumerate(idx):
        cur = status_now[g]
        # a txn enters the store PREACCEPTED (its batch), so only later statuses can follow
        allowed = (PREACCEPTED, ACCEPTED, COMMITTED, STABLE, APPLIED, INVALID) + ((ERASED,) if erased else ())
        choices = [x for x in allowed if x >= cur]
        w = np.array([0.12 if x >= INVALID else 1.0 for x in choices])
        nw = int(rng.choice(choices, p=w / w.sum()))
        if exec_now[g] is None:
            # executeAt >= txnId; node ids 8..15 never equal a stream TxnId (nodes 1..7), so no
            # executeAt ties a TxnId (Timestamp.compareTo == 0)
            d = int(rng.integers(0, delay + 1))
            if d == 0:
                exec_now[g] = (int(s.msb[g]), int(s.lsb[g]), int(s.node[g]))
            else:
                exec_now[g] = (int(s.msb[g]), ((int(s.lsb[g]) >> 16) + d) << 16, int(rng.integers(8, 16)))
        st[r] = nw
        em[r], el[r], en[r] = exec_now[g]
        status_now[g] = nw
    return idx, st, em, el, en


def committed_schedule(s, sizes, lag_applied=4, lag_rb=None):
    """The bench.py --registered event schedule over consecutive batches of the given sizes: right
    after batch b is computed its txns are COMMITTED at executeAt = TxnId, the txns of batch
    b - lag_applied become APPLIED, and (lag_rb set) the store's RedundantBefore moves to the first
    txn of batch b - lag_rb (shardAppliedOrInvalidatedBefore: everything before it applied).
    Yields, per batch, (lo, hi, events, rb): events = (idx, status) to register after computing
    [lo, hi), rb = the new RedundantBefore bound (a position) to set after that, or None."""
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    for b in range(len(sizes)):
        lo, hi = int(starts[b]), int(starts[b + 1])
        ev = [(np.arange(lo, hi), COMMITTED)]
        if b >= lag_applied:
            ev.append((np.arange(int(starts[b - lag_applied]), int(starts[b - lag_applied + 1])), APPLIED))
        # one register call per batch: TxnIds ascending
        idx = np.concatenate([e[0] for e in ev[::-1]])
        st = np.concatenate([np.full(len(e[0]), e[1], np.uint8) for e in ev[::-1]])
        rb = int(starts[b - lag_rb]) if lag_rb is not None and b >= lag_rb and starts[b - lag_rb] > 0 else None
        yield lo, hi, (idx, st), rb


def schedule_floors(sizes, lag_rb=None):
    """floor[i] of the schedule: the RedundantBefore bound in force when i's batch is computed."""
    starts = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    f = np.zeros(len(sizes), np.int64)
    if lag_rb is not None:
        for b in range(1, len(sizes)):
            f[b] = starts[b - 1 - lag_rb] if b - 1 >= lag_rb else 0
    return np.repeat(f, sizes).astype(np.uint32)


def rb_map(ks, bound):
    """A one-entry RedundantBefore map over the keyspace (keys 1..ks-1: (0, ks-1]), every epoch."""
    return dict(start=[0], end=[ks - 1], start_epoch=[0], end_epoch=[1 << 62], bound=[bound])


def register_events(target, s, idx, st):
    """target.register for events at stream positions idx (executeAt = TxnId)."""
    target.register(s.msb[idx], s.lsb[idx], s.node[idx], st, s.msb[idx], s.lsb[idx], s.node[idx])
