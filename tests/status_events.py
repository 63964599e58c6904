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
