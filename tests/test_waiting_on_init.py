"""WaitingOn of a registered-status store's batch: Commands.initialiseWaitingOn
(local/Commands.java:735-753) and its initial updateWaitingOn (:755-830; WaitingOn.Update,
local/Command.java:1403-1600) against the statuses registered when it runs.

CPU: the oracle restatement (or_initialise_waiting_on) against hand-derived known answers -- an
APPLIED dep executing before the txn is set applied (appliedOrInvalidated only for Range-domain
txns), a committed dep executing after it is removed (unless the txn awaitsOnlyDeps: an
ExclusiveSyncPoint keeps waiting), a not-yet-PreCommitted dep stays, an INVALID_OR_TRUNCATED dep is
set applied-or-invalidated, key bits stay set.  GPU: accord_waiting_on_initialise == the oracle on
the same KAT and over random event schedules with range txns and Accept batches, through the C ABI.
"""
import numpy as np
import pytest

from accord_amd import CommandStore, Stream, WINDOW_NONE, generate_stream
import oracle_lib as O
from status_events import ACCEPTED, APPLIED, COMMITTED, INVALID, PREACCEPTED, STABLE, events_for

KIND = {"R": 0, "W": 1, "ER": 2, "SP": 3, "XSP": 4}


def mk(txns):
    """txns: [(hlc, kind, node, keys or None, ranges or None)], epoch 1; ranges make a Range-domain txn."""
    n = len(txns)
    msb = np.full(n, 1 << 15, np.uint64)
    lsb = np.array([(h << 16) | (KIND[k] << 1) | (1 if rs is not None else 0) for h, k, _, _, rs in txns], np.uint64)
    node = np.array([t[2] for t in txns], np.int32)
    key_off = np.zeros(n + 1, np.uint32)
    key_off[1:] = np.cumsum([len(t[3] or []) for t in txns])
    key_ord = np.array([k for t in txns for k in (t[3] or [])], np.uint32)
    rng_off = np.zeros(n + 1, np.uint32)
    rng_off[1:] = np.cumsum([len(t[4] or []) for t in txns])
    rs = np.array([a for t in txns for a, _ in (t[4] or [])], np.uint32)
    re = np.array([b for t in txns for _, b in (t[4] or [])], np.uint32)
    return Stream(msb, lsb, node, key_off, key_ord, rng_off, rs, re)


def ts(s, g, hlc=None):
    """(msb, lsb, node) of txn g's TxnId, or an executeAt at another hlc (flags 0, node 9)."""
    if hlc is None:
        return (int(s.msb[g]), int(s.lsb[g]), int(s.node[g]))
    return (int(s.msb[g]), hlc << 16, 9)


def bit(words, wo_off, t, j):
    return int((int(words[wo_off[t] + j // 64]) >> (j % 64)) & 1)


# t0..t3 range commands; t4 a key txn on key 4; t5 a Range-domain Write over (2, 7]; t6 an
# ExclusiveSyncPoint over (2, 7] (awaitsOnlyDeps)
KAT = [(10, "W", 1, None, [(0, 5)]), (11, "W", 1, None, [(3, 9)]), (12, "W", 1, None, [(3, 6)]),
       (13, "W", 1, None, [(1, 8)]), (20, "W", 1, [4], None), (21, "W", 1, None, [(2, 7)]),
       (22, "XSP", 1, None, [(2, 7)])]


def kat_events(s):
    """t0 APPLIED at hlc 10; t1 COMMITTED at hlc 30 (after t4 / t5 / t6); t2 ACCEPTED at 15;
    t3 INVALID_OR_TRUNCATED; t4..t6 STABLE at their TxnIds."""
    ev = [(0, APPLIED, ts(s, 0)), (1, COMMITTED, ts(s, 1, 30)), (2, ACCEPTED, ts(s, 2, 15)), (3, INVALID, None),
          (4, STABLE, ts(s, 4)), (5, STABLE, ts(s, 5)), (6, STABLE, ts(s, 6))]
    status = np.full(s.n, PREACCEPTED, np.uint8)
    execs = [None] * s.n
    for g, st, x in ev:
        status[g] = st
        execs[g] = x
    return ev, status, execs


def register(st, s, ev):
    idx = np.array([g for g, _, _ in ev])
    xs = [x if x is not None else ts(s, g) for g, _, x in ev]
    st.register(s.msb[idx], s.lsb[idx], s.node[idx], np.array([e[1] for e in ev], np.uint8),
                np.array([x[0] for x in xs], np.uint64), np.array([x[1] for x in xs], np.uint64),
                np.array([x[2] for x in xs], np.int32))


def check_kat(d, wo_off, words, aoi):
    rv4 = [int(v) for v in np.unique(d.range_deps(4)[2])]
    rv5 = [int(v) for v in np.unique(d.range_deps(5)[2])]
    rv6 = [int(v) for v in np.unique(d.range_deps(6)[2])]
    assert rv4 == [0, 1, 2, 3] and rv5 == [0, 1, 2, 3] and rv6 == [0, 1, 2, 3, 5]
    # t4 (Key domain, executeAt hlc 20): t0 applied, t1 executes after, t2 not PreCommitted, t3 invalid
    assert [bit(words, wo_off, 4, j) for j in range(4)] == [0, 0, 1, 0]
    assert all(int(aoi[w]) == 0 for w in range(wo_off[4], wo_off[5]))          # null for Key-domain txns
    # t5 (Range domain, executeAt hlc 21): the same bits, appliedOrInvalidated for t0 and t3; its
    # KeyDeps key 4 (t4) is waited on
    assert [bit(words, wo_off, 5, j) for j in range(4)] == [0, 0, 1, 0]
    assert [bit(aoi, wo_off, 5, j) for j in range(4)] == [1, 0, 0, 1]
    keys5 = d.key_deps(5)[0]
    assert list(keys5) == [4] and bit(words, wo_off, 5, 4) == 1
    # t6 (ExclusiveSyncPoint: awaitsOnlyDeps): t1 and t5 execute later but are still waited on
    assert [bit(words, wo_off, 6, j) for j in range(5)] == [0, 1, 1, 0, 1]
    assert [bit(aoi, wo_off, 6, j) for j in range(5)] == [1, 0, 0, 1, 0]


def test_kat_oracle():
    s = mk(KAT)
    ora = O.LStore(16)
    try:
        d = ora.batch(s)
        ev, status, execs = kat_events(s)
        wo_off, words, aoi = O.initialise_waiting_on(d, s, 0, status, execs)
    finally:
        ora.close()
    check_kat(d, wo_off, words, aoi)


def test_oracle_nothing_committed_is_all_ones():
    # every dep PREACCEPTED: the WaitingOn is initialiseWaiting's full set (or_waiting_on's bits)
    s = generate_stream(600, 3, 60, 0.5, 0.5, range_frac=0.2, range_len_max=20, seed=3)
    ora = O.LStore(60)
    try:
        d = ora.batch(s)
    finally:
        ora.close()
    wo_off, words, aoi = O.initialise_waiting_on(d, s, 0, np.full(s.n, PREACCEPTED, np.uint8), [None] * s.n)
    _, wo_off2, words2 = O.waiting_on(d)
    assert np.array_equal(wo_off, wo_off2) and np.array_equal(words, words2) and not aoi.any()


@pytest.mark.gpu
def test_kat_gpu(gpu_device):
    s = mk(KAT)
    with CommandStore(device=0, key_lo=0, key_hi=16, window=WINDOW_NONE, resident=True) as st:
        d = st.calculate_deps_batch(s)
        ev, status, execs = kat_events(s)
        register(st, s, ev)
        w = st.waiting_on_initialise()
    check_kat(d, w.wo_off, w.words, w.applied_or_invalidated)


def run_schedule(s, ks, pts, seed, accept=None):
    rng = np.random.default_rng(seed)
    status = np.full(s.n, PREACCEPTED, np.uint8)
    execs = [None] * s.n
    ora = O.LStore(ks)
    checked = cleared = marked = 0
    try:
        with CommandStore(device=0, key_lo=0, key_hi=ks, window=WINDOW_NONE, resident=True) as st:
            for a, c in zip(pts[:-1], pts[1:]):
                part = s.slice(a, c) if accept is None else accept.slice(a, c)
                got = st.calculate_deps_batch(part)
                want = ora.batch(part)
                assert got.first_difference(want) is None
                # events up to and including this batch's txns, then the batch's WaitingOn
                idx, stt, em, el, en = events_for(s, 0, c, status, execs, rng, frac=0.6, delay=40, erased=True)
                st.register(s.msb[idx], s.lsb[idx], s.node[idx], stt, em, el, en)
                ora.register(s.msb[idx], s.lsb[idx], s.node[idx], stt, em, el, en)
                w = st.waiting_on_initialise()
                wo_off, words, aoi = O.initialise_waiting_on(want, part, a, status, execs)
                assert np.array_equal(w.wo_off, wo_off)
                assert np.array_equal(w.words, words)
                assert np.array_equal(w.applied_or_invalidated, aoi)
                checked += int(wo_off[-1])
                cleared += int((O.waiting_on(want)[2] ^ words).any())     # some dep resolved
                marked += int(aoi.any())
    finally:
        ora.close()
    assert checked > 0 and cleared > 0 and marked > 0


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,ks,rf,rl,parts,seed", [
    (3000, 4, 300, 0.2, 40, 5, 41),
    (2000, 2, 60, 0.4, 10, 6, 42),
])
def test_gpu_equals_oracle_over_events(gpu_device, n, k, ks, rf, rl, parts, seed):
    s = generate_stream(n, k, ks, 0.99, 0.5, range_frac=rf, range_len_max=rl, seed=seed)
    run_schedule(s, ks, [i * n // parts for i in range(parts + 1)], seed)


@pytest.mark.gpu
def test_gpu_equals_oracle_accept_batches(gpu_device):
    s = generate_stream(2000, 4, 200, 0.99, 0.5, range_frac=0.2, range_len_max=30, seed=43)
    acc = s.accept(frac=0.5, max_delay=30, seed=43)
    run_schedule(s, 200, [0, 500, 1100, 1600, 2000], 43, accept=acc)


@pytest.mark.gpu
def test_initialise_needs_registered_store(gpu_device):
    from accord_amd import IllegalStateException
    s = generate_stream(300, 2, 50, 0.0, 0.5, seed=44)
    with CommandStore(device=0, key_lo=0, key_hi=50, window=256) as st:          # status-at-time model
        st.calculate_deps_batch(s)
        with pytest.raises(IllegalStateException):
            st.waiting_on_initialise()
    with CommandStore(device=0, key_lo=0, key_hi=50, window=WINDOW_NONE, resident=True) as st:
        with pytest.raises(IllegalStateException):                              # nothing computed yet
            st.waiting_on_initialise()
        d = st.calculate_deps_batch(s)
        w = st.waiting_on_initialise()                                           # nothing registered: all set
        assert np.array_equal(w.words, O.waiting_on(d)[2])
        assert w.max_level == 0 and not w.level.any() and not w.applied_or_invalidated.any()

