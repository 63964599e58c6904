"""The stateful literal oracle (or_lstore: resident CommandStore + InternalStatus events, no
status-at-time model) against hand-derived known answers (local/CommandsForKey.java:614-650 with
the committed[] index of :422-470), and its batch-split invariance on seeded event schedules."""
import numpy as np
import pytest

from accord_amd import PartialDeps, Stream
import oracle_lib as O
from status_events import COMMITTED, STABLE, APPLIED, INVALID, ERASED, TK, ACCEPTED, events_for

KIND = {"R": 0, "W": 1, "ER": 2, "SP": 3}


def mk(txns):
    """txns: [(hlc, kind, node, [keys])] in TxnId order, epoch 1."""
    n = len(txns)
    msb = np.full(n, 1 << 15, np.uint64)
    lsb = np.array([(h << 16) | (KIND[k] << 1) for h, k, _, _ in txns], np.uint64)
    node = np.array([nd for _, _, nd, _ in txns], np.int32)
    key_off = np.zeros(n + 1, np.uint32)
    key_off[1:] = np.cumsum([len(ks) for *_, ks in txns])
    key_ord = np.array([k for *_, ks in txns for k in ks], np.uint32)
    return Stream(msb, lsb, node, key_off, key_ord, np.zeros(n + 1, np.uint32), np.zeros(0, np.uint32),
                  np.zeros(0, np.uint32))


def deps_of(d: PartialDeps, i):
    keys, vals, k2v = d.key_deps(i)
    out, t = {}, len(keys)
    for k, key in enumerate(keys):
        out[int(key)] = [int(vals[k2v[x]]) for x in range(t, k2v[k])]
        t = k2v[k]
    return out


def reg(st, s, idx, status, execs=None):
    idx = np.asarray(idx)
    if execs is None:
        execs = [(int(s.msb[g]), int(s.lsb[g]), int(s.node[g])) for g in idx]
    st.register(s.msb[idx], s.lsb[idx], s.node[idx], np.asarray(status, np.uint8),
                np.array([e[0] for e in execs], np.uint64), np.array([e[1] for e in execs], np.uint64),
                np.array([e[2] for e in execs], np.int32))


def test_kat_committed_write_prunes_and_invalid_skipped():
    s = mk([(10, "W", 1, [0]), (11, "W", 1, [0]), (12, "R", 1, [0]), (13, "W", 1, [0]), (14, "W", 1, [0])])
    st = O.LStore(4)
    first = st.batch(s.slice(0, 3))
    assert deps_of(first, 2) == {0: [0, 1]}                          # everything PREACCEPTED
    reg(st, s, [0, 1], [APPLIED, APPLIED])
    # t3: maxCommittedBefore = executeAt(t1); t0 is committed below it (pruned, :634-645),
    # t1 is committed at it (kept), t2 is PREACCEPTED (kept)
    d = st.batch(s.slice(3, 4))
    assert deps_of(d, 0) == {0: [1, 2]}
    reg(st, s, [2], [INVALID])                                       # INVALID_OR_TRUNCATED: skipped
    d = st.batch(s.slice(4, 5))
    assert deps_of(d, 0) == {0: [1, 3]}


def test_kat_executeat_after_startedbefore_does_not_prune():
    # t0 commits with executeAt hlc 100: not before t2's TxnId, so it is not maxCommittedBefore
    # and t1 (committed at its TxnId, below it) is still the bound
    s = mk([(10, "W", 1, [0]), (11, "W", 1, [0]), (20, "W", 1, [0])])
    st = O.LStore(2)
    st.batch(s.slice(0, 2))
    reg(st, s, [0, 1], [STABLE, COMMITTED], execs=[(1 << 15, 100 << 16, 9), (1 << 15, int(s.lsb[1]), 1)])
    d = st.batch(s.slice(2, 3))
    assert deps_of(d, 0) == {0: [0, 1]}       # t0: committed, executeAt 100 >= maxCommittedBefore(t1)


def test_kat_read_witnesses_writes_only_and_tk_is_unreachable():
    s = mk([(10, "W", 1, [0]), (11, "R", 1, [0]), (12, "R", 1, [0])])
    st = O.LStore(1)
    st.batch(s.slice(0, 2))
    d = st.batch(s.slice(2, 3))
    assert deps_of(d, 0) == {0: [0]}          # a Read witnesses Writes only (Txn.java:221-235)
    with pytest.raises(O.OracleError):        # entered PREACCEPTED: TRANSITIVELY_KNOWN is a regression
        reg(st, s, [0], [TK])


def test_kat_status_regression_rejected():
    s = mk([(10, "W", 1, [0]), (11, "W", 1, [0])])
    st = O.LStore(1)
    st.batch(s)
    reg(st, s, [0], [APPLIED])
    with pytest.raises(O.OracleError):
        reg(st, s, [0], [ACCEPTED])
    with pytest.raises(O.OracleError):        # a committed executeAt never changes
        reg(st, s, [0], [APPLIED], execs=[(1 << 15, 50 << 16, 9)])


def test_schedules_are_batch_split_invariant_without_events():
    # no events: a store fed batch by batch == one batch (everything PREACCEPTED, W = infinity)
    from accord_amd import generate_stream
    s = generate_stream(3000, 3, 200, 0.99, 0.5, seed=3)
    a = O.LStore(200)
    one = a.batch(s)
    b = O.LStore(200)
    parts = [b.batch(s.slice(x, y)) for x, y in ((0, 700), (700, 701), (701, 2500), (2500, 3000))]
    assert PartialDeps.concat(parts).first_difference(one) is None
    assert one.first_difference(O.deps_literal(s, 0xFFFFFFFF)) is None


def mk_mixed(txns):
    """txns: [(hlc, kind, node, keys or None, ranges or None)]: a key txn (domain 0) carries keys, a
    range txn (domain 1) (start, end] ranges."""
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


def range_deps_of(d: PartialDeps, i):
    rs, re, rv, r2v = d.range_deps(i)
    out, t = {}, len(rs)
    for k in range(len(rs)):
        out[(int(rs[k]), int(re[k]))] = [int(rv[r2v[x]]) for x in range(t, r2v[k])]
        t = r2v[k]
    return out


def test_kat5_erased_or_invalidated_range_command_still_visited():
    # SURVEY.md §8c KAT 5: mapReduceRangesInternal skips saveStatus >= Erased (impl/InMemoryCommandStore.
    # java:891); ErasedOrInvalidated precedes Erased in SaveStatus order (local/SaveStatus.java:83-86),
    # so a range command there is still a dependency.  Here INVALID_OR_TRUNCATED (the InternalStatus of
    # ErasedOrInvalidated / Truncated*) keeps the range command, ERASED removes it.
    s = mk_mixed([(10, "W", 1, None, [(0, 5)]), (11, "W", 1, None, [(3, 9)]), (12, "W", 1, [4], None),
                  (13, "W", 1, [4], None), (14, "W", 1, [4], None)])
    st = O.LStore(16)
    d = st.batch(s.slice(0, 3))
    assert range_deps_of(d, 2) == {(0, 5): [0], (3, 9): [1]}
    assert range_deps_of(d, 1) == {(0, 5): [0]}                       # ranges (0,5] and (3,9] meet
    reg(st, s, [0], [INVALID])                                         # ErasedOrInvalidated: still visited
    d = st.batch(s.slice(3, 4))
    assert range_deps_of(d, 0) == {(0, 5): [0], (3, 9): [1]}
    reg(st, s, [0, 1], [ERASED, INVALID])                              # Erased: off the scan
    d = st.batch(s.slice(4, 5))
    assert range_deps_of(d, 0) == {(3, 9): [1]}


def test_kat_range_txn_keydeps_use_cfk_filter():
    # a range txn's KeyDeps are mapReduceActive on every CFK key of its ranges
    # (impl/InMemoryCommandStore.java:274-289): committed pruning applies to them as to key txns
    s = mk_mixed([(10, "W", 1, [2], None), (11, "W", 1, [2], None), (12, "R", 1, [3], None),
                  (13, "W", 1, None, [(1, 3)])])
    st = O.LStore(8)
    st.batch(s.slice(0, 3))
    reg(st, s, [0, 1], [APPLIED, APPLIED])
    d = st.batch(s.slice(3, 4))
    assert deps_of(d, 0) == {2: [1], 3: [2]}                         # t0 pruned below executeAt(t1)
