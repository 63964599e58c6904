"""MaxConflicts fold (local/MaxConflicts.java:46-80,
local/CommandStore.java:280-289,320-349, local/SafeCommandStore.java:192-210).

CPU half: the oracle restatements -- or_max_conflicts (one entry per key) and or_max_conflicts_rm
(the map as disjoint intervals, ReducingRangeMap-style, key and range txns) -- against hand-derived
known answers and against each other (a range txn == the txn over the store keys it covers).  GPU
half (`-m gpu`): accord_max_conflicts_fold through the C ABI, bit-exact against the oracle on seeded
PreAccept and Accept streams with key and range txns, the per-key map carried across batches, tie
handling and errors.
The reference has no MaxConflicts test of its own; parity rests on the restatement + these KATs."""
import dataclasses

import numpy as np
import pytest

from accord_amd import Stream, generate_stream
import oracle_lib as O

KIND = {"R": 0, "W": 1, "ER": 2, "SP": 3, "XSP": 4}


def unique_now(minimum, node=9):
    """Stand-in for NodeTimeService.uniqueNow(atLeast) (local/CommandStore.java:348): a Timestamp
    strictly after `minimum` -- the next hlc, flags 0, this node's id."""
    m, l, _ = minimum
    return int(m), ((int(l) >> 16) + 1) << 16, node


def fold_all(fold, n):
    """Drive a fold to the end of the batch the way a caller does: every stop is a globally visible
    slow-path txn; give it uniqueNow(minNonConflicting) and continue.  `fold(first, exec_at, out)`
    returns (out5, folded).  Returns the outputs and the executeAts chosen."""
    out, folded = fold(0, None, None)
    chosen = {}
    while folded < n:
        ex = unique_now((out[0][folded], out[1][folded], out[2][folded]))
        chosen[folded] = ex
        out, f2 = fold(folded, ex, out)
        assert f2 > folded
        folded = f2
    return out, chosen


def mk(txns, execs=None):
    """txns: [(hlc, kind, node, [keys])] in TxnId order (epoch 1); execs: [(hlc, node, low16)] or None."""
    n = len(txns)
    msb = np.full(n, 1 << 16, np.uint64)          # epoch 1 in the msb's high bits (Timestamp.java:77-79)
    lsb = np.array([(h << 16) | (KIND[k] << 1) for h, k, _, _ in txns], np.uint64)
    node = np.array([nd for _, _, nd, _ in txns], np.int32)
    key_off = np.zeros(n + 1, np.uint32)
    key_off[1:] = np.cumsum([len(ks) for *_, ks in txns])
    key_ord = np.array([k for *_, ks in txns for k in ks], np.uint32)
    z = np.zeros(n + 1, np.uint32)
    s = Stream(msb, lsb, node, key_off, key_ord, z, np.zeros(0, np.uint32), np.zeros(0, np.uint32))
    if execs is not None:
        s = dataclasses.replace(s, exec_msb=msb.copy(),
                                exec_lsb=np.array([(h << 16) | lo for h, _, lo in execs], np.uint64),
                                exec_node=np.array([nd for _, nd, _ in execs], np.int32))
    return s


def test_kat_empty_map_is_none_and_fast():
    (m, l, nd, present, fast), st, _ = O.max_conflicts(mk([(10, "W", 1, [0, 3])]), 0, 8)
    assert present.tolist() == [0] and fast.tolist() == [1] and (m[0], l[0], nd[0]) == (0, 0, 0)
    assert st[3].tolist() == [1, 0, 0, 1, 0, 0, 0, 0]


def test_kat_max_over_keys_and_ephemeral_read_invisible():
    # t0 W{1} t1 ER{2} t2 R{1,2}: t2 sees t0 on key 1 only (ER is not globally visible, Txn.java:187-200)
    s = mk([(10, "W", 1, [1]), (11, "ER", 1, [2]), (12, "R", 2, [1, 2])])
    (m, l, nd, present, fast), st, _ = O.max_conflicts(s, 0, 4)
    assert present.tolist() == [0, 0, 1] and fast.tolist() == [1, 1, 1]
    assert (l[2] >> 16, nd[2]) == (10, 1)
    assert st[3].tolist() == [0, 1, 1, 0]   # t2 itself lands on keys 1 and 2


def test_kat_accept_executeat_forces_slow_path():
    # t0's executeAt (hlc 50) lies after t1's TxnId (hlc 20): t1 is not fast, t2 (hlc 60) is
    s = mk([(10, "W", 1, [0]), (20, "W", 1, [0]), (60, "R", 1, [0])], execs=[(50, 3, 0), (20, 1, 2), (60, 1, 0)])
    (m, l, nd, present, fast), _, folded = O.max_conflicts(s, 0, 1)
    assert fast.tolist() == [1, 0, 1] and folded == 3    # Accept batch: every executeAt is known
    assert (l[1] >> 16, nd[1]) == (50, 3) and (l[2] >> 16, nd[2]) == (50, 3)


def test_kat_ties_merge_keeps_old_fold_takes_later_key():
    # two executeAts that compare equal (bit 5 of lsb is outside the compared flags) but differ in bits
    s = mk([(10, "W", 1, [0]), (11, "W", 1, [0, 1]), (12, "R", 1, [0, 1])],
           execs=[(40, 2, 0x20), (40, 2, 0x00), (12, 1, 0)])
    (m, l, nd, present, fast), st, _ = O.max_conflicts(s, 0, 2)
    # key 0 keeps t0's bits (merge: Timestamp.max(old, new) keeps old on a tie); key 1 holds t1's
    assert st[1][0] & 0xFFFF == 0x20 and st[1][1] & 0xFFFF == 0x00
    # t2 folds key 0 then key 1 with Timestamp.max(value, acc): the tie takes key 1's value
    assert l[2] & 0xFFFF == 0x00


def test_kat_state_carries_over():
    a = mk([(10, "W", 1, [0])])
    _, st, _ = O.max_conflicts(a, 0, 2)
    (m, l, nd, present, fast), _, folded = O.max_conflicts(mk([(5, "R", 1, [0])]), 0, 2, st)
    assert present.tolist() == [1] and fast.tolist() == [0]
    assert folded == 0                    # slow-path read: its executeAt is the caller's uniqueNow


def advice_stream():
    # key 0 = A holds hlc 100 from an earlier batch, key 1 = B is empty.  t1 (hlc 50, {A, B}) is slow:
    # the reference merges its executeAt uniqueNow(100) >= 101 on B too, so t2 (hlc 60, {B}) is slow
    # as well -- folding with executeAt = txnId for t1 would make t2 fast (a wrong fast-path decision).
    return mk([(100, "W", 1, [0])]), mk([(50, "W", 1, [0, 1]), (60, "W", 1, [1])])


def test_kat_slow_path_executeat_is_merged_before_later_txns():
    first, second = advice_stream()
    _, st0, _ = O.max_conflicts(first, 0, 2)
    state = st0

    def fold(f, ex, out):
        nonlocal state
        o, state, folded = O.max_conflicts(second, 0, 2, state, first=f, exec_at=ex, out=out)
        return o, folded
    out, folded = fold(0, None, None)
    assert folded == 0 and out[4][0] == 0                    # t1 stops the fold: slow, executeAt unknown
    (m, l, nd, present, fast), chosen = fold_all(fold, 2)
    assert fast.tolist() == [0, 0]                           # t2 sees t1's uniqueNow(100) on B
    assert (l[1] >> 16) == 101 and chosen[0][1] >> 16 == 101


def test_kat_exclusive_sync_point_key_domain_rejected():
    with pytest.raises(O.OracleError) as e:
        O.max_conflicts(mk([(10, "XSP", 1, [0])]), 0, 1)
    assert e.value.rc == -3
    with pytest.raises(O.OracleError) as e:
        O.max_conflicts(mk([(10, "XSP", 1, [0])]), 0, 1, intervals=True)
    assert e.value.rc == -3


def mk_r(txns, execs=None):
    """txns: [(hlc, kind, node, keys or None, [(start, end)] or None)]; a txn with ranges is in the
    range domain (TxnId bit 0), its ranges (start, end] (Range.EndInclusive)."""
    base = mk([(h, k, nd, ks or []) for h, k, nd, ks, _ in txns], execs)
    lsb = base.lsb.copy()
    rng_off = np.zeros(len(txns) + 1, np.uint32)
    rs, re = [], []
    for i, (*_, rgs) in enumerate(txns):
        if rgs is not None:
            lsb[i] |= np.uint64(1)
            for a, b in rgs:
                rs.append(a); re.append(b)
        rng_off[i + 1] = len(rs)
    return dataclasses.replace(base, lsb=lsb, rng_off=rng_off, rng_start=np.array(rs, np.uint32),
                               rng_end=np.array(re, np.uint32))


def test_kat_range_reads_and_writes_covered_keys():
    # t0 W{3}, t1 W{6}; t2 range (3, 6] = keys 4..6: sees t1 (key 6), not t0 (key 3, start exclusive)
    s = mk_r([(10, "W", 1, [3], None), (20, "W", 1, [6], None), (30, "R", 2, None, [(3, 6)]),
              (25, "W", 1, [5], None)])
    (m, l, nd, present, fast), st, folded = O.max_conflicts(s, 0, 8)
    assert (l[2] >> 16, nd[2], present[2], fast[2]) == (20, 1, 1, 1)
    # t2's executeAt (txnId, hlc 30) covers keys 4..6: t3 (hlc 25) on key 5 is slow
    assert (l[3] >> 16, fast[3]) == (30, 0) and folded == 3
    assert [int(x) >> 16 if h else None for x, h in zip(st[1], st[3])] == [None, None, None, 10, 30, 30, 30, None]


def test_kat_range_clipped_to_store_and_xsp():
    # store keys [4, 8): range (0, 5] covers 4..5 only; XSP (range) reads nothing, is fast and merges
    s = mk_r([(10, "XSP", 1, None, [(0, 5)]), (5, "W", 1, [4], None), (11, "R", 1, None, [(5, 9)])])
    (m, l, nd, present, fast), st, folded = O.max_conflicts(s, 4, 4)
    assert present.tolist()[0] == 0 and fast.tolist()[0] == 1
    assert (l[1] >> 16, fast[1]) == (10, 0) and folded == 1      # XSP's txnId landed on key 4
    assert st[3].tolist() == [1, 1, 0, 0]


def test_kat_range_ties_fold_in_interval_order():
    # equal executeAts on keys 1 and 2 differing in an uncompared bit: a range over both folds
    # key 1 then key 2 (Timestamp.max(value, acc) takes the later interval's value on a tie)
    s = mk_r([(10, "W", 1, [1], None), (11, "W", 1, [2], None), (12, "R", 1, None, [(0, 2)])],
             execs=[(40, 2, 0x20), (40, 2, 0x00), (12, 1, 0)])
    (m, l, nd, present, fast), _, _ = O.max_conflicts(s, 0, 4)
    assert l[2] & 0xFFFF == 0x00 and fast[2] == 0


def expand_ranges(s, key_lo, nkeys):
    """The same stream with every range txn's ranges replaced by the store keys they cover (still
    range-domain txns): the per-key form the device fold uses."""
    ko, kk = [0], []
    for i in range(s.n):
        if int(s.lsb[i]) & 1:
            ks = [k for a, b in zip(s.rng_start[s.rng_off[i]:s.rng_off[i + 1]], s.rng_end[s.rng_off[i]:s.rng_off[i + 1]])
                  for k in range(max(int(a) + 1, key_lo), min(int(b), key_lo + nkeys - 1) + 1)]
        else:
            ks = list(s.key_ord[s.key_off[i]:s.key_off[i + 1]])
        kk += ks
        ko.append(len(kk))
    lsb = s.lsb & ~np.uint64(1)
    return dataclasses.replace(s, lsb=lsb, key_off=np.array(ko, np.uint32), key_ord=np.array(kk, np.uint32),
                               rng_off=np.zeros(s.n + 1, np.uint32))


def no_key_xsp(s):
    """XSP is range-domain only: turn key-domain XSPs into SyncPoints."""
    lsb = s.lsb.astype(np.uint64).copy()
    kind = (lsb >> np.uint64(1)) & np.uint64(7)
    bad = ((lsb & np.uint64(1)) == 0) & (kind == 4)
    lsb[bad] = (lsb[bad] & ~np.uint64(0xE)) | np.uint64(3 << 1)
    return dataclasses.replace(s, lsb=lsb)


@pytest.mark.parametrize("seed,rf,accept", [(1, 0.0, False), (2, 0.0, True), (3, 0.3, False), (4, 0.3, True)])
def test_interval_map_matches_per_key(seed, rf, accept):
    # the interval restatement equals the per-key one on key streams, and a range txn equals the
    # txn reading/writing every store key its ranges cover (IntKey ranges have no gaps to miss)
    from test_oracle_stream import with_random_kinds
    s = generate_stream(1500, 3, 60, 0.5, 0.5, seed=seed, range_frac=rf, range_len_max=12)
    s = no_key_xsp(with_random_kinds(s, seed))
    if accept:
        s = s.accept(frac=0.6, max_delay=300, seed=seed)
    for lo, nk in ((0, 60), (10, 30)):
        if rf == 0.0 and lo == 0:
            a = fold_all(lambda f, ex, out: (lambda r: (r[0], r[2]))(
                O.max_conflicts(s, lo, nk, first=f, exec_at=ex, out=out, intervals=True)), s.n)
            b = fold_all(lambda f, ex, out: (lambda r: (r[0], r[2]))(
                O.max_conflicts(s, lo, nk, first=f, exec_at=ex, out=out, intervals=False)), s.n)
            assert a[1] == b[1] and all(np.array_equal(x, y) for x, y in zip(a[0], b[0]))
        if rf == 0.0:
            continue
        sub = s.restrict_keys(lo, lo + nk, drop_empty=False) if lo else s
        e = expand_ranges(sub, lo, nk)
        xs = [fold_all(lambda f, ex, out, t=t, iv=iv: (lambda r: (r[0], r[2]))(
            O.max_conflicts(t, lo, nk, first=f, exec_at=ex, out=out, intervals=iv)), t.n)
            for t, iv in ((sub, True), (e, False))]
        # the expanded form has no range-domain XSP: compare txns other than those
        xsp = (((sub.lsb >> np.uint64(1)) & np.uint64(7)) == 4) & ((sub.lsb & np.uint64(1)) == 1)
        if not xsp.any():
            # (the expanded copy drops the range-domain bit, lsb bit 0, which Timestamp.compareTo
            # ignores: compare values without it)
            strip = lambda t: (t[0], t[1] & ~1, t[2]) if t is not None else t
            assert {k: strip(v) for k, v in xs[0][1].items()} == {k: strip(v) for k, v in xs[1][1].items()}
            for j, (x, y) in enumerate(zip(xs[0][0], xs[1][0])):
                if j == 1:
                    x, y = x & ~np.uint64(1), y & ~np.uint64(1)
                assert np.array_equal(x, y)


# ------------------------------------------------------------------------------------------ GPU
def gpu_fold(streams, keyspace):
    from accord_amd import CommandStore
    outs = []
    with CommandStore(device=0, key_lo=0, key_hi=keyspace, window=0) as st:
        for s in streams:
            st.upload(s)

            def fold(f, ex, out):
                r = st.max_conflicts_fold(first=f, exec_at=ex, out=out)
                return r[:5], r[5]
            outs.append(fold_all(fold, s.n))
        return outs, st.max_conflicts_state()


def check(streams, keyspace):
    got, gst = gpu_fold(streams, keyspace)
    state = None
    for s, (g, gchosen) in zip(streams, got):
        st0 = state

        def fold(f, ex, out):
            nonlocal state
            o, state, folded = O.max_conflicts(s, 0, keyspace, state if f else st0, first=f, exec_at=ex, out=out)
            return o, folded
        want, chosen = fold_all(fold, s.n)
        assert chosen == gchosen
        for a, b, name in zip(g, want, ("msb", "lsb", "node", "present", "fast")):
            assert np.array_equal(a, b), (name, int(np.flatnonzero(a != b)[0]))
    for a, b in zip(gst, state):
        assert np.array_equal(a, b)


@pytest.mark.gpu
def test_gpu_slow_path_stops_and_continues(gpu_device):
    first, second = advice_stream()
    check([first, second], 2)
    # a PreAccept stream whose later batches are slow on many keys: many stops and continuations
    s = generate_stream(3000, 3, 40, 0.0, 0.5, seed=11)
    check([s.prefix(1500).accept(frac=1.0, max_delay=400, seed=3), s], 40)


@pytest.mark.gpu
def test_gpu_refold_and_xsp_rejected(gpu_device):
    from accord_amd import CommandStore, AccordError
    with CommandStore(device=0, key_lo=0, key_hi=4, window=0) as st:
        st.upload(mk([(10, "W", 1, [0])]))
        assert st.max_conflicts_fold()[5] == 1
        with pytest.raises(AccordError):
            st.max_conflicts_fold()                         # the batch is already merged
        with pytest.raises(AccordError):
            st.max_conflicts_fold(mk([(20, "XSP", 1, [1])]))


@pytest.mark.gpu
@pytest.mark.parametrize("fn", [test_kat_empty_map_is_none_and_fast, test_kat_max_over_keys_and_ephemeral_read_invisible])
def test_gpu_kat_streams(gpu_device, fn):
    s = {test_kat_empty_map_is_none_and_fast: mk([(10, "W", 1, [0, 3])]),
         test_kat_max_over_keys_and_ephemeral_read_invisible: mk([(10, "W", 1, [1]), (11, "ER", 1, [2]), (12, "R", 2, [1, 2])])}[fn]
    check([s], 8)


@pytest.mark.gpu
def test_gpu_ties_and_accept(gpu_device):
    check([mk([(10, "W", 1, [0]), (11, "W", 1, [0, 1]), (12, "R", 1, [0, 1])],
              execs=[(40, 2, 0x20), (40, 2, 0x00), (12, 1, 0)])], 2)
    check([mk([(10, "W", 1, [0]), (20, "W", 1, [0]), (60, "R", 1, [0])], execs=[(50, 3, 0), (20, 1, 2), (60, 1, 0)])], 1)


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,ks,z,seed,frac,delay", [
    (1, 1, 10, 0.0, 1, 0.0, 0),
    (5000, 4, 300, 0.0, 2, 0.0, 0),
    (20000, 8, 2000, 0.99, 3, 1.0, 500),
    (30000, 8, 50, 0.99, 4, 0.7, 5000),       # hot keys: segments span many 1024-pair tiles
    (4000, 12, 100000, 0.99, 5, 0.5, 64),
    (50000, 1, 3, 0.0, 6, 1.0, 100000),
])
def test_gpu_vs_oracle(gpu_device, n, k, ks, z, seed, frac, delay):
    s = generate_stream(n, k, ks, z, 0.5, seed=seed)
    if frac:
        s = s.accept(frac=frac, max_delay=delay, seed=seed)
    check([s], ks)


@pytest.mark.gpu
def test_gpu_state_across_batches(gpu_device):
    s = generate_stream(30000, 8, 3000, 0.99, 0.5, seed=8).accept(frac=0.5, max_delay=2000, seed=8)
    check([s.prefix(10000), s.prefix(30000), s.prefix(7)], 3000)


@pytest.mark.gpu
def test_gpu_config2_full(gpu_device):
    s = generate_stream(1 << 20, 8, 100_000, 0.99, 0.5, seed=2)
    check([s], 100_000)


@pytest.mark.gpu
def test_gpu_errors(gpu_device):
    from accord_amd import CommandStore, AccordError
    with CommandStore(device=0, key_lo=0, key_hi=4, window=0) as st:
        with pytest.raises(AccordError):
            st.max_conflicts_fold(mk([(10, "W", 1, [5])]))      # key outside the store
        # a rejected batch leaves the map untouched
        assert st.max_conflicts_state()[3].sum() == 0
        with pytest.raises(AccordError):
            st.max_conflicts_fold(mk_r([(10, "R", 1, None, [(3, 2)])]))   # empty range
        with pytest.raises(AccordError):
            st.max_conflicts_fold(mk_r([(10, "R", 1, None, [(0, 3), (2, 4)])]))   # overlapping ranges
        assert st.max_conflicts_state()[3].sum() == 0


@pytest.mark.gpu
def test_gpu_range_kats(gpu_device):
    check([mk_r([(10, "W", 1, [3], None), (20, "W", 1, [6], None), (30, "R", 2, None, [(3, 6)]),
                 (25, "W", 1, [5], None)])], 8)
    check([mk_r([(10, "W", 1, [1], None), (11, "W", 1, [2], None), (12, "R", 1, None, [(0, 2)])],
                execs=[(40, 2, 0x20), (40, 2, 0x00), (12, 1, 0)])], 4)


def check_window(streams, key_lo, nkeys):
    """check() for a store owning keys [key_lo, key_lo + nkeys)."""
    from accord_amd import CommandStore
    outs = []
    with CommandStore(device=0, key_lo=key_lo, key_hi=key_lo + nkeys, window=0) as st:
        for s in streams:
            st.upload(s)

            def fold(f, ex, out):
                r = st.max_conflicts_fold(first=f, exec_at=ex, out=out)
                return r[:5], r[5]
            outs.append(fold_all(fold, s.n))
        gst = st.max_conflicts_state()
    state = None
    for s, (g, gchosen) in zip(streams, outs):
        st0 = state

        def fold(f, ex, out):
            nonlocal state
            o, state, folded = O.max_conflicts(s, key_lo, nkeys, state if f else st0, first=f, exec_at=ex, out=out,
                                               intervals=True)
            return o, folded
        want, chosen = fold_all(fold, s.n)
        assert chosen == gchosen
        for a, b, name in zip(g, want, ("msb", "lsb", "node", "present", "fast")):
            assert np.array_equal(a, b), (name, int(np.flatnonzero(a != b)[0]))
    for a, b in zip(gst, state):
        assert np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,ks,rf,rl,seed,accept,kinds,window", [
    (3000, 3, 60, 0.3, 12, 21, False, True, (0, 60)),
    (3000, 3, 60, 0.3, 12, 22, True, True, (10, 30)),           # ranges clipped to the store
    (20000, 4, 500, 0.2, 200, 23, True, False, (0, 500)),       # long ranges: many pairs per txn
    (20000, 8, 5000, 0.05, 2000, 24, False, False, (1000, 2000)),
    (5000, 2, 10, 0.5, 5, 25, True, True, (0, 10)),             # hot keys, every txn conflicts
])
def test_gpu_ranges_vs_interval_oracle(gpu_device, n, k, ks, rf, rl, seed, accept, kinds, window):
    from test_oracle_stream import with_random_kinds
    s = generate_stream(n, k, ks, 0.99, 0.5, seed=seed, range_frac=rf, range_len_max=rl)
    if kinds:
        s = no_key_xsp(with_random_kinds(s, seed))
        # some range txns become ExclusiveSyncPoints (markExclusiveSyncPoint: read nothing, fast)
        lsb = s.lsb.copy()
        rng = np.random.default_rng(seed)
        pick = ((lsb & np.uint64(1)) == 1) & (rng.random(s.n) < 0.3)
        lsb[pick] = (lsb[pick] & ~np.uint64(0xE)) | np.uint64(4 << 1)
        s = dataclasses.replace(s, lsb=lsb)
    if accept:
        s = s.accept(frac=0.5, max_delay=500, seed=seed)
    lo, nk = window
    sub = s.restrict_keys(lo, lo + nk, drop_empty=False)
    check_window([sub.prefix(sub.n // 2), sub], lo, nk)
