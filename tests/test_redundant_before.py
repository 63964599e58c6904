"""RedundantBefore.collectDeps (local/RedundantBefore.java:181-190, 418-421) and its union into the
PreAccept result (messages/PreAccept.java:260-263).

CPU: the oracle's literal restatement (ReducingRangeMap.foldl over the (starts[], values[]) map with
inclusiveEnds, utils/ReducingRangeMap.java:111-194) against hand-derived known answers and against a
direct model of the same rule (every entry a key lies in / a range intersects, once, ascending;
Entry.outOfBounds :260-263; NONE skipped).  GPU: accord_redundant_before_set + compute ==
oracle deps_union(deps_fast, redundant_collect), byte for byte through the C ABI.
"""
import numpy as np
import pytest

from accord_amd import NO_TXN, CommandStore, Stream, generate_stream, rangedeps_str
import oracle_lib as O
from depset_util import canon


def stream_of(keys_or_ranges, epoch=5):
    """Tiny stream: a list of ('k', [keys]) / ('r', [(s, e), ...]); txn i has TxnId (epoch, hlc=i+1)."""
    n = len(keys_or_ranges)
    msb = np.array([(epoch << 15) for _ in range(n)], np.uint64)
    lsb = np.array([((i + 1) << 16) | (0 if t == 'k' else 1) for i, (t, _) in enumerate(keys_or_ranges)], np.uint64)
    node = np.ones(n, np.int32)
    ko, kk, ro, rs, re = [0], [], [0], [], []
    for t, v in keys_or_ranges:
        if t == 'k':
            kk += list(v)
        else:
            rs += [a for a, _ in v]; re += [b for _, b in v]
        ko.append(len(kk)); ro.append(len(rs))
    u = lambda a: np.asarray(a, np.uint32)
    return Stream(msb, lsb, node, u(ko), u(kk), u(ro), u(rs), u(re))


def model(s, es, ee, sep, eep, bound, min_epoch):
    """Direct statement of the rule: per txn {(entry range): {bound}} (canonical map)."""
    out = []
    for t in range(s.n):
        em = int(s.exec_msb[t]) if s.exec_msb is not None else int(s.msb[t])
        ep = em >> 15
        touched = set()
        r0, r1 = int(s.rng_off[t]), int(s.rng_off[t + 1])
        if r1 > r0:
            for r in range(r0, r1):
                a, b = int(s.rng_start[r]), int(s.rng_end[r])
                touched |= {x for x in range(len(es)) if a < ee[x] and es[x] < b}
        else:
            for k in s.key_ord[s.key_off[t]:s.key_off[t + 1]]:
                touched |= {x for x in range(len(es)) if es[x] < int(k) <= ee[x]}
        rd = {}
        for x in sorted(touched):
            if bound[x] == NO_TXN or ep < sep[x] or min_epoch >= eep[x]:
                continue
            rd[(int(es[x]), int(ee[x]))] = [int(bound[x])]
        out.append(({}, rd))
    return out


def test_kat_keys_inclusive_ends_and_bounds():
    # entries (0,5] (5,8] (10,20]; txn 0 keys {5, 10}: 5 is in (0,5] (inclusive end), 10 in no entry
    # (the gap (8,10] is a null value and 10 is the start of (10,20]); txn 1 keys {6, 7, 15}: (5,8]
    # once for both keys, then (10,20]
    s = stream_of([('k', [5, 10]), ('k', [6, 7, 15]), ('k', [21])])
    es, ee = [0, 5, 10], [5, 8, 20]
    sep, eep, bound = [0, 0, 0], [100, 100, 100], [0, 1, 0]
    d = O.redundant_collect(s, es, ee, sep, eep, bound, 0)
    assert canon(d, 0) == ({}, {(0, 5): [0]})
    assert canon(d, 1) == ({}, {(5, 8): [1], (10, 20): [0]})
    assert canon(d, 2) == ({}, {})
    # RangeDeps layout: ranges ascending, txnIds unique ascending, keysToTxnIds = header then ranks
    rs, re, rv, r2v = d.range_deps(1)
    assert list(rs) == [5, 10] and list(re) == [8, 20] and list(rv) == [0, 1] and list(r2v) == [3, 4, 1, 0]


def test_kat_ranges_touching_and_duplicate_bounds():
    # (0,8] meets (5,8] but not (8,12] (Range (s,e] and (es,ee] intersect iff s < ee and es < e);
    # (7,9] meets both; two entries with the same bound give one txnId under two ranges
    s = stream_of([('r', [(0, 8)]), ('r', [(7, 9)]), ('r', [(1, 2), (3, 4)])])
    es, ee = [0, 5, 8], [5, 8, 12]
    bound = [2, 2, 1]
    d = O.redundant_collect(s, es, ee, [0, 0, 0], [9, 9, 9], bound, 0)
    assert canon(d, 0) == ({}, {(0, 5): [2], (5, 8): [2]})
    assert canon(d, 1) == ({}, {(5, 8): [2], (8, 12): [1]})
    assert canon(d, 2) == ({}, {(0, 5): [2]})        # both ranges inside one entry: visited once
    rs, re, rv, r2v = d.range_deps(0)
    assert list(rv) == [2] and list(r2v) == [3, 4, 0, 0]


def test_kat_epoch_bounds_and_none():
    # txn epoch 5: entry with startEpoch 6 is out of bounds (executeAt.epoch() < startEpoch); endEpoch
    # <= minEpoch is out of bounds (minEpoch >= endEpoch); a NONE bound adds nothing
    s = stream_of([('k', [1, 11, 21, 31])], epoch=5)
    es, ee = [0, 10, 20, 30], [5, 15, 25, 35]
    sep = [5, 6, 0, 0]
    eep = [6, 9, 3, 9]
    bound = [0, 0, 0, NO_TXN]
    d = O.redundant_collect(s, es, ee, sep, eep, bound, 3)
    assert canon(d, 0) == ({}, {(0, 5): [0]})        # (10,15] startEpoch 6 > 5; (20,25] endEpoch 3 <= 3


def random_map(rng, keyspace, m, n):
    cuts = np.sort(rng.choice(np.arange(1, keyspace), size=2 * m, replace=False))
    es, ee = cuts[0::2].astype(np.uint32), cuts[1::2].astype(np.uint32)
    # about half the neighbours adjacent (shared boundary): the map has no null gap there
    for i in range(1, m):
        if rng.random() < 0.5:
            es[i] = ee[i - 1]
    sep = rng.integers(0, 4, size=m).astype(np.uint64)
    eep = sep + rng.integers(1, 6, size=m).astype(np.uint64)
    bound = rng.integers(0, n, size=m).astype(np.uint32)
    bound[rng.random(m) < 0.15] = NO_TXN
    return es, ee, sep, eep, bound


def with_epochs(s, rng, lo=0, hi=6):
    """Re-stamp TxnIds with epochs in [lo, hi), still ascending (epoch is the top of msb)."""
    ep = np.sort(rng.integers(lo, hi, size=s.n)).astype(np.uint64)
    s.msb = (ep << np.uint64(15)) | (s.msb & np.uint64(0x7FFF))
    return s


@pytest.mark.parametrize("seed,rf", [(1, 0.0), (2, 0.3), (3, 0.9)])
def test_literal_foldl_equals_direct_model(seed, rf):
    rng = np.random.default_rng(seed)
    s = with_epochs(generate_stream(400, 3, 200, 0.0, 0.5, range_frac=rf, range_len_max=40, seed=seed), rng)
    es, ee, sep, eep, bound = random_map(rng, 200, 25, s.n)
    for min_epoch in (0, 2):
        d = O.redundant_collect(s, es, ee, sep, eep, bound, min_epoch)
        want = model(s, es, ee, sep, eep, bound, min_epoch)
        assert [canon(d, t) for t in range(s.n)] == want


# ---------------------------------------------------------------- GPU

def expected(s, W, es, ee, sep, eep, bound, min_epoch):
    base = O.deps_fast(s, W)
    red = O.redundant_collect(s, es, ee, sep, eep, bound, min_epoch)
    return O.deps_union([base, red])


@pytest.mark.gpu
@pytest.mark.parametrize("n,k,ks,z,rf,W,m,seed", [
    (3000, 4, 500, 0.99, 0.0, 64, 40, 21),
    (3000, 8, 2000, 0.99, 0.2, 256, 200, 22),
    (2000, 2, 300, 0.0, 0.5, 16, 10, 23),
])
def test_gpu_redundant_before(gpu_device, n, k, ks, z, rf, W, m, seed):
    rng = np.random.default_rng(seed)
    s = with_epochs(generate_stream(n, k, ks, z, 0.5, range_frac=rf, range_len_max=60, seed=seed), rng)
    es, ee, sep, eep, bound = random_map(rng, ks, m, n)
    want = expected(s, W, es, ee, sep, eep, bound, 1)
    with CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as st:
        st.redundant_before(es, ee, sep, eep, bound, min_epoch=1)
        got = st.calculate_deps_batch(s)
        diff = got.first_difference(want)
        assert diff is None, diff
        # clearing the map restores the plain result
        st.redundant_before()
        got2 = st.calculate_deps_batch(s)
    assert got2.first_difference(O.deps_fast(s, W)) is None


@pytest.mark.gpu
def test_gpu_redundant_before_accept_epochs(gpu_device):
    # Accept batches test the executeAt epoch (Entry.outOfBounds ub = executeAt)
    rng = np.random.default_rng(31)
    s = with_epochs(generate_stream(1500, 4, 400, 0.0, 0.5, seed=31), rng, 0, 3)
    s.exec_msb = s.msb + (np.uint64(2) << np.uint64(15))        # executeAt two epochs later
    s.exec_lsb = s.lsb.copy(); s.exec_node = s.node.copy()
    es, ee, sep, eep, bound = random_map(rng, 400, 30, s.n)
    want = expected(s, 32, es, ee, sep, eep, bound, 0)
    with CommandStore(device=0, key_lo=0, key_hi=400, window=32) as st:
        st.redundant_before(es, ee, sep, eep, bound, min_epoch=0)
        got = st.calculate_deps_batch(s)
    assert got.first_difference(want) is None


@pytest.mark.gpu
def test_gpu_reset_clears_redundant_before_and_max_conflicts(gpu_device):
    # accord_store_reset = an empty CommandStore: RedundantBefore.EMPTY and MaxConflicts.EMPTY too
    rng = np.random.default_rng(41)
    s = with_epochs(generate_stream(2000, 4, 500, 0.99, 0.5, seed=41), rng)
    es, ee, sep, eep, bound = random_map(rng, 500, 40, s.n)
    with CommandStore(device=0, key_lo=0, key_hi=500, window=64) as st, \
            CommandStore(device=0, key_lo=0, key_hi=500, window=64) as fresh:
        st.redundant_before(es, ee, sep, eep, bound, min_epoch=1)
        st.calculate_deps_batch(s)
        st.max_conflicts_fold(s)
        st.reset()
        got = st.calculate_deps_batch(s)
        assert got.first_difference(fresh.calculate_deps_batch(s)) is None
        assert got.first_difference(O.deps_fast(s, 64)) is None
        a = st.max_conflicts_fold(s)
        b = fresh.max_conflicts_fold(s)
        for x, y in zip(a[:5], b[:5]):
            assert np.array_equal(x, y)
        assert a[5] == b[5]
