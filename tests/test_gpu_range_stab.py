"""SearchableRangeList stabbing of RangeDeps built on the device:
accord_deps_range_stab against the brute force of SearchableRangeListTest
(test/.../utils/SearchableRangeListTest.java:61-115: every range intersecting the query), mapped to
RangeDeps.computeTxnIds (the txnIds of the matching ranges, ascending unique).

The CPU half checks the brute force itself against the oracle's or_stab_key on key queries."""
import numpy as np
import pytest

import oracle_lib as O
from accord_amd import CommandStore, generate_stream
from depset_util import from_canon, random_depset


def stab_brute(p, q_off, qs, qe):
    """off[nq+1], txns: for every query (qs, qe] of txn i, the txnIds of txn i's RangeDeps ranges
    (s, e] with s < qe and qs < e (Range.compareIntersecting), ascending unique."""
    off, out = [0], []
    for i in range(p.n):
        rs, re, vals, r2v = p.range_deps(i)
        nr = len(rs)
        for q in range(int(q_off[i]), int(q_off[i + 1])):
            hit = set()
            for r in range(nr):
                if rs[r] < qe[q] and qs[q] < re[r]:
                    b = nr if r == 0 else int(r2v[r - 1])
                    hit.update(int(vals[int(x)]) for x in r2v[b:int(r2v[r])])
            out += sorted(hit)
            off.append(len(out))
    return np.asarray(off, np.uint32), np.asarray(out, np.uint32)


def random_queries(rng, n, keyspace, max_q, key_frac=0.5, max_len=None):
    q_off = np.zeros(n + 1, np.uint32)
    cnt = rng.integers(0, max_q + 1, size=n)
    q_off[1:] = np.cumsum(cnt)
    nq = int(q_off[-1])
    a = rng.integers(0, keyspace, size=nq)
    ln = rng.integers(1, (max_len or keyspace // 8) + 1, size=nq)
    key = rng.random(nq) < key_frac
    qs = np.where(key, a, a).astype(np.uint32)
    qe = np.where(key, a + 1, a + ln).astype(np.uint32)       # a key k is (k-1, k]
    return q_off, qs, qe


def test_brute_force_matches_or_stab_key():
    rng = np.random.default_rng(3)
    p = from_canon(random_depset(rng, 30, 200, 500, 3, 12, 5))
    for i in range(p.n):
        rs, re, vals, r2v = p.range_deps(i)
        for k in rng.integers(0, 520, size=20):
            idx = O.stab_key(rs, re, int(k)) if hasattr(O, "stab_key") else None
            q_off = np.zeros(p.n + 1, np.uint32)
            q_off[i + 1:] = 1
            off, got = stab_brute(p, q_off, np.array([k - 1], np.uint32), np.array([k], np.uint32))
            nr = len(rs)
            want = set()
            for r in range(nr):
                if rs[r] < k <= re[r]:
                    b = nr if r == 0 else int(r2v[r - 1])
                    want.update(int(vals[int(x)]) for x in r2v[b:int(r2v[r])])
            assert got.tolist() == sorted(want)
            if idx is not None:
                assert sorted(idx) == [r for r in range(nr) if rs[r] < k <= re[r]]


@pytest.mark.gpu
@pytest.mark.parametrize("seed,max_ranges,keyspace", [(1, 8, 400), (2, 40, 2000), (3, 200, 100000), (4, 600, 3000)])
def test_stab_random_depsets(gpu_device, seed, max_ranges, keyspace):
    rng = np.random.default_rng(seed)
    p = from_canon(random_depset(rng, 80, 5000, keyspace, 2, max_ranges, 6))
    q_off, qs, qe = random_queries(rng, p.n, keyspace + 10, 12)
    with CommandStore(device=0, key_lo=0, key_hi=1 << 20, window=64) as src, \
            CommandStore(device=0, key_lo=0, key_hi=1 << 20, window=64) as st:
        src.upload_deps(p)
        off, txns = st.range_stab(src, q_off, qs, qe)
    woff, wtx = stab_brute(p, q_off, qs, qe)
    assert np.array_equal(off, woff)
    assert np.array_equal(txns, wtx)


@pytest.mark.gpu
def test_stab_nested_long_ranges(gpu_device):
    # every range spans most of the keyspace: long checkpoint lists, every query hits many ranges
    rng = np.random.default_rng(9)
    txns = []
    for t in range(6):
        rd = {}
        for _ in range(300):
            s = int(rng.integers(0, 100))
            rd[(s, s + int(rng.integers(500, 1000)))] = sorted(set(int(v) for v in rng.integers(0, 2000, size=3)))
        txns.append(({}, rd))
    p = from_canon(txns)
    q_off, qs, qe = random_queries(rng, p.n, 1200, 40, max_len=50)
    with CommandStore(device=0, key_lo=0, key_hi=1 << 20, window=64) as src, \
            CommandStore(device=0, key_lo=0, key_hi=1 << 20, window=64) as st:
        src.upload_deps(p)
        off, txns_got = st.range_stab(src, q_off, qs, qe)
    woff, wtx = stab_brute(p, q_off, qs, qe)
    assert np.array_equal(off, woff) and np.array_equal(txns_got, wtx)


@pytest.mark.gpu
def test_stab_computed_mixed_stream(gpu_device):
    # the RangeDeps the pipeline computed for a mixed key/range stream (config-3 shape, reduced)
    s = generate_stream(20000, 4, 3000, 0.99, 0.5, range_frac=0.2, range_len_max=200, seed=27)
    rng = np.random.default_rng(27)
    with CommandStore(device=0, key_lo=0, key_hi=3000, window=128) as st, \
            CommandStore(device=0, key_lo=0, key_hi=3000, window=128) as op:
        st.upload(s)
        st.compute()
        p = st.download()
        q_off, qs, qe = random_queries(rng, p.n, 3000, 3, key_frac=0.7, max_len=300)
        off, txns = op.range_stab(st, q_off, qs, qe)
    woff, wtx = stab_brute(p, q_off, qs, qe)
    assert np.array_equal(off, woff) and np.array_equal(txns, wtx)
    assert int(off[-1]) > 0


@pytest.mark.gpu
def test_stab_empty_and_degenerate(gpu_device):
    p = from_canon([({}, {}), ({}, {(5, 9): [1, 2]}), ({}, {(0, 3): [4], (3, 6): [5]})])
    q_off = np.array([0, 1, 3, 6], np.uint32)
    qs = np.array([0, 9, 5, 2, 3, 7], np.uint32)
    qe = np.array([10, 10, 6, 3, 4, 7], np.uint32)    # last: empty query (qs == qe) -> nothing
    with CommandStore(device=0, key_lo=0, key_hi=64, window=8) as src, \
            CommandStore(device=0, key_lo=0, key_hi=64, window=8) as st:
        src.upload_deps(p)
        off, txns = st.range_stab(src, q_off, qs, qe)
    # txn 0: no RangeDeps; txn 1: (9,10] misses (5,9], (5,6] hits it; txn 2: (2,3] -> (0,3] only
    # (touching (3,6] at 3 is no intersection), (3,4] -> (3,6]; (7,7] empty
    assert off.tolist() == [0, 0, 0, 2, 3, 4, 4]
    assert txns.tolist() == [1, 2, 4, 5]
