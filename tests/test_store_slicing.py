"""Range commands sliced to each CommandStore's ranges (SURVEY.md §7 "Hard parts" 5).

A store registers a range command with its ranges sliced Minimal to the store's own ranges
(InMemoryCommandStore.update, impl/InMemoryCommandStore.java:757-760) and slices the query the same
way (mapReduceRangesInternal :886); each intersecting *sliced* range maps to the txn (:950-959).
After PreAccept.reduce (messages/PreAccept.java:140-156) the per-store slices stay separate RangeDeps
entries (primitives/RangeDeps.java:462-465).  The oracle's or_stream_deps_stores restates that
(per store: Keys.slice + AbstractRanges.sliceMinimal, then the union of the parts); these CPU tests
pin it by a hand-derived KAT and by properties against the single-store restatements."""
import numpy as np
import pytest

from accord_amd import generate_stream, keydeps_str, rangedeps_str
import oracle_lib as O
from kat_util import kat_stream

END = O.KEY_END

# Two stores split at ordinal 10: store 0 = (-inf, 9], store 1 = (9, +inf).
#  t0 W ranges (5,15]    registered in store 0 as (5,9], in store 1 as (9,15]
#  t1 R key 12           store 1: (9,15] contains 12 -> RangeDeps {(9,15]: t0}   (single store: (5,15])
#  t2 R ranges (0,20]    store 0 query (0,9] meets (5,9]; store 1 query (9,20] meets (9,15]
#                        -> {(5,9]: t0, (9,15]: t0}; KeyDeps: key 12 holds only the Read t1 -> {}
#  t3 W key 3            store 0: t2's (0,9] contains 3, t0's (5,9] does not -> {(0,9]: t2}
#  t4 W ranges (8,11]    store 0 piece (8,9] meets t0's (5,9] and t2's (0,9]; store 1 piece (9,11]
#                        meets (9,15] (t0) and (9,20] (t2); KeyDeps: no key in (8,11] -> {}
#                        -> {(0,9]: t2, (5,9]: t0, (9,15]: t0, (9,20]: t2}
KAT = {
    "window": 16,
    "txns": [
        {"kind": "W", "ranges": [[5, 15]]},
        {"kind": "R", "keys": [12]},
        {"kind": "R", "ranges": [[0, 20]]},
        {"kind": "W", "keys": [3]},
        {"kind": "W", "ranges": [[8, 11]]},
    ],
    "bounds": [0, 10, END],
    "expect_range": [
        "{}",
        "{(9,15]:[[1,1000000,3(RW),1]]}",
        "{(5,9]:[[1,1000000,3(RW),1]], (9,15]:[[1,1000000,3(RW),1]]}",
        "{(0,9]:[[1,1000002,1(RR),3]]}",
        "{(0,9]:[[1,1000002,1(RR),3]], (5,9]:[[1,1000000,3(RW),1]], (9,15]:[[1,1000000,3(RW),1]], "
        "(9,20]:[[1,1000002,1(RR),3]]}",
    ],
    "expect_range_single": [
        "{}",
        "{(5,15]:[[1,1000000,3(RW),1]]}",
        "{(5,15]:[[1,1000000,3(RW),1]]}",
        "{(0,20]:[[1,1000002,1(RR),3]]}",
        "{(0,20]:[[1,1000002,1(RR),3]], (5,15]:[[1,1000000,3(RW),1]]}",
    ],
}


@pytest.mark.parametrize("literal", [True, False])
def test_kat_two_stores(literal):
    s = kat_stream(KAT)
    d = O.deps_stores(s, KAT["window"], KAT["bounds"], literal=literal)
    got = [rangedeps_str(*d.range_deps(i), s) for i in range(s.n)]
    assert got == KAT["expect_range"]
    one = O.deps_literal(s, KAT["window"])
    assert [rangedeps_str(*one.range_deps(i), s) for i in range(s.n)] == KAT["expect_range_single"]
    # KeyDeps do not depend on the split: keys partition the stores
    for i in range(s.n):
        assert keydeps_str(*d.key_deps(i), s) == keydeps_str(*one.key_deps(i), s)


def test_one_open_store_is_the_single_store():
    s = generate_stream(3000, 6, 2000, 0.99, 0.5, seed=71, range_frac=0.2, range_len_max=400)
    a = O.deps_stores(s, 64, [0, END])
    assert a.first_difference(O.deps_fast(s, 64)) is None


@pytest.mark.parametrize("nstores", [2, 3, 8])
def test_key_txns_unaffected_by_split(nstores):
    s = generate_stream(4000, 8, 3000, 0.99, 0.5, seed=72)
    a = O.deps_stores(s, 128, O.store_bounds(3000, nstores))
    assert a.first_difference(O.deps_fast(s, 128)) is None


@pytest.mark.parametrize("nstores,rl,W", [(2, 40, 16), (3, 400, 64), (8, 2000, 64)])
def test_stores_literal_equals_fast(nstores, rl, W):
    s = generate_stream(2500, 6, 5000, 0.99, 0.5, seed=73 + nstores, range_frac=0.15, range_len_max=rl)
    b = O.store_bounds(5000, nstores)
    lit = O.deps_stores(s, W, b, literal=True)
    fast = O.deps_stores(s, W, b)
    assert lit.first_difference(fast) is None


@pytest.mark.parametrize("nstores", [2, 8])
def test_split_pieces_cover_the_single_store_ranges(nstores):
    # every (range, txn) entry of the single store is the union of its store pieces: the pieces of
    # a txn's RangeDeps lie inside its single-store ranges, and the txnIds are the same set
    ks = 4000
    s = generate_stream(2000, 4, ks, 0.99, 0.5, seed=79, range_frac=0.3, range_len_max=1500)
    b = O.store_bounds(ks, nstores)
    split = O.deps_stores(s, 64, b)
    one = O.deps_fast(s, 64)
    cuts = np.array(b[1:-1], np.int64) - 1            # internal boundaries as range points
    for i in range(s.n):
        ss, se, sv, _ = split.range_deps(i)
        os_, oe, ov, _ = one.range_deps(i)
        assert set(sv.tolist()) == set(ov.tolist()), i
        for a, z in zip(ss.tolist(), se.tolist()):
            # a piece never straddles a store boundary
            assert not np.any((cuts > a) & (cuts < z)), (i, a, z)
            assert np.any((os_ <= a) & (z <= oe)), (i, a, z)
