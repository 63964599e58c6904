"""The oracle's primitives against the reference's own property tests, restated.

* Timestamp/TxnId order and identity (primitives/Timestamp.java:208-249, Node.java:134-137)
* KeyDepsTest canonical model (test:primitives/KeyDepsTest.java:304-431): KeyDeps built from a
  TreeMap<Key, TreeSet<TxnId>> in all four in-order/reverse key/value combinations equals the
  canonical keys, per-key lists and the exact toString.
* KeyDepsTest merge/with (:75-114, :242-283): linearUnion equals the canonical set union.
* SearchableRangeListTest (test:utils/SearchableRangeListTest.java:61-115): stabbing returns
  exactly the ranges containing the key, ascending.
"""
import numpy as np
import pytest

import accord_amd as A
import oracle_lib as O

MASK64 = (1 << 64) - 1


def tid(epoch, hlc, flags, node):
    msb = ((epoch << 15) | (hlc >> 48)) & MASK64
    lsb = ((hlc << 16) | flags) & MASK64
    return (msb, lsb, node)


def test_compare_msb_unsigned():
    a = (0x8000000000000000, 0, 1)
    b = (0x0000000000000001, 0, 1)
    assert O.ts_compare(a, b) > 0 and O.ts_compare(b, a) < 0


def test_compare_node_signed():
    # SURVEY.md §8c KAT 7: Node.Id.compareTo is Integer.compare (signed)
    a = tid(1, 10, 2, -5)
    b = tid(1, 10, 2, 3)
    assert O.ts_compare(a, b) < 0


def test_domain_bit_and_rejected_flag_not_identity():
    # SURVEY.md §8c KAT 6: flags & 0x1E only; equals masks with 0xFFFFFFFFFFFF001E
    a = tid(1, 10, 2, 1)
    b = tid(1, 10, 3, 1)           # domain bit differs
    c = tid(1, 10, 2 | 0x8000, 1)  # REJECTED differs
    d = tid(1, 10, 4, 1)           # kind differs -> identity differs
    assert O.ts_compare(a, b) == 0 and O.ts_equals(a, b)
    assert O.ts_compare(a, c) == 0 and O.ts_equals(a, c)
    assert O.ts_compare(a, d) < 0 and not O.ts_equals(a, d)


def test_compare_hlc_then_flags():
    assert O.ts_compare(tid(1, 9, 4, 1), tid(1, 10, 0, 0)) < 0
    assert O.ts_compare(tid(1, 10, 2, 9), tid(1, 10, 4, 0)) < 0
    assert O.ts_compare(tid(2, 0, 0, 0), tid(1, 1 << 47, 0, 0)) > 0


# ---------------------------------------------------------------- KeyDepsTest canonical model
def random_deps(rng):
    """KeyDepsTest.Deps.generate (:318-374) with IntKey keys (no hash collisions)."""
    epoch_range, hlc_range = 3, 500
    unique = int(rng.integers(1, int(hlc_range * epoch_range * 0.66)))
    node_range = int(rng.integers(1, 4))
    unique_keys = int(rng.integers(2, 200))
    key_range = int(rng.integers(unique_keys + 10, 400))
    total = int(rng.integers(1, 1000))
    keys = sorted(rng.choice(key_range, size=unique_keys, replace=False).tolist())
    ids = set()
    while len(ids) < unique:
        ids.add((int(rng.integers(0, epoch_range)), int(rng.integers(0, hlc_range)), int(rng.integers(0, node_range))))
    ids = sorted(ids)  # (epoch, hlc, node) order == TxnId order for flags 0
    tbl = [tid(e, h, 0, nd) for (e, h, nd) in ids]
    canonical = {}
    for _ in range(total):
        k = keys[int(rng.integers(0, unique_keys))]
        v = int(rng.integers(0, unique))
        canonical.setdefault(k, set()).add(v)
    return tbl, canonical


def tostr(tbl, canonical):
    parts = []
    for k in sorted(canonical):
        parts.append(f"{k}:[" + ", ".join(A.txn_id_str(*tbl[v]) for v in sorted(canonical[k])) + "]")
    return "{" + ", ".join(parts) + "}"


def built_str(tbl, keys, vals, k2v):
    if len(keys) == len(k2v):
        return "{}"
    parts, t = [], len(keys)
    for k, key in enumerate(keys):
        ids = []
        while t < k2v[k]:
            ids.append(A.txn_id_str(*tbl[vals[k2v[t]]]))
            t += 1
        parts.append(f"{int(key)}:[" + ", ".join(ids) + "]")
    return "{" + ", ".join(parts) + "}"


@pytest.mark.parametrize("seed", range(40))
@pytest.mark.parametrize("order", [(True, True), (True, False), (False, True), (False, False)])
def test_keydeps_builder_canonical(seed, order):
    rng = np.random.default_rng(seed)
    tbl, canonical = random_deps(rng)
    in_order_keys, in_order_values = order
    adds_k, adds_v = [], []
    for k in (sorted(canonical) if in_order_keys else sorted(canonical, reverse=True)):
        for v in (sorted(canonical[k]) if in_order_values else sorted(canonical[k], reverse=True)):
            adds_k.append(k)
            adds_v.append(v)
    tm = np.array([t[0] for t in tbl], np.uint64)
    tl = np.array([t[1] for t in tbl], np.uint64)
    tn = np.array([t[2] for t in tbl], np.int32)
    keys, vals, k2v = O.keydeps_build(adds_k, adds_v, tm, tl, tn)
    assert list(keys) == sorted(canonical)
    uniq = sorted(set().union(*canonical.values()))
    assert list(vals) == uniq
    # layout: header = end offsets starting at keyCount (KeyDeps.java:153-169)
    assert k2v[len(keys) - 1] == len(k2v)
    t = len(keys)
    for ki, k in enumerate(keys):
        got = [int(vals[k2v[j]]) for j in range(t, k2v[ki])]
        assert got == sorted(canonical[int(k)])
        t = k2v[ki]
    assert built_str(tbl, keys, vals, k2v) == tostr(tbl, canonical)


def test_builder_duplicate_values_and_empty():
    tbl = [tid(1, h, 0, 1) for h in range(5)]
    tm = np.array([t[0] for t in tbl], np.uint64)
    tl = np.array([t[1] for t in tbl], np.uint64)
    tn = np.array([t[2] for t in tbl], np.int32)
    keys, vals, k2v = O.keydeps_build([3, 3, 3, 5], [2, 1, 2, 4], tm, tl, tn)
    assert list(keys) == [3, 5] and list(vals) == [1, 2, 4]
    assert list(k2v) == [4, 5, 0, 1, 2]
    keys, vals, k2v = O.keydeps_build([], [], tm, tl, tn)
    assert len(keys) == 0 and len(k2v) == 0


def test_builder_key_visited_twice_throws():
    # RelationMultiMap.java:234-238: "Key ... has been visited more than once"
    tbl = [tid(1, h, 0, 1) for h in range(5)]
    tm = np.array([t[0] for t in tbl], np.uint64)
    tl = np.array([t[1] for t in tbl], np.uint64)
    tn = np.array([t[2] for t in tbl], np.int32)
    assert O.keydeps_build([5, 3, 5], [0, 1, 2], tm, tl, tn) is None


@pytest.mark.parametrize("seed", range(25))
def test_keydeps_union_canonical(seed):
    rng = np.random.default_rng(100 + seed)
    tbl, ca = random_deps(rng)
    rng2 = np.random.default_rng(200 + seed)
    # second deps over the same table
    cb = {}
    for _ in range(int(rng2.integers(1, 600))):
        k = int(rng2.integers(0, 400))
        cb.setdefault(k, set()).add(int(rng2.integers(0, len(tbl))))
    tm = np.array([t[0] for t in tbl], np.uint64)
    tl = np.array([t[1] for t in tbl], np.uint64)
    tn = np.array([t[2] for t in tbl], np.int32)

    def build(c):
        ks, vs = [], []
        for k in sorted(c):
            for v in sorted(c[k]):
                ks.append(k)
                vs.append(v)
        return O.keydeps_build(ks, vs, tm, tl, tn)

    u = O.keydeps_union(build(ca), build(cb), tm, tl, tn)
    canon = {}
    for c in (ca, cb):
        for k, vs in c.items():
            canon.setdefault(k, set()).update(vs)
    assert built_str(tbl, *u) == tostr(tbl, canon)
    assert list(u[1]) == sorted(set().union(*canon.values()))


@pytest.mark.parametrize("seed", range(20))
def test_stab_key_brute_force(seed):
    rng = np.random.default_rng(seed)
    nr = int(rng.integers(1, 200))
    st = rng.integers(0, 1000, size=nr)
    ln = rng.integers(1, 100, size=nr)
    order = np.lexsort((st + ln, st))
    starts, ends = st[order], (st + ln)[order]
    for key in rng.integers(0, 1100, size=50):
        want = [i for i in range(nr) if starts[i] < key <= ends[i]]
        assert list(O.stab_key(starts, ends, int(key))) == want
