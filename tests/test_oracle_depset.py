"""Oracle deps-set operations (SURVEY.md §8a a9 linearUnion / Deps.merge, a10 slice / invert /
trimUnusedValues) against the reference tests' canonical model, restated from
test:primitives/KeyDepsTest.java:376-455 (select / with / merge / invertCanonical) and :504-564
(random Ranges slicing, nested selects, no-op merges), plus the RangeDeps stabbing property of
test:primitives/RangeDepsTest.java:87-148 and hand-derived known answers for RangeDeps.slice."""
import numpy as np
import pytest

import oracle_lib as O
from depset_util import canon, from_canon, invert_canon, random_depset, random_select


def _eq(a, b):
    d = a.first_difference(b)
    assert d is None, d


def _contains(ss, se, key):
    return any(s < key <= e for s, e in zip(ss, se))


@pytest.mark.parametrize("seed", range(6))
def test_union_equals_canonical_union(seed):
    rng = np.random.default_rng(100 + seed)
    n, G = 40, 1 + seed % 4
    parts = [random_depset(rng, n, 300, 60, 6, 3, 12, shared_keys=np.arange(20)) for _ in range(G)]
    got = O.deps_union([from_canon(p) for p in parts])
    want = []
    for i in range(n):
        kd, rd = {}, {}
        for p in parts:
            for k, v in p[i][0].items():
                kd.setdefault(k, set()).update(v)
            for k, v in p[i][1].items():
                rd.setdefault(k, set()).update(v)
        want.append(({k: sorted(v) for k, v in kd.items()}, {k: sorted(v) for k, v in rd.items()}))
    _eq(got, from_canon(want))


def test_union_with_self_and_empty_is_identity():
    rng = np.random.default_rng(7)
    a = from_canon(random_depset(rng, 30, 200, 50, 5, 3, 10))
    empty = from_canon([({}, {})] * 30)
    _eq(O.deps_union([a, a]), a)
    _eq(O.deps_union([a, empty]), a)
    _eq(O.deps_union([empty, a]), a)


@pytest.mark.parametrize("seed", range(6))
def test_keydeps_slice_equals_canonical_select(seed):
    rng = np.random.default_rng(200 + seed)
    n, ks = 50, 80
    txns = random_depset(rng, n, 400, ks, 8, 0, 10)
    d = from_canon(txns)
    nested, nested_txns = None, None
    for _ in range(3):
        ss, se = random_select(rng, ks, 4)
        got = O.deps_slice(d, ss, se)
        want = [({k: v for k, v in kd.items() if _contains(ss, se, k)}, {}) for kd, _ in txns]
        _eq(got, from_canon(want))
        # no-op merge of a selection with its source (KeyDepsTest.java:550)
        _eq(O.deps_union([d, got]), d)
        if nested is None:
            nested, nested_txns = got, want
        else:
            nested = O.deps_slice(nested, ss, se)
            nested_txns = [({k: v for k, v in kd.items() if _contains(ss, se, k)}, {}) for kd, _ in nested_txns]
            _eq(nested, from_canon(nested_txns))


def test_keydeps_slice_per_txn_ranges():
    rng = np.random.default_rng(9)
    n, ks = 40, 60
    txns = random_depset(rng, n, 300, ks, 8, 0, 8)
    d = from_canon(txns)
    off, S, E, want = [0], [], [], []
    for kd, _ in txns:
        ss, se = random_select(rng, ks, 3)
        S += list(ss); E += list(se); off.append(len(S))
        want.append(({k: v for k, v in kd.items() if _contains(ss, se, k)}, {}))
    _eq(O.deps_slice(d, S, E, sel_off=off), from_canon(want))


@pytest.mark.parametrize("seed", range(6))
def test_rangedeps_slice_single_range_equals_brute_force(seed):
    """One select range: the collector reports every intersecting range (checkpoint + scan
    matches flushed by the run) except when the run is empty, see the KAT below."""
    rng = np.random.default_rng(300 + seed)
    n, ks = 60, 200
    txns = random_depset(rng, n, 300, ks, 0, 6, 8)
    d = from_canon(txns)
    for _ in range(4):
        ss, se = random_select(rng, ks, 1)
        got = O.deps_slice(d, ss, se)
        for i, (_, rd) in enumerate(txns):
            keys = sorted(k for k in rd if rd[k])
            inter = [k for k in keys if len(ss) and ss[0] < k[1] and k[0] < se[0]]
            # the run: ranges starting inside [qs, qe), plus the floor range (last start < qs)
            # when it reaches past qs; everything else is a buffered scan/checkpoint match
            below = [k for k in keys if len(ss) and k[0] < ss[0]]
            run = [k for k in inter if ss[0] <= k[0] or (below and k == below[-1])]
            gs, ge, gv, gx = got.range_deps(i)
            got_keys = list(zip(gs.tolist(), ge.tolist()))
            assert got_keys == (inter if run else []), (i, got_keys, inter)


def test_rangedeps_slice_kats():
    """Hand-derived from CheckpointIntervalArray.forEach (utils/CheckpointIntervalArray.java:100-221)
    and RangeDeps.RangeCollector (primitives/RangeDeps.java:727-797).
    RangeDeps {(0,100]:[t0], (50,60]:[t1]} (sorted by start):
      * select (70,80]: end = CEIL(80) = 2, floor = 1 ((50,60] ends <= 70 so start = 2); (0,100]
        is a scan match buffered out of order, the run [2,2) is empty so accept() never flushes it
        -> rangesCount 0 -> the empty RangeDeps.
      * select (55,80]: floor = 1, (50,60] ends after 55 so start = 1, run [1,2) flushes the
        buffered (0,100] first -> both ranges -> the input unchanged.
      * select (70,80], (90,95]: second query: minIndex = 2 = n -> nothing; still empty.
      * select (5,10], (55,80]: first query buffers nothing (floor 0 = (0,100] itself, start 0, run
        [0,1) reported), second: minIndex 1, run [1,2) -> both.
      * select (0,40]: exact start match floor = start = 0, end = CEIL(40) = 1 -> (0,100] only,
        t1 trimmed (trimUnusedValues)."""
    d = from_canon([({}, {(0, 100): [0], (50, 60): [1]})])
    cases = [
        (([70], [80]), {}),
        (([55], [80]), {(0, 100): [0], (50, 60): [1]}),
        (([70, 90], [80, 95]), {}),
        (([5, 55], [10, 80]), {(0, 100): [0], (50, 60): [1]}),
        (([0], [40]), {(0, 100): [0]}),
    ]
    for (ss, se), want in cases:
        _eq(O.deps_slice(d, ss, se), from_canon([({}, want)]))


@pytest.mark.parametrize("seed", range(4))
def test_invert_equals_canonical_inverse(seed):
    rng = np.random.default_rng(400 + seed)
    n = 40
    txns = random_depset(rng, n, 200, 50, 8, 5, 12)
    d = from_canon(txns)
    for side in (0, 1):
        off, ints = O.deps_invert(d, bool(side))
        for i, t in enumerate(txns):
            m = t[side]
            vals = sorted({v for k in m for v in m[k]})
            inv = invert_canon(m)
            seg = ints[off[i]:off[i + 1]]
            assert len(seg) == len(vals) + sum(len(v) for v in m.values())
            start = len(vals)
            for r, v in enumerate(vals):
                assert seg[r] == start + len(inv[v])
                assert list(seg[start:seg[r]]) == inv[v]
                start = seg[r]


def test_ops_on_stream_deps():
    """The ops on real PreAccept deps of a mixed key/range stream: slice to the whole keyspace is
    the identity; union with a slice is the identity; slice then invert is consistent."""
    from accord_amd import generate_stream
    s = generate_stream(1500, 4, 500, 0.9, 0.5, range_frac=0.2, range_len_max=60, seed=5)
    d = O.deps_fast(s, 64)
    _eq(O.deps_slice(d, [0], [1 << 31]), d)
    half = O.deps_slice(d, [0], [250])
    _eq(O.deps_union([d, half]), d)
    _eq(O.deps_union([half, d]), d)
    off, ints = O.deps_invert(half)
    assert int(off[-1]) == int(half.kd_val_off[-1]) + int(half.kd_k2v_off[-1] - half.kd_key_off[-1])
