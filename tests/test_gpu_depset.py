"""GPU deps-set operations through the C ABI (accord_deps_union / _slice / _invert / _upload),
byte-exact against the oracle's restatements (SURVEY.md §8a a9 linearUnion / Deps.merge with
overlapping keys, a10 KeyDeps.slice / RangeDeps.slice / trimUnusedValues / invert)."""
import numpy as np
import pytest

import oracle_lib as O
from accord_amd import CommandStore, IllegalArgumentException, generate_stream
from depset_util import from_canon, random_depset, random_select

pytestmark = pytest.mark.gpu


def _eq(got, want):
    d = got.first_difference(want)
    assert d is None, d


def _store():
    return CommandStore(device=0, key_lo=0, key_hi=1 << 20, window=64)


def _uploaded(p):
    s = _store()
    s.upload_deps(p)
    return s


@pytest.mark.parametrize("G", [1, 2, 3, 5])
def test_union_random_overlapping(gpu_device, G):
    rng = np.random.default_rng(10 + G)
    n = 300
    parts = [from_canon(random_depset(rng, n, 2000, 200, 10, 4, 40, shared_keys=np.arange(40))) for _ in range(G)]
    stores = [_uploaded(p) for p in parts]
    with _store() as out:
        out.union(stores)
        _eq(out.download(), O.deps_union(parts))
    for s in stores:
        s.close()


def test_union_with_empty_txns_and_long_lists(gpu_device):
    rng = np.random.default_rng(3)
    n = 64
    a = random_depset(rng, n, 20000, 50, 4, 2, 3000, shared_keys=np.arange(6))
    b = random_depset(rng, n, 20000, 50, 4, 2, 3000, shared_keys=np.arange(6))
    for i in range(0, n, 5):
        a[i] = ({}, {})
    pa, pb = from_canon(a), from_canon(b)
    with _uploaded(pa) as sa, _uploaded(pb) as sb, _store() as out:
        out.union([sa, sb])
        _eq(out.download(), O.deps_union([pa, pb]))
        out.union([sb, sa, out])     # a source may be the store's own current deps
        _eq(out.download(), O.deps_union([pa, pb]))


def test_union_of_more_than_64_sets(gpu_device):
    # 130 parts (10 distinct sets, repeated): three passes of at most 64 parts each
    rng = np.random.default_rng(17)
    n = 200
    parts = [from_canon(random_depset(rng, n, 3000, 100, 8, 3, 30, shared_keys=np.arange(30))) for _ in range(10)]
    stores = [_uploaded(p) for p in parts]
    try:
        with _store() as out:
            out.union([stores[g % 10] for g in range(130)])
            _eq(out.download(), O.deps_union(parts))
            with pytest.raises(IllegalArgumentException):    # own deps past the first 64 parts
                out.union([stores[g % 10] for g in range(70)] + [out])
    finally:
        for s in stores:
            s.close()


@pytest.mark.parametrize("seed", range(3))
def test_slice_random_shared_and_per_txn(gpu_device, seed):
    rng = np.random.default_rng(40 + seed)
    n, ks = 400, 300
    p = from_canon(random_depset(rng, n, 3000, ks, 12, 6, 30))
    with _uploaded(p) as src, _store() as out:
        for _ in range(3):
            ss, se = random_select(rng, ks, 5)
            out.slice(src, ss, se)
            _eq(out.download(), O.deps_slice(p, ss, se))
        off, S, E = [0], [], []
        for _ in range(n):
            a, b = random_select(rng, ks, 4)
            S += list(a); E += list(b); off.append(len(S))
        out.slice(src, S, E, sel_off=off)
        want = O.deps_slice(p, S, E, sel_off=off)
        _eq(out.download(), want)
        # nested select on the store's own result
        ss, se = random_select(rng, ks, 3)
        out.slice(out, ss, se)
        _eq(out.download(), O.deps_slice(want, ss, se))


def test_rangedeps_slice_kats_on_gpu(gpu_device):
    p = from_canon([({}, {(0, 100): [0], (50, 60): [1]})] * 3)
    cases = [([70], [80]), ([55], [80]), ([70, 90], [80, 95]), ([5, 55], [10, 80]), ([0], [40])]
    with _uploaded(p) as src, _store() as out:
        for ss, se in cases:
            out.slice(src, ss, se)
            _eq(out.download(), O.deps_slice(p, ss, se))


def test_invert_random(gpu_device):
    rng = np.random.default_rng(77)
    p = from_canon(random_depset(rng, 500, 5000, 400, 16, 8, 200))
    with _uploaded(p) as src, _store() as out:
        ko, kv, ro, rv = out.invert(src)
    wko, wkv = O.deps_invert(p, False)
    wro, wrv = O.deps_invert(p, True)
    assert np.array_equal(ko, wko) and np.array_equal(kv, wkv)
    assert np.array_equal(ro, wro) and np.array_equal(rv, wrv)


def test_ops_on_computed_mixed_stream(gpu_device):
    """Ops over the deps the GPU pipeline computed for a mixed key/range stream: slice per
    destination shard, re-union of the slices == the original, invert == oracle."""
    s = generate_stream(20000, 4, 3000, 0.99, 0.5, range_frac=0.2, range_len_max=200, seed=21)
    want = O.deps_fast(s, 128)
    with CommandStore(device=0, key_lo=0, key_hi=3000, window=128) as st, _store() as a, _store() as b, \
            _store() as u:
        st.upload(s)
        st.compute()
        _eq(st.download(), want)
        a.slice(st, [0], [1500])
        b.slice(st, [1500], [3000])
        wa, wb = O.deps_slice(want, [0], [1500]), O.deps_slice(want, [1500], [3000])
        _eq(a.download(), wa)
        _eq(b.download(), wb)
        u.union([a, b])
        _eq(u.download(), O.deps_union([wa, wb]))
        ko, kv, ro, rv = u.invert(st)
        wko, wkv = O.deps_invert(want, False)
        wro, wrv = O.deps_invert(want, True)
        assert np.array_equal(ko, wko) and np.array_equal(kv, wkv)
        assert np.array_equal(ro, wro) and np.array_equal(rv, wrv)


def test_config2_sized_union_of_shard_slices(gpu_device):
    """Size-independent property at config-2 scale (1 Mi txns, Zipf 0.99): the union of the
    slices to a 4-way split of the keyspace is the original deps, and the slices' sizes add up."""
    s = generate_stream(1 << 20, 8, 100_000, 0.99, 0.5, seed=2)
    with CommandStore(device=0, key_lo=0, key_hi=100_000, window=256) as st, _store() as pos:
        st.upload(s)
        st.compute()
        # ranges are (start, end]: every key but ordinal 0 lies in (0, 100000]
        pos.slice(st, [0], [100_000])
        full = pos.download()
        k0 = st.download()
        assert int(full.kd_key_off[-1]) == int(k0.kd_key_off[-1]) - int(np.count_nonzero(k0.kd_keys == 0))
        cuts = [0, 25_000, 50_000, 75_000, 100_000]
        parts = []
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            x = _store()
            x.slice(st, [lo], [hi])
            parts.append(x)
        keys = sum(int(x.download().kd_key_off[-1]) for x in parts)
        assert keys == int(full.kd_key_off[-1])
        with _store() as u:
            u.union(parts)
            _eq(u.download(), full)
        for x in parts:
            x.close()


def test_slice_rejects_bad_ranges(gpu_device):
    p = from_canon([({1: [0]}, {})])
    with _uploaded(p) as src, _store() as out:
        with pytest.raises(IllegalArgumentException):
            out.slice(src, [5, 3], [10, 8])    # overlapping
        with pytest.raises(IllegalArgumentException):
            out.slice(src, [5], [5])           # empty
