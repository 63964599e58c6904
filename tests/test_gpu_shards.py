"""Multi-store union (K6) on one GPU and the RCCL exchange path with a 1-rank communicator.

The stores of a node partition the keyspace (EvenSplit, local/ShardDistributor.java:46-157); the
union of their per-store PartialDeps (PreAccept.reduce, messages/PreAccept.java:140-156) must equal
the deps computed by a single store over the whole keyspace."""
import numpy as np
import pytest

from accord_amd import CommandStore, IllegalArgumentException, generate_stream
import oracle_lib as O

pytestmark = pytest.mark.gpu


def even_split(keyspace, stores):
    return [(b * keyspace // stores, (b + 1) * keyspace // stores) for b in range(stores)]


@pytest.mark.parametrize("nstores", [2, 3, 8])
def test_local_stores_union_equals_single_store(gpu_device, nstores):
    ks, W = 5000, 128
    s = generate_stream(20000, 8, ks, 0.99, 0.5, seed=31)
    stores = []
    try:
        for lo, hi in even_split(ks, nstores):
            st = CommandStore(device=0, key_lo=lo, key_hi=hi, window=W)
            st.upload(s.restrict_keys(lo, hi))
            st.compute()
            stores.append(st)
        with CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as merger:
            merger.merge(stores, txn_lo=0)
            got = merger.download()
    finally:
        for st in stores:
            st.close()
    want = O.deps_fast(s, W)
    assert got.first_difference(want) is None, got.first_difference(want)


@pytest.mark.parametrize("nstores,rl", [(2, 40), (3, 400), (8, 2000)])
def test_local_stores_union_with_ranges(gpu_device, nstores, rl):
    # range txns span store blocks: every store reports them (their KeyDeps cut to its keys, the
    # same range keys in RangeDeps), so the union is RelationMultiMap.linearUnion, not concatenation
    ks, W = 5000, 64
    s = generate_stream(12000, 6, ks, 0.99, 0.5, seed=35, range_frac=0.1, range_len_max=rl)
    stores = []
    try:
        for lo, hi in even_split(ks, nstores):
            st = CommandStore(device=0, key_lo=lo, key_hi=hi, window=W)
            st.upload(s.restrict_keys(lo, hi))
            st.compute()
            stores.append(st)
        with CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as merger:
            merger.merge(stores, txn_lo=0)
            got = merger.download()
    finally:
        for st in stores:
            st.close()
    want = O.deps_fast(s, W)
    assert got.first_difference(want) is None, got.first_difference(want)


def test_exchange_merge_single_rank_ranges(gpu_device):
    ks, W = 4000, 128
    s = generate_stream(20000, 6, ks, 0.99, 0.5, seed=36, range_frac=0.1, range_len_max=300)
    with CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as st:
        st.comm_init(1, 0, CommandStore.comm_unique_id())
        st.upload(s)
        st.compute()
        st.exchange_merge(s.n)
        got = st.download()
    want = O.deps_fast(s, W)
    assert got.first_difference(want) is None, got.first_difference(want)


def test_store_subset_with_txn_index(gpu_device):
    # a store that only receives the txns intersecting its keys keeps global coordinates
    ks, W = 3000, 64
    s = generate_stream(15000, 4, ks, 0.99, 0.5, seed=32)
    lo, hi = 1000, 2000
    sub = s.restrict_keys(lo, hi, drop_empty=True)
    assert sub.n < s.n
    with CommandStore(device=0, key_lo=lo, key_hi=hi, window=W) as st:
        got = st.calculate_deps_batch(sub)
    want = O.deps_fast(s.restrict_keys(lo, hi), W)
    for local, g in enumerate(sub.txn_index[:4000]):
        g = int(g)
        a = got.key_deps(local)
        b = want.key_deps(g)
        for x, y in zip(a, b):
            assert np.array_equal(x, y), (local, g)


def test_exchange_merge_single_rank(gpu_device):
    ks, W = 4000, 256
    s = generate_stream(30000, 8, ks, 0.99, 0.5, seed=33)
    sub = s.restrict_keys(0, ks, drop_empty=True)
    with CommandStore(device=0, key_lo=0, key_hi=ks, window=W, profile=True) as st:
        st.comm_init(1, 0, CommandStore.comm_unique_id())
        st.upload(sub)
        st.compute()
        st.exchange_merge(s.n)
        got = st.download()
        xms, mms = st.shard_timing()
    want = O.deps_fast(s, W)
    assert got.first_difference(want) is None, got.first_difference(want)
    assert mms > 0


def test_merge_rejects_overlapping_parts(gpu_device):
    ks, W = 1000, 32
    s = generate_stream(2000, 4, ks, 0.0, 0.5, seed=34)
    with CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as a, \
            CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as b, \
            CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as m:
        for st in (a, b):
            st.upload(s)
            st.compute()
        with pytest.raises(IllegalArgumentException):
            m.merge([a, b])


def test_merge_of_more_than_64_stores(gpu_device):
    # 80 key-disjoint stores: past the merge kernel's 64 lanes the general union folds 64 parts per pass
    ks, W = 4000, 64
    s = generate_stream(6000, 6, ks, 0.99, 0.5, seed=37)
    stores = []
    try:
        for lo, hi in even_split(ks, 80):
            st = CommandStore(device=0, key_lo=lo, key_hi=hi, window=W)
            st.upload(s.restrict_keys(lo, hi))
            st.compute()
            stores.append(st)
        with CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as merger:
            merger.merge(stores, txn_lo=0)
            got = merger.download()
    finally:
        for st in stores:
            st.close()
    want = O.deps_fast(s, W)
    assert got.first_difference(want) is None, got.first_difference(want)
