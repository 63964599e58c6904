"""Multi-store union (K6) on one GPU and the RCCL exchange path with a 1-rank communicator.

The stores of a node partition the keyspace (EvenSplit, local/ShardDistributor.java:46-157); the
union of their per-store PartialDeps (PreAccept.reduce, messages/PreAccept.java:140-156) must equal
the node-level deps of the S-store oracle (oracle_lib.deps_stores): for key txns that is the deps of
a single store over the whole keyspace; range commands and queries are sliced to each store's range
(impl/InMemoryCommandStore.java:757-760), so spanning ranges appear once per store slice."""
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
    # range txns span store blocks: every store registers and queries its Minimal slice of their
    # ranges (impl/InMemoryCommandStore.java:757-760, 886), so a spanning range reaches the union as
    # one RangeDeps entry per store slice (primitives/RangeDeps.java:462-465) -- the S-store oracle
    ks, W = 5000, 64
    s = generate_stream(12000, 6, ks, 0.99, 0.5, seed=35, range_frac=0.1, range_len_max=rl)
    b = O.store_bounds(ks, nstores)
    stores = []
    try:
        for j, (lo, hi) in enumerate(even_split(ks, nstores)):
            st = CommandStore(device=0, key_lo=lo, key_hi=hi, window=W, store_bounds=b[j:j + 2])
            st.upload(s.restrict_keys(lo, hi))
            st.compute()
            stores.append(st)
        with CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as merger:
            merger.merge(stores, txn_lo=0)
            got = merger.download()
    finally:
        for st in stores:
            st.close()
    want = O.deps_stores(s, W, b)
    assert got.first_difference(want) is None, got.first_difference(want)
    # a spanning range really is split: the single-store result differs once ranges cross blocks
    if rl > ks // nstores:
        assert got.first_difference(O.deps_fast(s, W)) is not None


@pytest.mark.parametrize("nstores,rl", [(2, 300), (8, 2000)])
def test_one_handle_hosting_many_stores(gpu_device, nstores, rl):
    # one handle hosting the node's S stores slices at their internal bounds: == the S-store oracle
    # (literal restatement at this size) == S handles of one store each unioned
    ks, W = 3000, 64
    s = generate_stream(3000, 6, ks, 0.99, 0.5, seed=36, range_frac=0.2, range_len_max=rl)
    b = O.store_bounds(ks, nstores)
    with CommandStore(device=0, key_lo=0, key_hi=ks, window=W, store_bounds=b) as st:
        got = st.calculate_deps_batch(s)
    want = O.deps_stores(s, W, b, literal=True)
    assert got.first_difference(want) is None, got.first_difference(want)


def test_handle_drops_pieces_outside_its_stores(gpu_device):
    # a handle hosting stores [1000, 2000) of a 3-store node: range pieces below / above are not its
    # own (another store registers them); keys outside the handle are the caller's error as before
    ks, W = 3000, 32
    s = generate_stream(2000, 4, ks, 0.99, 0.5, seed=38, range_frac=0.3, range_len_max=2500)
    b = [0, 1000, 2000, O.KEY_END]
    with CommandStore(device=0, key_lo=1000, key_hi=2000, window=W, store_bounds=b[1:3]) as st:
        got = st.calculate_deps_batch(s.restrict_keys(1000, 2000))
    want = O.deps_stores(s, W, b[1:3])
    assert got.first_difference(want) is None, got.first_difference(want)
    for i in range(s.n):
        rs, re, _, _ = got.range_deps(i)
        assert np.all(rs >= 999) and np.all(re <= 1999)


def test_store_bounds_rejected(gpu_device):
    with pytest.raises(IllegalArgumentException):
        CommandStore(device=0, key_lo=0, key_hi=100, window=8, store_bounds=[0, 50, 50])
    with pytest.raises(IllegalArgumentException):
        CommandStore(device=0, key_lo=0, key_hi=100, window=8, store_bounds=[10, 100])


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
