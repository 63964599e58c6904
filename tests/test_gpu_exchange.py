"""Config 4 on one GPU: the multi-rank exchange with G = 2, 4, 8 simulated ranks.

Every rank is a CommandStore over its contiguous block of the 8*G EvenSplit stores
(local/ShardDistributor.java:46-157) holding the partial deps of the txns intersecting it
(CommandStores.mapReduce fan-out, local/CommandStores.java:575-592).  accord_deps_exchange_local
runs the product's exchange plan (expanded offsets, the G x G count table, receive layouts, segment
lists) and its on-device union (PreAccept.reduce, messages/PreAccept.java:140-156) for all G ranks,
with the RCCL transport replaced by device copies of the same segment lists.  Afterwards rank r
holds the node-level deps of txns [r*n/G, (r+1)*n/G), which must equal the single-store oracle
deps of those txns byte for byte."""
import numpy as np
import pytest

from accord_amd import CommandStore, IllegalStateException, generate_stream
import oracle_lib as O

pytestmark = pytest.mark.gpu


def rank_blocks(keyspace, G):
    S = 8 * G
    return [((8 * r) * keyspace // S, (8 * r + 8) * keyspace // S) for r in range(G)]


def run_exchange(s, keyspace, G, W, subset):
    b = O.store_bounds(keyspace, 8 * G)
    stores = []
    try:
        for r, (lo, hi) in enumerate(rank_blocks(keyspace, G)):
            # rank r hosts the 8 EvenSplit CommandStores [8r, 8r + 8): ranges sliced at their bounds
            st = CommandStore(device=0, key_lo=lo, key_hi=hi, window=W, profile=True, store_bounds=b[8 * r:8 * r + 9])
            st.upload(s.restrict_keys(lo, hi, drop_empty=subset))
            st.compute()
            stores.append(st)
        CommandStore.exchange_local(stores, s.n)
        out = [st.download() for st in stores]
        timing = [st.shard_timing() for st in stores]
    finally:
        for st in stores:
            st.close()
    return out, timing


def check_ranks(out, want, n, G):
    for r, got in enumerate(out):
        a, b = r * n // G, (r + 1) * n // G
        assert got.n == b - a
        exp = want.txns(a, b)
        diff = got.first_difference(exp)
        assert diff is None, (r, diff)


@pytest.mark.parametrize("G", [2, 4, 8])
def test_exchange_key_txns_store_subsets(gpu_device, G):
    # key txns: every rank holds only the txns intersecting its key block (txn_index subsets), so the
    # plan expands its offsets onto every global position
    ks, W, n = 20000, 256, 60000
    s = generate_stream(n, 8, ks, 0.99, 0.5, seed=40 + G)
    out, timing = run_exchange(s, ks, G, W, subset=True)
    check_ranks(out, O.deps_fast(s, W), n, G)
    assert all(m > 0 for _, m in timing)


@pytest.mark.parametrize("G", [2, 4, 8])
def test_exchange_with_range_txns(gpu_device, G):
    # range txns span rank blocks: every rank's stores register and query their slices of the ranges,
    # the parts reach the owner as store-sliced RangeDeps and it unions them with
    # RelationMultiMap.linearUnion (general union path) -- equal to the 8G-store oracle
    ks, W, n = 8000, 128, 16000
    s = generate_stream(n, 6, ks, 0.99, 0.5, seed=50 + G, range_frac=0.15, range_len_max=1500)
    out, _ = run_exchange(s, ks, G, W, subset=False)
    check_ranks(out, O.deps_stores(s, W, O.store_bounds(ks, 8 * G)), n, G)


def test_exchange_uneven_homes_and_empty_ranks(gpu_device):
    # n not divisible by G, and a keyspace where high ranks see few txns: some send nothing
    ks, W, n, G = 64, 32, 2003, 8
    s = generate_stream(n, 2, ks, 1.2, 0.5, seed=61)
    out, _ = run_exchange(s, ks, G, W, subset=True)
    check_ranks(out, O.deps_fast(s, W), n, G)


def test_exchange_repeated_reuses_buffers(gpu_device):
    # a second exchange of the same stores (grown receive buffers kept) gives the same result
    ks, W, n, G = 5000, 64, 12000, 4
    s = generate_stream(n, 4, ks, 0.99, 0.5, seed=62)
    want = O.deps_fast(s, W)
    stores = []
    try:
        for lo, hi in rank_blocks(ks, G):
            st = CommandStore(device=0, key_lo=lo, key_hi=hi, window=W)
            st.upload(s.restrict_keys(lo, hi, drop_empty=True))
            stores.append(st)
        for _ in range(2):
            for st in stores:
                st.compute()
            CommandStore.exchange_local(stores, n)
            check_ranks([st.download() for st in stores], want, n, G)
    finally:
        for st in stores:
            st.close()


def test_exchange_rejects_uncomputed_rank(gpu_device):
    ks, W, n, G = 2000, 64, 3000, 2
    s = generate_stream(n, 4, ks, 0.99, 0.5, seed=63)
    stores = []
    try:
        for r, (lo, hi) in enumerate(rank_blocks(ks, G)):
            st = CommandStore(device=0, key_lo=lo, key_hi=hi, window=W)
            st.upload(s.restrict_keys(lo, hi, drop_empty=True))
            if r == 0:
                st.compute()
            stores.append(st)
        with pytest.raises(IllegalStateException):
            CommandStore.exchange_local(stores, n)
    finally:
        for st in stores:
            st.close()
