"""GPU parity of Accept batches (Accept.calculatePartialDeps, messages/Accept.java:113-117):
startedBefore = executeAt and p1 = txnId (messages/PreAccept.java:253-259), bit-exact against the
CPU oracle through the C ABI.  The Accept KATs themselves run in test_gpu_ranges.test_kats_on_gpu."""
import dataclasses

import pytest

from accord_amd import CommandStore, IllegalArgumentException, IllegalStateException, generate_stream
import oracle_lib as O

pytestmark = pytest.mark.gpu


def run_gpu(s, window, keyspace):
    with CommandStore(device=0, key_lo=0, key_hi=keyspace, window=window) as st:
        return st.calculate_deps_batch(s)


def check(s, window, keyspace, literal=False):
    got = run_gpu(s, window, keyspace)
    want = O.deps_literal(s, window) if literal else O.deps_fast(s, window)
    assert got.first_difference(want) is None, got.first_difference(want)
    return got


@pytest.mark.parametrize("n,k,ks,z,wf,W,seed,frac,delay", [
    (1, 1, 10, 0.0, 0.5, 0, 1, 1.0, 4),
    (2000, 4, 200, 0.0, 0.5, 16, 3, 0.5, 16),
    (3000, 8, 1000, 0.99, 0.5, 64, 4, 1.0, 64),
    (2000, 3, 50, 0.99, 0.1, 8, 5, 1.0, 300),
    (1500, 2, 30, 0.0, 0.9, 0, 6, 0.3, 8),
    (3000, 12, 500, 0.99, 0.5, 64, 10, 1.0, 32),   # > 8 keys: general kernel
    (5000, 1, 3, 0.0, 1.0, 32, 9, 1.0, 100),       # all writes on 3 keys
])
def test_accept_keys_vs_literal(gpu_device, n, k, ks, z, wf, W, seed, frac, delay):
    s = generate_stream(n, k, ks, z, wf, seed=seed).accept(frac=frac, max_delay=delay, seed=seed)
    check(s, W, ks, literal=True)


@pytest.mark.parametrize("W,delay", [(0, 64), (64, 1000), (256, 256), (1024, 64), (3000, 500)])
def test_accept_windows(gpu_device, W, delay):
    s = generate_stream(20000, 8, 3000, 0.99, 0.5, seed=11).accept(frac=0.7, max_delay=delay, seed=5)
    check(s, W, 3000)


@pytest.mark.parametrize("n,k,ks,z,wf,W,seed,rf,rl,delay", [
    (1500, 4, 300, 0.0, 0.5, 16, 6, 0.2, 30, 16),
    (2000, 8, 1000, 0.99, 0.5, 64, 7, 0.2, 100, 200),
    (1000, 3, 60, 0.99, 0.3, 8, 8, 0.5, 10, 50),
    (3000, 8, 2000, 0.99, 0.5, 256, 9, 0.2, 1000, 64),
])
def test_accept_mixed_ranges_vs_literal(gpu_device, n, k, ks, z, wf, W, seed, rf, rl, delay):
    s = generate_stream(n, k, ks, z, wf, range_frac=rf, range_len_max=rl, seed=seed)
    check(s.accept(frac=0.8, max_delay=delay, seed=seed), W, ks, literal=True)


def test_accept_block_boundary_bound(gpu_device):
    # n a multiple of the range-key checkpoint block (4096): executeAt past the last txn
    s = generate_stream(8192, 4, 500, 0.99, 0.5, range_frac=0.2, range_len_max=100, seed=41)
    check(s.accept(frac=1.0, max_delay=100, seed=2), 64, 500)


def test_accept_config2_full(gpu_device):
    s = generate_stream(1 << 20, 8, 100_000, 0.99, 0.5, seed=2).accept(frac=0.5, max_delay=32, seed=2)
    check(s, 256, 100_000)


def test_accept_config3_full(gpu_device):
    s = generate_stream(1 << 20, 8, 100_000, 0.99, 0.5, range_frac=0.2, range_len_max=1000, seed=3)
    check(s.accept(frac=0.5, max_delay=32, seed=3), 256, 100_000)


def test_accept_store_subset(gpu_device):
    ks, W = 3000, 64
    s = generate_stream(15000, 4, ks, 0.99, 0.5, seed=32).accept(frac=0.6, max_delay=40, seed=7)
    lo, hi = 1000, 2000
    sub = s.restrict_keys(lo, hi, drop_empty=True)
    with CommandStore(device=0, key_lo=lo, key_hi=hi, window=W) as st:
        got = st.calculate_deps_batch(sub)
    want = O.deps_fast(s.restrict_keys(lo, hi), W)
    for local, g in enumerate(sub.txn_index.tolist()):
        a, b = got.key_deps(local), want.key_deps(g)
        assert all((x == y).all() and x.shape == y.shape for x, y in zip(a, b)), (local, g)


def test_accept_executeAt_before_txnId_rejected(gpu_device):
    s = generate_stream(100, 2, 50, 0.0, 0.5, seed=3).accept(frac=1.0, max_delay=4, seed=1)
    el = s.exec_lsb.copy()
    el[37] = s.lsb[37] - (1 << 16)
    with pytest.raises(IllegalArgumentException):
        run_gpu(dataclasses.replace(s, exec_lsb=el), 8, 50)


def test_accept_waiting_on_rejected(gpu_device):
    s = generate_stream(1000, 2, 50, 0.0, 0.5, seed=3).accept(frac=1.0, max_delay=4, seed=1)
    with CommandStore(device=0, key_lo=0, key_hi=50, window=8) as st:
        st.upload(s)
        st.compute()
        with pytest.raises(IllegalStateException):
            st.waiting_on_compute()
