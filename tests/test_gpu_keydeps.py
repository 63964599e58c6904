"""GPU parity of the KeyDeps path against the CPU oracle (bit-exact), through the C ABI."""
import numpy as np
import pytest

from accord_amd import CommandStore, IllegalArgumentException, Stream, generate_stream
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


@pytest.mark.parametrize("n,k,ks,z,wf,W,seed", [
    (1, 1, 10, 0.0, 0.5, 0, 1),
    (64, 2, 8, 0.0, 0.5, 0, 2),
    (2000, 4, 200, 0.0, 0.5, 16, 3),
    (3000, 8, 1000, 0.99, 0.5, 64, 4),
    (2000, 3, 50, 0.99, 0.1, 8, 5),
    (1500, 2, 30, 0.0, 0.9, 0, 6),
    (4000, 8, 5000, 0.99, 0.5, 256, 7),
    (5000, 1, 3, 0.0, 0.0, 32, 8),      # all reads: deps empty
    (5000, 1, 3, 0.0, 1.0, 32, 9),      # all writes: long chains
    (3000, 12, 500, 0.99, 0.5, 64, 10),  # more than 8 keys per txn (general kernel)
    (1500, 40, 2000, 0.0, 0.5, 128, 14),
])
def test_small_vs_literal(gpu_device, n, k, ks, z, wf, W, seed):
    s = generate_stream(n, k, ks, z, wf, seed=seed)
    check(s, W, ks, literal=True)


@pytest.mark.parametrize("W", [0, 1, 63, 64, 255, 1024, 3000])
def test_windows(gpu_device, W):
    s = generate_stream(20000, 8, 3000, 0.99, 0.5, seed=11)
    check(s, W, 3000)


def test_far_history(gpu_device):
    # a cold keyspace with rare writes: many deps fall outside the near bitmap span
    s = generate_stream(30000, 2, 50000, 0.0, 0.02, seed=12)
    check(s, 16, 50000)


def test_config1_full(gpu_device):
    s = generate_stream(65536, 4, 100_000, 0.0, 0.5, seed=1)
    check(s, 256, 100_000)


def test_config2_full(gpu_device):
    s = generate_stream(1 << 20, 8, 100_000, 0.99, 0.5, seed=2)
    got = check(s, 256, 100_000)
    t = got.totals()
    assert t["body"] > 10**8 // 2


def test_kinds_ephemeral_and_syncpoints(gpu_device):
    s = generate_stream(3000, 3, 40, 0.0, 0.5, seed=13)
    rng = np.random.default_rng(5)
    kinds = rng.choice([0, 1, 2, 3, 4], size=s.n, p=[0.35, 0.35, 0.1, 0.1, 0.1]).astype(np.uint64)
    lsb = (s.lsb & ~np.uint64(0xE)) | (kinds << np.uint64(1))
    s2 = Stream(s.msb, lsb, s.node, s.key_off, s.key_ord, s.rng_off, s.rng_start, s.rng_end)
    check(s2, 32, 40, literal=True)


def test_unsorted_rejected(gpu_device):
    s = generate_stream(100, 2, 10, seed=3)
    msb = s.msb.copy()
    msb[50], msb[51] = msb[51], msb[50]
    lsb = s.lsb.copy()
    lsb[50], lsb[51] = lsb[51], lsb[50]
    bad = Stream(msb, lsb, s.node, s.key_off, s.key_ord, s.rng_off, s.rng_start, s.rng_end)
    with pytest.raises(IllegalArgumentException):
        run_gpu(bad, 8, 10)


def test_local_only_rejected(gpu_device):
    s = generate_stream(100, 2, 10, seed=3)
    lsb = s.lsb.copy()
    lsb[7] = (lsb[7] & ~np.uint64(0xE)) | np.uint64(5 << 1)
    bad = Stream(s.msb, lsb, s.node, s.key_off, s.key_ord, s.rng_off, s.rng_start, s.rng_end)
    with pytest.raises(IllegalArgumentException):
        run_gpu(bad, 8, 10)


def test_keys_outside_store_rejected(gpu_device):
    s = generate_stream(100, 2, 1000, seed=3)
    with pytest.raises(IllegalArgumentException):
        run_gpu(s, 8, 10)


def test_device_resident_repeat(gpu_device):
    s = generate_stream(50000, 8, 10000, 0.99, 0.5, seed=21)
    with CommandStore(device=0, key_lo=0, key_hi=10000, window=256, profile=True) as st:
        st.upload(s)
        st.compute()
        a = st.download()
        st.compute()
        b = st.download()
        t = st.timing()
    assert a.equals(b)
    assert t.total_ms > 0
    assert a.first_difference(O.deps_fast(s, 256)) is None


def test_speculative_fill_grow_shrink_and_errors(gpu_device):
    # one store over batches of changing size: after the first, the fill runs speculatively into the
    # arrays an earlier batch sized (store.cpp, launch_spec_check) -- a larger batch aborts it and is
    # filled again into grown arrays; an invalid batch fails as before and leaves the store usable
    ks, W = 3000, 256
    with CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as st:
        for n, k, z, seed in [(500, 4, 0.0, 21), (2000, 4, 0.0, 22), (60000, 8, 0.99, 23), (100, 2, 0.0, 24),
                              (60000, 8, 0.99, 25), (30000, 12, 0.99, 26)]:
            s = generate_stream(n, k, ks, z, 0.5, seed=seed)
            got = st.calculate_deps_batch(s)
            assert got.first_difference(O.deps_fast(s, W)) is None, (n, seed)
            if n == 100:
                bad = generate_stream(200, 2, ks * 2, seed=3)      # keys outside the store
                with pytest.raises(IllegalArgumentException):
                    st.calculate_deps_batch(bad)


def test_profile_switch(gpu_device):
    # accord_store_set_profile: a store created without events gains them, computes stay exact either way
    s = generate_stream(3000, 4, 500, 0.99, 0.5, seed=41)
    want = O.deps_fast(s, 64)
    with CommandStore(device=0, key_lo=0, key_hi=500, window=64) as st:
        assert st.calculate_deps_batch(s).first_difference(want) is None
        st.set_profile(True)
        assert st.calculate_deps_batch(s).first_difference(want) is None
        assert st.timing().total_ms > 0
        st.set_profile(False)
        assert st.calculate_deps_batch(s).first_difference(want) is None
