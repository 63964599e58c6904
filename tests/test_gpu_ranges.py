"""GPU parity for range transactions (RangeDeps of every txn + KeyDeps of range txns) and the
hand-derived KATs, bit-exact against the oracle through the C ABI."""
import numpy as np
import pytest

from accord_amd import CommandStore, IllegalArgumentException, generate_stream, keydeps_str, rangedeps_str
import oracle_lib as O
from kat_util import kat_stream, load_kats, max_key

pytestmark = pytest.mark.gpu

KATS = load_kats()


def run_gpu(s, window, keyspace):
    with CommandStore(device=0, key_lo=0, key_hi=keyspace, window=window) as st:
        return st.calculate_deps_batch(s)


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_kats_on_gpu(gpu_device, kat):
    s = kat_stream(kat)
    ks = max_key(s) + 1
    if "expect_error" in kat:
        with pytest.raises(IllegalArgumentException):
            run_gpu(s, kat["window"], ks)
        return
    d = run_gpu(s, kat["window"], ks)
    assert [keydeps_str(*d.key_deps(i), s) for i in range(s.n)] == kat["expect_key"]
    if "expect_range" in kat:
        assert [rangedeps_str(*d.range_deps(i), s) for i in range(s.n)] == kat["expect_range"]


@pytest.mark.parametrize("n,k,ks,z,wf,W,seed,rf,rl", [
    (1500, 4, 300, 0.0, 0.5, 16, 6, 0.2, 30),
    (2000, 8, 1000, 0.99, 0.5, 64, 7, 0.2, 100),
    (1000, 3, 60, 0.99, 0.3, 8, 8, 0.5, 10),
    (3000, 8, 2000, 0.99, 0.5, 256, 9, 0.2, 1000),
    (2000, 2, 500, 0.0, 0.5, 0, 10, 0.3, 50),
    (500, 2, 100, 0.0, 0.5, 1000, 11, 0.9, 20),
    (800, 4, 8000, 0.0, 0.9, 64, 12, 0.3, 3000),       # range txns with 2k-6k deps (largest union classes)
])
def test_mixed_vs_literal(gpu_device, n, k, ks, z, wf, W, seed, rf, rl):
    s = generate_stream(n, k, ks, z, wf, range_frac=rf, range_len_max=rl, seed=seed)
    got = run_gpu(s, W, ks)
    want = O.deps_literal(s, W)
    assert got.first_difference(want) is None, got.first_difference(want)


def test_config3_full(gpu_device):
    s = generate_stream(1 << 20, 8, 100_000, 0.99, 0.5, range_frac=0.2, range_len_max=1000, seed=3)
    got = run_gpu(s, 256, 100_000)
    want = O.deps_fast(s, 256)
    assert got.first_difference(want) is None, got.first_difference(want)
    assert int(got.rd_val_off[-1]) > 0


def test_range_batch_rejects_overlapping_ranges(gpu_device):
    s = generate_stream(100, 2, 100, 0.0, 0.5, range_frac=0.5, range_len_max=10, seed=4)
    i = int(np.nonzero(s.domains())[0][0])
    a = int(s.rng_off[i])
    st = s.rng_start.copy()
    en = s.rng_end.copy()
    st[a], en[a] = 5, 5          # empty range (start >= end)
    from accord_amd import Stream
    bad = Stream(s.msb, s.lsb, s.node, s.key_off, s.key_ord, s.rng_off, st, en)
    with pytest.raises(IllegalArgumentException):
        run_gpu(bad, 8, 100)


@pytest.mark.parametrize("seed,kinds_p", [
    (14, [0.35, 0.35, 0.1, 0.1, 0.1]),     # every kind: range Writes must still skip SyncPoints/EphemeralReads
    (15, [0.0, 1.0, 0.0, 0.0, 0.0]),       # Writes only: every entry witnessed by every range txn
    (16, [0.5, 0.5, 0.0, 0.0, 0.0]),       # R/W: range Writes witness all, range Reads only Writes
    (17, [0.3, 0.3, 0.0, 0.4, 0.0]),       # SyncPoints in the histories
])
def test_mixed_kinds_vs_literal(gpu_device, seed, kinds_p):
    from accord_amd import Stream
    s = generate_stream(2500, 4, 400, 0.99, 0.5, range_frac=0.25, range_len_max=120, seed=seed)
    rng = np.random.default_rng(seed)
    kinds = rng.choice([0, 1, 2, 3, 4], size=s.n, p=kinds_p).astype(np.uint64)
    lsb = (s.lsb & ~np.uint64(0xE)) | (kinds << np.uint64(1))
    s2 = Stream(s.msb, lsb, s.node, s.key_off, s.key_ord, s.rng_off, s.rng_start, s.rng_end)
    got = run_gpu(s2, 64, 400)
    want = O.deps_literal(s2, 64)
    assert got.first_difference(want) is None, got.first_difference(want)


@pytest.mark.parametrize("env", [{"ACCORD_RT_REUSE": "1"}, {"ACCORD_RT_REUSE": "0"}],
                         ids=["hit-reuse", "hit-rescan"])
def test_range_pass_variants_vs_literal(gpu_device, monkeypatch, env):
    """The RangeDeps fill with the count pass's hits reused or rescanned (the rescan is also the
    path of a txn whose hits overflow the count pass's slots), both equal to the literal oracle
    (knob read per compute)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    for seed, W, rl in ((21, 64, 100), (22, 256, 1000), (23, 16, 30)):
        s = generate_stream(2500, 8, 1500, 0.99, 0.5, range_frac=0.25, range_len_max=rl, seed=seed)
        got = run_gpu(s, W, 1500)
        want = O.deps_literal(s, W)
        assert got.first_difference(want) is None, (env, seed, got.first_difference(want))
