"""Txns beyond the per-wave kernels' bounds go to the big-txn kernel (keydeps_big_kernel): more keys
than a wave has lanes (k > 64) and more distinct deps older than the near span than the general
kernel's far list holds (> 256).  The reference has neither limit (Keys and CommandsForKey are
unbounded), so these are byte-compared with the oracle like every other txn."""
import numpy as np
import pytest

from accord_amd import CommandStore, Stream, generate_stream
import oracle_lib as O

pytestmark = pytest.mark.gpu


def widen(s: Stream, rng, every: int, kmin: int, kmax: int, keyspace: int) -> Stream:
    """Every `every`-th key txn gets kmin..kmax random keys (sorted unique) instead of its own."""
    ko, kk = [0], []
    for t in range(s.n):
        keys = s.key_ord[s.key_off[t]:s.key_off[t + 1]]
        if len(keys) and t % every == 0:
            keys = np.sort(rng.choice(keyspace, size=int(rng.integers(kmin, kmax + 1)), replace=False))
        kk.extend(int(x) for x in keys)
        ko.append(len(kk))
    return Stream(s.msb, s.lsb, s.node, np.asarray(ko, np.uint32), np.asarray(kk, np.uint32),
                  s.rng_off, s.rng_start, s.rng_end)


def run(s, W, ks):
    with CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as st:
        return st.calculate_deps_batch(s)


@pytest.mark.parametrize("n,k,ks,z,W,every,kmin,kmax,seed", [
    (3000, 4, 2000, 0.99, 64, 10, 65, 300, 1),      # many keys: fast -> general -> big
    (2000, 8, 5000, 0.0, 256, 3, 60, 70, 2),        # around the 64-lane boundary
    (1500, 4, 800, 0.99, 1024, 7, 100, 800, 3),     # general-only mode (W > 512)
])
def test_many_keys(gpu_device, n, k, ks, z, W, every, kmin, kmax, seed):
    rng = np.random.default_rng(seed)
    s = widen(generate_stream(n, k, ks, z, 0.5, seed=seed), rng, every, kmin, kmax, ks)
    want = O.deps_fast(s, W)
    got = run(s, W, ks)
    assert got.first_difference(want) is None
    if n <= 2000:
        assert got.first_difference(O.deps_literal(s, W)) is None


def test_many_far_deps(gpu_device):
    # few keys, 1% writes: a Write's slice holds every Read since the last Write before the window,
    # most of them more than the near span back -> more far deps than the general kernel's list
    s = generate_stream(20000, 2, 4, 0.0, 0.01, seed=4)
    W = 16
    got = run(s, W, 4)
    assert got.first_difference(O.deps_fast(s, W)) is None


def test_many_keys_accept(gpu_device):
    rng = np.random.default_rng(5)
    s = widen(generate_stream(1500, 4, 1000, 0.99, 0.5, seed=5), rng, 5, 70, 200, 1000)
    # executeAt a few txns past the TxnId (Accept.calculatePartialDeps)
    ahead = np.minimum(np.arange(s.n) + rng.integers(0, 20, size=s.n), s.n - 1)
    s.exec_msb = s.msb[ahead].copy(); s.exec_lsb = s.lsb[ahead].copy(); s.exec_node = s.node[ahead].copy()
    got = run(s, 32, 1000)
    assert got.first_difference(O.deps_fast(s, 32)) is None
