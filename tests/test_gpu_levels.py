"""Execution levelling by stripes (csrc/levels.hip) against the oracle's levels
(or_waiting_on over the downloaded deps): stripe lengths forced small so that many stripes, their
sources and the relaxation sweeps are exercised; the serial resolver alone (ACCORD_LV_MODE=serial)
and the fallback to it when the sweep bound is too small to reach the fixpoint (ACCORD_LV_RELAX=1)."""
import numpy as np
import pytest

from accord_amd import CommandStore, generate_stream
import oracle_lib as O
from test_oracle_stream import with_random_kinds

pytestmark = pytest.mark.gpu


def _levels(s, ks, W):
    with CommandStore(device=0, key_lo=0, key_hi=ks, window=W) as st:
        st.upload(s)
        st.compute()
        wo = st.waiting_on()
        wo.stripe, wo.fallback = st.waiting_on_levelling()
        d = st.download()
    level, _, _ = O.waiting_on(d)
    return wo, level


def _assert_levels(wo, level):
    bad = np.nonzero(wo.level != level)[0]
    assert bad.size == 0, (bad[:5], wo.level[bad[:5]], level[bad[:5]])
    assert wo.max_level == int(level.max(initial=0))


CASES = [
    # n, k, keyspace, zipf, write_frac, window, seed, range_frac, range_len, kinds, stripe
    (40000, 4, 2000, 0.99, 0.9, 256, 71, 0.0, 0, False, 1024),     # config 5 shape, 40 stripes
    (40000, 4, 2000, 0.99, 0.9, 256, 72, 0.0, 0, False, 4096),
    (30000, 8, 5000, 0.99, 0.5, 64, 73, 0.0, 0, False, 1024),
    (20000, 4, 500, 0.0, 0.5, 32, 74, 0.2, 50, False, 1024),        # range txns: long predecessor lists
    (20000, 4, 300, 0.99, 0.7, 16, 75, 0.0, 0, True, 1024),         # SyncPoints: full lists (> 4 in a chunk)
    (9000, 1, 1, 0.0, 1.0, 4096, 76, 0.0, 0, False, 1024),          # one key, all writes: level = i
    (60000, 4, 50000, 0.99, 0.9, 256, 77, 0.0, 0, False, 1024),     # cold keys: sources miss old Writes
    (20000, 6, 40, 0.0, 0.3, 2000, 78, 0.0, 0, False, 2048),        # read-heavy
    (1024, 4, 100, 0.99, 0.9, 64, 79, 0.0, 0, False, 1024),         # n == one stripe
    (1025, 4, 100, 0.99, 0.9, 64, 80, 0.0, 0, False, 1024),         # one txn in the second stripe
    (700, 4, 100, 0.99, 0.9, 64, 81, 0.0, 0, False, 1024),          # shorter than a stripe
]


@pytest.mark.parametrize("case", CASES, ids=[f"c{i}" for i in range(len(CASES))])
def test_striped_levels_match_oracle(gpu_device, monkeypatch, case):
    n, k, ks, z, wf, W, seed, rf, rl, kinds, stripe = case
    monkeypatch.setenv("ACCORD_LV_STRIPE", str(stripe))
    s = generate_stream(n, k, ks, z, wf, seed=seed, range_frac=rf, range_len_max=rl)
    if kinds:
        s = with_random_kinds(s, seed)
    wo, level = _levels(s, ks, W)
    _assert_levels(wo, level)
    assert wo.stripe == stripe
    if ks == 1:
        assert np.array_equal(wo.level, np.arange(n, dtype=np.uint32))


@pytest.mark.parametrize("mode", ["serial", "fallback"])
def test_serial_resolver_and_fallback(gpu_device, monkeypatch, mode):
    """The serial resolver on its own, and the striped path with one sweep allowed: the deep chains
    of this stream need more, so the call falls back to the serial resolver -- same levels."""
    if mode == "serial":
        monkeypatch.setenv("ACCORD_LV_MODE", "serial")
    else:
        monkeypatch.setenv("ACCORD_LV_STRIPE", "1024")
        monkeypatch.setenv("ACCORD_LV_RELAX", "1")
    s = generate_stream(30000, 4, 3000, 0.99, 0.9, seed=82)
    wo, level = _levels(s, 3000, 256)
    _assert_levels(wo, level)
    if mode == "fallback":
        assert wo.fallback and wo.stripe == 1024
    else:
        assert wo.stripe == 0 and not wo.fallback
